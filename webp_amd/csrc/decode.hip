// decode.hip -- VP8 decoder reconstruct + loop filter for whole frames on
// gfx950 (replaces reconstructRow / filterRowAt of parseFrame,
// internal/lossy/decode.go:532-560 and decode_frame.go:83-342).
//
// Schedule.  Macroblock (x, y) needs the *unfiltered* reconstruction of
// (x-1, y), (x-1..x+1, y-1) for intra prediction, and its loop filter needs
// (x-1, y), (x, y-1), (x+1, y-1) already filtered (their edge filters write
// 3 pixels into it).  Both dependencies are satisfied by the anti-diagonal
// order t = x + 2y, so one launch per t processes every MB on that diagonal
// of every image in the batch: reconstruct, then filter, in the same wave.
// Unfiltered context travels through two small side buffers (the GPU form of
// the decoder's yuvT / left-sample rotation, decode_frame.go:118-126,190):
//   top[img][mbx]  : bottom row of the MB above   (Y16 U8 V8)
//   left[img][mby] : right column of the MB to the left + its top-left pixels
//
// One 64-lane wave per macroblock.  Luma lanes: block b = lane/4 (raster),
// row r = lane%4, 4 pixels per lane.  Chroma: lanes 0-15 U, 16-31 V.  The MB
// and its prediction border live in LDS with the reference's BPS=32 stride;
// the filter works on a 20x20 (Y) / 12x12 (U, V) LDS tile that includes the
// 4 pixels on the far side of the left and top edges.
#include "wg_common.h"
#include "wg_dsp.h"

namespace {

using namespace wg;

// LDS work-buffer layout (stride WG_BPS).  Origins are 16-byte aligned so
// whole rows move with one 16-byte access.  The Y top-right pixels at
// columns 16..19 land in columns 0..3 of the next row, which nothing else
// uses (the left border is column 15, the V block's left border column 31).
constexpr int LY = 1 * WG_BPS + 16;   // Y origin: row 1, col 16
constexpr int LU = 19 * WG_BPS + 16;  // U origin: row 19, col 16
constexpr int LV = 19 * WG_BPS + 0;   // V origin: row 19, col 0 (left border = col 31 of the row above)
constexpr int WB_SIZE = 27 * WG_BPS;

// Filter tiles: Y 20 rows x 32 (cols -4..15 at bytes 12..31), UV 12 rows x 16 (cols -4..7 at 4..15)
constexpr int FY_STRIDE = 32, FY_X0 = 16;
constexpr int FC_STRIDE = 16, FC_X0 = 8;

constexpr int TOP_BYTES = 32;   // per MB column: Y16 U8 V8
constexpr int LEFT_BYTES = 64;  // per MB row: Ycol16 Ucol8 Vcol8 tlY tlU tlV

// checkMode (decode_frame.go:6-19).  Written as one select chain: the
// early-return form was miscompiled by hipcc (ROCm 7.2, -O3) -- the NoTop
// constant overwrote the register holding `mode` on the mbx>0 && mby>0 path.
__device__ __forceinline__ int check_mode(int mbx, int mby, int mode) {
  const int edge = (mbx == 0) ? ((mby == 0) ? 6 : 5) : ((mby == 0) ? 4 : 0);
  return mode == 0 ? edge : mode;
}

struct DecArgs {
  const wg_mb_info* mb;
  const int16_t* coeffs;
  uint8_t* Y;
  uint8_t* U;
  uint8_t* V;
  uint8_t* top;
  uint8_t* left;
  int filter_type, mbw, mbh;
};

__global__ __launch_bounds__(64) void k_decode_diag(DecArgs a, int t, int x_lo, int count) {
  __shared__ __attribute__((aligned(16))) uint8_t wb[WB_SIZE];
  __shared__ __attribute__((aligned(16))) uint8_t fy[20 * FY_STRIDE];
  __shared__ __attribute__((aligned(16))) uint8_t fu[12 * FC_STRIDE];
  __shared__ __attribute__((aligned(16))) uint8_t fv[12 * FC_STRIDE];

  const int lane = threadIdx.x;
  const int img = blockIdx.x / count;
  const int mbx = x_lo + 2 * (blockIdx.x % count);
  const int mby = (t - mbx) >> 1;
  const int mbw = a.mbw, mbh = a.mbh;
  const int64_t mbi = (int64_t)img * mbw * mbh + (int64_t)mby * mbw + mbx;
  const wg_mb_info info = a.mb[mbi];
  const int16_t* co = a.coeffs + mbi * 384;
  uint8_t* top = a.top + (int64_t)img * mbw * TOP_BYTES;
  uint8_t* left = a.left + ((int64_t)img * mbh + mby) * LEFT_BYTES;
  const int ys = 16 * mbw, uvs = 8 * mbw;
  uint8_t* Yp = a.Y + (int64_t)img * ys * 16 * mbh;
  uint8_t* Up = a.U + (int64_t)img * uvs * 8 * mbh;
  uint8_t* Vp = a.V + (int64_t)img * uvs * 8 * mbh;

  // ---- 1. prediction context (decode_frame.go:93-160) ----
  {
    const uint8_t* tc = top + mbx * TOP_BYTES;
    int v;
    if (lane < 16) {  // Y top row
      v = mby > 0 ? tc[lane] : 127;
      wb[LY - WG_BPS + lane] = v;
    } else if (lane < 20) {  // Y top-right (cols 16..19)
      if (mby == 0) v = 127;
      else if (mbx < mbw - 1) v = tc[TOP_BYTES + lane - 16];
      else v = tc[15];
      wb[LY - WG_BPS + lane] = v;
    } else if (lane < 23) {  // top-left of Y, U, V
      const int pl = lane - 20;
      v = mby == 0 ? 127 : (mbx == 0 ? 129 : left[48 + pl]);
      const int o = pl == 0 ? LY : (pl == 1 ? LU : LV);
      wb[o - WG_BPS - 1] = v;
    } else if (lane >= 24 && lane < 40) {  // U / V top row
      const int pl = (lane - 24) >> 3, i = (lane - 24) & 7;
      v = mby > 0 ? tc[16 + 8 * pl + i] : 127;
      wb[(pl ? LV : LU) - WG_BPS + i] = v;
    } else if (lane >= 40 && lane < 56) {  // Y left column
      const int j = lane - 40;
      wb[LY - 1 + j * WG_BPS] = mbx > 0 ? left[j] : 129;
    } else if (lane >= 56) {  // U left column
      const int j = lane - 56;
      wb[LU - 1 + j * WG_BPS] = mbx > 0 ? left[16 + j] : 129;
    }
    if (lane < 8) wb[LV - 1 + lane * WG_BPS] = mbx > 0 ? left[24 + lane] : 129;
  }
  __syncthreads();
  if (info.is_i4x4 && lane < 12) {  // replicate top-right down to rows 3, 7, 11 (:155-160)
    const int r = 4 * (lane / 4 + 1) - 1, i = lane & 3;
    wb[LY + r * WG_BPS + 16 + i] = wb[LY - WG_BPS + 16 + i];
  }
  __syncthreads();

  // ---- 2. luma prediction + residual ----
  {
    const int blk = lane >> 2, r = lane & 3, bx = blk & 3, by = blk >> 2;
    const int off = LY + (4 * by + r) * WG_BPS + 4 * bx;
    const int code = (info.non_zero_y >> (30 - 2 * blk)) & 3;
    const int16_t* bco = co + blk * 16;
    if (!info.is_i4x4) {
      const int mode = check_mode(mbx, mby, info.imodes[0]);
      const int dc = predsq_dc(mode, wb + LY, 16);
      const uint32_t pred = predsq_row4(mode, wb + LY, 4 * bx, 4 * by + r, dc);
      int res[4];
      dec_residual_row(bco, code, r, res);
      *reinterpret_cast<uint32_t*>(wb + off) =
          pack4(clip8(byte_of(pred, 0) + res[0]), clip8(byte_of(pred, 1) + res[1]),
                clip8(byte_of(pred, 2) + res[2]), clip8(byte_of(pred, 3) + res[3]));
    } else {
      const int my_step = bx + 2 * by;  // in-MB dependency wavefront
      int res[4];
      dec_residual_row(bco, code, r, res);
      const int mode = info.imodes[blk];
      for (int s = 0; s < 10; s++) {
        if (s == my_step) {
          int X, T[8], L[4];
          pred4_ctx(wb, LY + 4 * by * WG_BPS + 4 * bx, X, T, L);
          const uint32_t pred = pred4_row(mode, r, X, T, L);
          *reinterpret_cast<uint32_t*>(wb + off) =
              pack4(clip8(byte_of(pred, 0) + res[0]), clip8(byte_of(pred, 1) + res[1]),
                    clip8(byte_of(pred, 2) + res[2]), clip8(byte_of(pred, 3) + res[3]));
        }
        __syncthreads();
      }
    }
  }
  // ---- 3. chroma prediction + residual (doUVTransform :47-68) ----
  if (lane < 32) {
    const int pl = lane >> 4, cblk = (lane >> 2) & 3, r = lane & 3;
    const int cbx = cblk & 1, cby = cblk >> 1;
    const int base = pl ? LV : LU;
    const int mode = check_mode(mbx, mby, info.uv_mode);
    const int dc = predsq_dc(mode, wb + base, 8);
    const uint32_t pred = predsq_row4(mode, wb + base, 4 * cbx, 4 * cby + r, dc);
    const uint32_t bits = info.non_zero_uv >> (8 * pl);
    const int16_t* bco = co + (16 + 4 * pl + cblk) * 16;
    int res[4] = {0, 0, 0, 0};
    if (bits & 0xff) {
      if (bits & 0xaa) dec_residual_row(bco, 3, r, res);
      else if (bco[0] != 0) dec_residual_row(bco, 1, r, res);
    }
    *reinterpret_cast<uint32_t*>(wb + base + (4 * cby + r) * WG_BPS + 4 * cbx) =
        pack4(clip8(byte_of(pred, 0) + res[0]), clip8(byte_of(pred, 1) + res[1]),
              clip8(byte_of(pred, 2) + res[2]), clip8(byte_of(pred, 3) + res[3]));
  }
  __syncthreads();

  // ---- 4. unfiltered context for the neighbours (:190-194 and the rotation :118-126) ----
  if (mby < mbh - 1) {
    uint8_t* tc = top + mbx * TOP_BYTES;
    if (lane == 32) *reinterpret_cast<uint4*>(tc) = *reinterpret_cast<const uint4*>(wb + LY + 15 * WG_BPS);
    if (lane == 33) *reinterpret_cast<uint2*>(tc + 16) = *reinterpret_cast<const uint2*>(wb + LU + 7 * WG_BPS);
    if (lane == 34) *reinterpret_cast<uint2*>(tc + 24) = *reinterpret_cast<const uint2*>(wb + LV + 7 * WG_BPS);
  }
  if (mbx < mbw - 1) {
    if (lane >= 40 && lane < 56) left[lane - 40] = wb[LY + (lane - 40) * WG_BPS + 15];
    if (lane >= 56) left[16 + lane - 56] = wb[LU + (lane - 56) * WG_BPS + 7];
    if (lane < 8) left[24 + lane] = wb[LV + lane * WG_BPS + 7];
    if (lane == 8) left[48] = wb[LY - WG_BPS + 15];
    if (lane == 9) left[49] = wb[LU - WG_BPS + 7];
    if (lane == 10) left[50] = wb[LV - WG_BPS + 7];
  }

  const bool do_filter = a.filter_type > 0 && info.f_limit > 0;
  if (!do_filter) {
    if (lane < 16)
      *reinterpret_cast<uint4*>(Yp + (int64_t)(16 * mby + lane) * ys + 16 * mbx) =
          *reinterpret_cast<const uint4*>(wb + LY + lane * WG_BPS);
    else if (lane < 24)
      *reinterpret_cast<uint2*>(Up + (int64_t)(8 * mby + lane - 16) * uvs + 8 * mbx) =
          *reinterpret_cast<const uint2*>(wb + LU + (lane - 16) * WG_BPS);
    else if (lane < 32)
      *reinterpret_cast<uint2*>(Vp + (int64_t)(8 * mby + lane - 24) * uvs + 8 * mbx) =
          *reinterpret_cast<const uint2*>(wb + LV + (lane - 24) * WG_BPS);
    return;
  }

  // ---- 5. loop filter (doFilter :293-342) on the LDS tiles ----
  const bool luma_only = a.filter_type == 1;
  // 5a. load tiles: MB from wb, left 4 columns and top 4 rows from the (already filtered) frame
  if (lane < 16) {
    *reinterpret_cast<uint4*>(fy + (lane + 4) * FY_STRIDE + FY_X0) =
        *reinterpret_cast<const uint4*>(wb + LY + lane * WG_BPS);
    if (mbx > 0)
      *reinterpret_cast<uint32_t*>(fy + (lane + 4) * FY_STRIDE + FY_X0 - 4) =
          *reinterpret_cast<const uint32_t*>(Yp + (int64_t)(16 * mby + lane) * ys + 16 * mbx - 4);
  } else if (lane < 20) {
    if (mby > 0)
      *reinterpret_cast<uint4*>(fy + (lane - 16) * FY_STRIDE + FY_X0) =
          *reinterpret_cast<const uint4*>(Yp + (int64_t)(16 * mby - 4 + lane - 16) * ys + 16 * mbx);
  } else if (!luma_only && lane < 44) {
    // lanes 20..31: U rows -4..7, lanes 32..43: V rows -4..7
    const int pl = lane >= 32, j = (pl ? lane - 32 : lane - 20) - 4;
    uint8_t* ft = pl ? fv : fu;
    uint8_t* P = pl ? Vp : Up;
    const uint8_t* src = wb + (pl ? LV : LU);
    if (j >= 0) {
      *reinterpret_cast<uint2*>(ft + (j + 4) * FC_STRIDE + FC_X0) = *reinterpret_cast<const uint2*>(src + j * WG_BPS);
      if (mbx > 0)
        *reinterpret_cast<uint32_t*>(ft + (j + 4) * FC_STRIDE + FC_X0 - 4) =
            *reinterpret_cast<const uint32_t*>(P + (int64_t)(8 * mby + j) * uvs + 8 * mbx - 4);
    } else if (mby > 0) {
      *reinterpret_cast<uint2*>(ft + (j + 4) * FC_STRIDE + FC_X0) =
          *reinterpret_cast<const uint2*>(P + (int64_t)(8 * mby + j) * uvs + 8 * mbx);
    }
  }
  __syncthreads();

  const int limit = info.f_limit, ilevel = info.f_ilevel, hev_t = info.hev_thresh;
  const bool inner = info.f_inner != 0;
  // 5b. horizontal filtering across vertical edges: left MB edge, then inner edges x = 4, 8, 12
  if (lane < 16) {
    uint8_t* row = fy + (lane + 4) * FY_STRIDE + FY_X0;
    if (luma_only) {
      if (mbx > 0) f_simple(row, 0, 1, limit + 4);
      if (inner)
        for (int e = 4; e < 16; e += 4) f_simple(row, e, 1, limit);
    } else {
      if (mbx > 0) f_complex(row, 0, 1, limit + 4, ilevel, hev_t, false);
      if (inner)
        for (int e = 4; e < 16; e += 4) f_complex(row, e, 1, limit, ilevel, hev_t, true);
    }
  } else if (!luma_only && lane < 32) {
    const int pl = lane >= 24, j = lane - (pl ? 24 : 16);
    uint8_t* row = (pl ? fv : fu) + (j + 4) * FC_STRIDE + FC_X0;
    if (mbx > 0) f_complex(row, 0, 1, limit + 4, ilevel, hev_t, false);
    if (inner) f_complex(row, 4, 1, limit, ilevel, hev_t, true);
  }
  __syncthreads();
  // 5c. vertical filtering across horizontal edges: top MB edge, then inner edges y = 4, 8, 12
  if (lane < 16) {
    uint8_t* col = fy + 4 * FY_STRIDE + FY_X0 + lane;
    if (luma_only) {
      if (mby > 0) f_simple(col, 0, FY_STRIDE, limit + 4);
      if (inner)
        for (int e = 4; e < 16; e += 4) f_simple(col, e * FY_STRIDE, FY_STRIDE, limit);
    } else {
      if (mby > 0) f_complex(col, 0, FY_STRIDE, limit + 4, ilevel, hev_t, false);
      if (inner)
        for (int e = 4; e < 16; e += 4) f_complex(col, e * FY_STRIDE, FY_STRIDE, limit, ilevel, hev_t, true);
    }
  } else if (!luma_only && lane < 32) {
    const int pl = lane >= 24, i = lane - (pl ? 24 : 16);
    uint8_t* col = (pl ? fv : fu) + 4 * FC_STRIDE + FC_X0 + i;
    if (mby > 0) f_complex(col, 0, FC_STRIDE, limit + 4, ilevel, hev_t, false);
    if (inner) f_complex(col, 4 * FC_STRIDE, FC_STRIDE, limit, ilevel, hev_t, true);
  }
  __syncthreads();

  // 5d. write back: the MB, the 3 modified columns of the left MB, the 3 modified rows above
  if (lane < 16) {
    *reinterpret_cast<uint4*>(Yp + (int64_t)(16 * mby + lane) * ys + 16 * mbx) =
        *reinterpret_cast<const uint4*>(fy + (lane + 4) * FY_STRIDE + FY_X0);
    if (mbx > 0)
      *reinterpret_cast<uint32_t*>(Yp + (int64_t)(16 * mby + lane) * ys + 16 * mbx - 4) =
          *reinterpret_cast<const uint32_t*>(fy + (lane + 4) * FY_STRIDE + FY_X0 - 4);
  } else if (lane < 19) {
    if (mby > 0) {
      const int j = lane - 16 + 1;  // rows -3..-1
      *reinterpret_cast<uint4*>(Yp + (int64_t)(16 * mby - 4 + j) * ys + 16 * mbx) =
          *reinterpret_cast<const uint4*>(fy + j * FY_STRIDE + FY_X0);
    }
  } else if (lane >= 20 && lane < 44) {
    const int pl = lane >= 32, j = (pl ? lane - 32 : lane - 20) - 4;
    const uint8_t* ft = pl ? fv : fu;
    uint8_t* P = pl ? Vp : Up;
    const uint8_t* src = luma_only ? wb + (pl ? LV : LU) + j * WG_BPS : ft + (j + 4) * FC_STRIDE + FC_X0;
    if (j >= 0) {
      *reinterpret_cast<uint2*>(P + (int64_t)(8 * mby + j) * uvs + 8 * mbx) = *reinterpret_cast<const uint2*>(src);
      if (!luma_only && mbx > 0)
        *reinterpret_cast<uint32_t*>(P + (int64_t)(8 * mby + j) * uvs + 8 * mbx - 4) =
            *reinterpret_cast<const uint32_t*>(ft + (j + 4) * FC_STRIDE + FC_X0 - 4);
    } else if (!luma_only && mby > 0 && j >= -3) {
      *reinterpret_cast<uint2*>(P + (int64_t)(8 * mby + j) * uvs + 8 * mbx) =
          *reinterpret_cast<const uint2*>(ft + (j + 4) * FC_STRIDE + FC_X0);
    }
  }
}

}  // namespace

extern "C" size_t wg_decode_work_bytes(int32_t mbw, int32_t mbh, int32_t n_images) {
  if (mbw <= 0 || mbh <= 0 || n_images <= 0) return 0;
  return (size_t)n_images * ((size_t)mbw * TOP_BYTES + (size_t)mbh * LEFT_BYTES);
}

extern "C" int wg_decode_frames(const wg_mb_info* mb, const int16_t* coeffs, int32_t filter_type, int32_t mbw,
                                int32_t mbh, int32_t n_images, uint8_t* y, uint8_t* u, uint8_t* v, void* work,
                                void* stream) {
  WG_REQUIRE(mb && coeffs && y && u && v && work);
  WG_REQUIRE(mbw > 0 && mbh > 0 && n_images > 0);
  WG_REQUIRE(filter_type >= 0 && filter_type <= 2);
  WG_REQUIRE((reinterpret_cast<uintptr_t>(y) & 15) == 0 && (reinterpret_cast<uintptr_t>(u) & 7) == 0 &&
             (reinterpret_cast<uintptr_t>(v) & 7) == 0 && (reinterpret_cast<uintptr_t>(coeffs) & 15) == 0);
  DecArgs a;
  a.mb = mb;
  a.coeffs = coeffs;
  a.Y = y;
  a.U = u;
  a.V = v;
  a.top = static_cast<uint8_t*>(work);
  a.left = a.top + (size_t)n_images * mbw * TOP_BYTES;
  a.filter_type = filter_type;
  a.mbw = mbw;
  a.mbh = mbh;
  hipStream_t s = wg::as_stream(stream);
  const int T = mbw + 2 * (mbh - 1);
  for (int t = 0; t < T; t++) {
    int x_lo = t - 2 * (mbh - 1);
    if (x_lo < 0) x_lo = (t & 1);  // smallest x >= 0 with x == t (mod 2)
    const int x_hi = t < mbw - 1 ? t : mbw - 1;
    if (x_hi < x_lo) continue;
    const int count = (x_hi - x_lo) / 2 + 1;
    hipLaunchKernelGGL(k_decode_diag, dim3((unsigned)(count * n_images)), dim3(64), 0, s, a, t, x_lo, count);
  }
  return wg::check_launch("k_decode_diag");
}
