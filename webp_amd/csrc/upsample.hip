// upsample.hip -- "fancy" 4:2:0 -> 4:4:4 chroma upsampling + YUV->RGB to
// NRGBA on gfx950: replaces buildNRGBA (webp.go:379-450) and the line-pair
// kernel it drives, UpsampleLinePairNRGBA (upsample.go:130-236,
// upsample_direct_amd64.go:10-134).
//
// The reference walks overlapping line pairs; every output pixel is a pure
// function of one luma sample and a 2x2 chroma neighbourhood, so here each
// thread produces four 4-pixel groups of both rows of a line pair.  Which
// two chroma rows a luma row reads, and whether it takes the "top" or
// "bottom" half of the diamond kernel, follows buildNRGBA's row schedule:
//   row 0 -> chroma (0, 0), top;  odd r -> ((r-1)/2, (r+1)/2 or (r-1)/2 on the
//   last row of an even-height image), top;  even r>0 -> (r/2-1, r/2), bottom.
// u and v travel as two 16-bit lanes of one word (like the LOAD_UV packing of
// upsample.go:14-16, and likewise never carrying between the halves).
#include <algorithm>

#include "wg_common.h"
#include "wg_dsp.h"
#include "wg_yuv.h"

namespace {
using namespace wg;

struct UpArgs {
  const uint8_t *y, *u, *v, *alpha;
  uint8_t* out;
  int64_t y_pitch, uv_pitch, a_pitch, out_pitch;
  int y_stride, uv_stride, w, h;
  int fast_uv;   // chroma rows 8-byte aligned -> 8-byte chunk loads into LDS
  int fast_y;    // luma rows 4-byte aligned -> one dword per group
  int fast_a;    // alpha rows 4-byte aligned
  int fast_out;  // output rows 16-byte aligned -> one 16-byte store per group
};

constexpr int UP_T = 256;                // most threads per block
constexpr int UP_GROUPS = 4;             // 4-pixel groups per thread and row

// Packed chroma: word = u | v << 16, so U and V are interpolated together as
// two 16-bit lanes.  Right shifts let the v lane's low bits fall into the u
// lane's bits 12-15; every intermediate stays below 2^16 per lane and only
// the low 8 bits of each lane are kept, so the stray bits never reach a result.
__device__ __forceinline__ uint32_t uv_pack(uint32_t ub, uint32_t vb, int byte) {  // bytes of two dwords
  const uint32_t sel = (uint32_t)byte | 0x0cu << 8 | (uint32_t)(4 + byte) << 16 | 0x0cu << 24;
  return __builtin_amdgcn_perm(vb, ub, sel);
}

// The diamond kernel of chroma pair (tl, tt / l, cur) (upsample.go:140-230):
// diag12 / diag03 are shared by the pair's two pixels and by both output rows
//   top row:    odd pixel (diag12 + tl) >> 1, even pixel (diag03 + tt) >> 1
//   bottom row: odd pixel (diag03 + l) >> 1,  even pixel (diag12 + cur) >> 1
struct Diamond {
  uint32_t d12, d03;
  __device__ __forceinline__ Diamond(uint32_t tl, uint32_t tt, uint32_t l, uint32_t cur) {
    const uint32_t avg = tl + tt + l + cur + 0x00080008u;
    d12 = (avg + 2 * (tt + l)) >> 3;
    d03 = (avg + 2 * (tl + cur)) >> 3;
  }
};

__device__ __forceinline__ uint32_t load4(const uint8_t* row, int x, int w, bool fast) {
  if (fast) return *reinterpret_cast<const uint32_t*>(row + x);
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) v |= (uint32_t)row[min(x + i, w - 1)] << (8 * i);
  return v;
}

__device__ __forceinline__ void store4(const UpArgs& a, uint8_t* orow, int x, const uint32_t* px) {
  if (a.fast_out && x + 4 <= a.w) {
    *reinterpret_cast<uint4*>(orow + 4 * x) = make_uint4(px[0], px[1], px[2], px[3]);
  } else {
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (x + i < a.w) *reinterpret_cast<uint32_t*>(orow + 4 * (x + i)) = px[i];
  }
}

__device__ __forceinline__ uint32_t rgba_of(uint32_t yw, uint32_t aw, int i, uint32_t cuv) {
  return yuv_to_rgba((int)((yw >> (8 * i)) & 0xff), (int)(cuv & 0xff), (int)((cuv >> 16) & 0xff),
                     (int)((aw >> (8 * i)) & 0xff));
}

// One block = one LINE PAIR of one image over 16 * blockDim.x columns
// (blockDim.x = 64..256, the fewest waves that cover the width).  Output rows
// 2p-1 (odd, "top" half of the diamond) and 2p (even, "bottom" half) read the
// same two chroma rows (max(p-1,0), min(p,ch-1)) -- buildNRGBA's schedule
// (webp.go:379-450) folded into pairs: row 0 is pair 0 alone, and on an even
// height the last odd row repeats its chroma row.
//
// The two chroma rows are staged in LDS as packed u|v words (8-byte loads).
// Lane l of wave k owns the 4-pixel groups at x = 1024k + 256g + 4l (g = 0..3),
// so every luma load and every 16-byte NRGBA store of a wave is one
// contiguous span (with 16 contiguous pixels per lane the stores were 64 B
// apart and the L2 wrote the partial lines back twice: WRITE_SIZE 1.9x).
__global__ __launch_bounds__(UP_T) void k_upsample(const UpArgs a) {
  // word i = chroma column cbase - 8 + i of the top (wt) and bottom (wb)
  // chroma row; dynamic LDS sized to the block (2 x (8 * blockDim.x + 16) words)
  extern __shared__ uint4 up_lds[];
  const int up_c = 8 * (int)blockDim.x;  // chroma columns of this block
  uint32_t* wt = reinterpret_cast<uint32_t*>(up_lds);
  uint32_t* wb = wt + up_c + 16;
  const int p = blockIdx.y, img = blockIdx.z, t = threadIdx.x;
  const int w = a.w, h = a.h, cw = (w + 1) >> 1, ch = (h + 1) >> 1;
  const int ct = max(p - 1, 0), cb = min(p, ch - 1);
  const int cbase = blockIdx.x * up_c;
  const uint8_t* U = a.u + img * a.uv_pitch;
  const uint8_t* V = a.v + img * a.uv_pitch;
  {
    const uint8_t* rows[2][2] = {{U + (int64_t)ct * a.uv_stride, V + (int64_t)ct * a.uv_stride},
                                 {U + (int64_t)cb * a.uv_stride, V + (int64_t)cb * a.uv_stride}};
    const int c0 = cbase + 8 * t;  // this thread's 8 chroma columns
    if (c0 < cw + 8) {
#pragma unroll
      for (int r = 0; r < 2; r++) {
        uint2 q[2];
#pragma unroll
        for (int pl = 0; pl < 2; pl++) {
          if (a.fast_uv && c0 + 8 <= cw) {
            q[pl] = *reinterpret_cast<const uint2*>(rows[r][pl] + c0);
          } else {
            q[pl] = make_uint2(load4(rows[r][pl], min(c0, cw - 1), cw, false),
                               load4(rows[r][pl], min(c0 + 4, cw - 1), cw, false));
          }
        }
        uint32_t* dst = (r ? wb : wt) + 8 + 8 * t;
        *reinterpret_cast<uint4*>(dst) = make_uint4(uv_pack(q[0].x, q[1].x, 0), uv_pack(q[0].x, q[1].x, 1),
                                                    uv_pack(q[0].x, q[1].x, 2), uv_pack(q[0].x, q[1].x, 3));
        *reinterpret_cast<uint4*>(dst + 4) = make_uint4(uv_pack(q[0].y, q[1].y, 0), uv_pack(q[0].y, q[1].y, 1),
                                                        uv_pack(q[0].y, q[1].y, 2), uv_pack(q[0].y, q[1].y, 3));
      }
    }
    if (t < 4) {  // halo: 8 columns left of cbase and right of cbase + up_c, clamped
      const int r = t & 1;
      const bool right = t >= 2;
      const int cc = right ? cbase + up_c : cbase - 8;
      uint32_t* dst = (r ? wb : wt) + (right ? 8 + up_c : 0);
      for (int i = 0; i < 8; i++) {
        const int c = min(max(cc + i, 0), cw - 1);
        dst[i] = (uint32_t)rows[r][0][c] | (uint32_t)rows[r][1][c] << 16;
      }
    }
  }
  // luma / alpha of all groups are loaded before the barrier, so their
  // latency overlaps the chroma staging
  const int rt = p == 0 ? 0 : 2 * p - 1, rb = 2 * p;
  const bool has_t = rt < h, has_b = p > 0 && rb < h;
  const uint8_t* yt = a.y + img * a.y_pitch + (int64_t)rt * a.y_stride;
  const uint8_t* yb = a.y + img * a.y_pitch + (int64_t)rb * a.y_stride;
  const uint8_t* at = a.alpha ? a.alpha + img * a.a_pitch + (int64_t)rt * w : nullptr;
  const uint8_t* ab = a.alpha ? a.alpha + img * a.a_pitch + (int64_t)rb * w : nullptr;
  uint8_t* ot = a.out + img * a.out_pitch + (int64_t)rt * 4 * w;
  uint8_t* ob = a.out + img * a.out_pitch + (int64_t)rb * 4 * w;
  const int xw = 2 * blockIdx.x * up_c + 1024 * (t >> 6) + 4 * (t & 63);
  uint32_t ywt[UP_GROUPS], ywb[UP_GROUPS], awt[UP_GROUPS], awb[UP_GROUPS];
#pragma unroll
  for (int g = 0; g < UP_GROUPS; g++) {
    const int x = xw + 256 * g;
    ywt[g] = ywb[g] = 0;
    awt[g] = awb[g] = ~0u;
    if (x < w) {
      const bool fy = a.fast_y && x + 4 <= w, fa = a.fast_a && x + 4 <= w;
      if (has_t) ywt[g] = load4(yt, x, w, fy);
      if (has_b) ywb[g] = load4(yb, x, w, fy);
      if (at && has_t) awt[g] = load4(at, x, w, fa);
      if (ab && has_b) awb[g] = load4(ab, x, w, fa);
    }
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < UP_GROUPS; g++) {
    const int x = xw + 256 * g;
    if (x >= w) break;
    const int i0 = x / 2 - 1 - cbase + 8;  // LDS word of window column 0 (chroma x/2 - 1)
    const uint32_t T0 = wt[i0], T1 = wt[i0 + 1], T2 = wt[i0 + 2], T3 = wt[i0 + 3];
    const uint32_t B0 = wb[i0], B1 = wb[i0 + 1], B2 = wb[i0 + 2], B3 = wb[i0 + 3];
    uint32_t top[4], bot[4];
    if (x != 0 && x + 4 < w) {  // interior group
      const Diamond k1(T0, T1, B0, B1), k2(T1, T2, B1, B2), k3(T2, T3, B2, B3);
      top[0] = (k1.d03 + T1) >> 1;
      bot[0] = (k1.d12 + B1) >> 1;
      top[1] = (k2.d12 + T1) >> 1;
      bot[1] = (k2.d03 + B1) >> 1;
      top[2] = (k2.d03 + T2) >> 1;
      bot[2] = (k2.d12 + B2) >> 1;
      top[3] = (k3.d12 + T2) >> 1;
      bot[3] = (k3.d03 + B2) >> 1;
    } else {  // border rules: x == 0 vertical only; trailing pixel of an even width vertical only
      const uint32_t Tw[4] = {T0, T1, T2, T3}, Bw[4] = {B0, B1, B2, B3};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int k = ((i + 1) >> 1) + 1;
        const int xi = x + i;
        if (xi == 0) {
          top[i] = (3 * Tw[1] + Bw[1] + 0x00020002u) >> 2;
          bot[i] = (3 * Bw[1] + Tw[1] + 0x00020002u) >> 2;
        } else if ((i & 1) && xi == w - 1 && (w & 1) == 0) {
          top[i] = (3 * Tw[k - 1] + Bw[k - 1] + 0x00020002u) >> 2;
          bot[i] = (3 * Bw[k - 1] + Tw[k - 1] + 0x00020002u) >> 2;
        } else {
          const Diamond d(Tw[k - 1], Tw[k], Bw[k - 1], Bw[k]);
          top[i] = (i & 1) ? (d.d12 + Tw[k - 1]) >> 1 : (d.d03 + Tw[k]) >> 1;
          bot[i] = (i & 1) ? (d.d03 + Bw[k - 1]) >> 1 : (d.d12 + Bw[k]) >> 1;
        }
      }
    }
    if (has_t) {
      uint32_t px[4];
#pragma unroll
      for (int i = 0; i < 4; i++) px[i] = rgba_of(ywt[g], awt[g], i, top[i]);
      store4(a, ot, x, px);
    }
    if (has_b) {
      uint32_t px[4];
#pragma unroll
      for (int i = 0; i < 4; i++) px[i] = rgba_of(ywb[g], awb[g], i, bot[i]);
      store4(a, ob, x, px);
    }
  }
}

}  // namespace

extern "C" int wg_upsample_nrgba(const uint8_t* y, int32_t y_stride, int64_t y_pitch, const uint8_t* u,
                                 const uint8_t* v, int32_t uv_stride, int64_t uv_pitch, const uint8_t* alpha,
                                 int64_t a_pitch, int32_t w, int32_t h, uint8_t* out, int64_t out_pitch,
                                 int32_t n_images, void* stream) {
  WG_REQUIRE(y && u && v && out && w > 0 && h > 0 && n_images > 0);
  WG_REQUIRE(y_stride >= w && uv_stride >= (w + 1) / 2 && out_pitch >= (int64_t)4 * w * h);
  WG_REQUIRE((reinterpret_cast<uintptr_t>(out) & 3) == 0 && (out_pitch & 3) == 0);
  WG_REQUIRE(h / 2 + 1 <= 65535 && n_images <= 65535);
  UpArgs a;
  a.y = y;
  a.u = u;
  a.v = v;
  a.alpha = alpha;
  a.out = out;
  a.y_pitch = y_pitch;
  a.uv_pitch = uv_pitch;
  a.a_pitch = a_pitch;
  a.out_pitch = out_pitch;
  a.y_stride = y_stride;
  a.uv_stride = uv_stride;
  a.w = w;
  a.h = h;
  a.fast_uv = ((reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(v) | (uintptr_t)uv_stride |
                (uintptr_t)uv_pitch) & 7) == 0;
  a.fast_y = ((reinterpret_cast<uintptr_t>(y) | (uintptr_t)y_stride | (uintptr_t)y_pitch) & 3) == 0;
  a.fast_a = alpha && ((reinterpret_cast<uintptr_t>(alpha) | (uintptr_t)w | (uintptr_t)a_pitch) & 3) == 0;
  a.fast_out = ((reinterpret_cast<uintptr_t>(out) | (uintptr_t)out_pitch) & 15) == 0 && (w & 3) == 0;
  const int threads = (int)std::min<int64_t>(UP_T, (w + 1023) / 1024 * 64);  // a wave covers 1024 columns
  const dim3 grid((unsigned)((w + 16 * threads - 1) / (16 * threads)), (unsigned)(h / 2 + 1), (unsigned)n_images);
  const size_t lds = 2 * sizeof(uint32_t) * (8 * threads + 16);
  hipLaunchKernelGGL(k_upsample, grid, dim3(threads), lds, wg::as_stream(stream), a);
  return wg::check_launch("k_upsample");
}
