// decode.hip -- VP8 decoder reconstruct + loop filter for whole frames on
// gfx950 (replaces reconstructRow / filterRowAt of parseFrame,
// internal/lossy/decode.go:532-560 and decode_frame.go:83-342).
//
// Schedule: one persistent launch per batch.  Each 64-lane workgroup
// dequeues a macroblock ROW (ordered counter, row-major over y then image)
// and walks it left to right, exactly like the reference's serial row loop,
// keeping the left context (the decoder's yuvB rotation,
// decode_frame.go:118-126) in LDS.  Row y may process MB x once row y-1 has
// completed MB x+1: that covers intra prediction (top / top-right from the
// unfiltered MB above) and the loop filter (the MB above and above-right
// already filtered, since their edge filters write 3 pixels into row y-1's
// bottom rows).  Because rows are dequeued in order, a row only ever waits
// on rows owned by already-running workgroups: no deadlock for any grid
// size, and every wait is bounded (a timeout sets an error flag).
//
// Cross-workgroup hand-off (MI355X_MICROARCH.md, "Valid forms", sc1 row):
// every byte another workgroup reads -- the unfiltered top context and all
// frame pixels -- is stored with sc1 (write-through) stores and loaded with
// sc1 loads; the producer drains its stores (s_waitcnt vmcnt(0)) before the
// progress flag store; the consumer polls the flag with sc1 loads.
//
// Lane mapping per macroblock: luma block b = lane/4 (raster), row lane%4,
// 4 pixels per lane; chroma lanes 0-15 U, 16-31 V.
#include <cstddef>
#include <cstdlib>

#include "wg_common.h"
#include "wg_dsp.h"

namespace {

using namespace wg;

// LDS work-buffer layout (stride WG_BPS).  Origins are 16-byte aligned.  The Y
// top-right pixels at columns 16..19 land in columns 0..3 of the next row,
// which nothing else uses (the left border is column 15, the V block's left
// border column 31 of the previous row).
constexpr int LY = 1 * WG_BPS + 16;   // Y origin: row 1, col 16
constexpr int LU = 19 * WG_BPS + 16;  // U origin: row 19, col 16
constexpr int LV = 19 * WG_BPS + 0;   // V origin: row 19, col 0
constexpr int WB_SIZE = 27 * WG_BPS;

// Filter tiles: rows -4..15 (Y) / -4..7 (U,V) of the MB, columns -4..15 / -4..7.
constexpr int FY_STRIDE = 32, FY_X0 = 16;  // Y col c at byte FY_X0 + c
constexpr int FC_STRIDE = 16, FC_X0 = 8;

constexpr int TOP_BYTES = 32;  // per MB column: unfiltered Y16 U8 V8 of the MB above

__device__ __forceinline__ int check_mode(int mbx, int mby, int mode) {
  // checkMode (decode_frame.go:6-19) as one select chain: the early-return
  // form was miscompiled by hipcc (ROCm 7.2, -O3; the NoTop constant
  // overwrote `mode` on the mbx>0 && mby>0 path).
  const int edge = (mbx == 0) ? ((mby == 0) ? 6 : 5) : ((mby == 0) ? 4 : 0);
  return mode == 0 ? edge : mode;
}

// sc1 (agent-coherent, L1-bypassing, write-through) accesses for hand-off data.
__device__ __forceinline__ uint64_t ld_sc1_64(const uint8_t* p) {
  return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_64(uint8_t* p, uint64_t v) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_32(uint8_t* p, uint32_t v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lds64(const uint8_t* p) { return *reinterpret_cast<const uint64_t*>(p); }
__device__ __forceinline__ uint32_t lds32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }

static_assert(sizeof(wg_mb_info) == 32 && offsetof(wg_mb_info, imodes) == 8 && offsetof(wg_mb_info, is_i4x4) == 24 &&
                  offsetof(wg_mb_info, f_limit) == 28 && offsetof(wg_mb_info, hev_thresh) == 31,
              "k_decode_rows reads wg_mb_info as 8 words");

struct DecArgs {
  const wg_mb_info* mb;
  const int16_t* coeffs;
  uint8_t* Y;
  uint8_t* U;
  uint8_t* V;
  uint8_t* top;   // [n_img][mbw][TOP_BYTES]
  int* progress;  // [n_img][mbh]: macroblocks completed (reconstructed + filtered + stored)
  int* ctl;       // [0] row dequeue counter, [1] error flag (wait timeout)
  int filter_type, mbw, mbh, n_img;
};

#ifdef WG_STAMPS
// Diagnostic build only: cycles spent per phase, summed over all macroblocks.
__device__ unsigned long long g_phase[16];
#define STAMP_DECL unsigned long long st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_prev = 0
#define STAMP(k)                                                                   \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    unsigned long long ts_;                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ts_)::"memory");  \
    __builtin_amdgcn_sched_barrier(0);                                             \
    if ((k) > 0) st_acc[(k)-1] += ts_ - st_prev;                                   \
    st_prev = ts_;                                                                 \
  } while (0)
#define STAMP_FLUSH()                                                          \
  do {                                                                         \
    if (lane == 0)                                                             \
      for (int k_ = 0; k_ < 10; k_++) atomicAdd(&g_phase[k_], st_acc[k_]);     \
  } while (0)
#else
#define STAMP_DECL int st_unused_ = 0
#define STAMP(k) (void)st_unused_
#define STAMP_FLUSH() (void)st_unused_
#endif

// Loop filter of one MB on the LDS tiles (doFilter, decode_frame.go:293-342):
// lanes 0-15 luma line 0-15, lanes 16-31 chroma line 0-7 of U / V.  A line is
// 20 (luma) / 12 (chroma) pixels: 4 of the left / upper neighbour, then the
// MB.  Each lane filters all edges of its line in registers (rf_line); the
// row pass (H edges) completes before the column pass (V edges).
template <bool COMPLEX>
__device__ __forceinline__ void filter_mb(uint8_t* fy, uint8_t* fu, uint8_t* fv, int lane, bool chroma, bool left,
                                          bool top, bool inner, int limit, int ilevel, int hev_t) {
  const bool luma = lane < 16;
  const bool active = luma || (chroma && lane < 32);
  const int pl = lane >= 24, j = (lane - 16) & 7;
  if (active) {
    uint8_t* rowp = luma ? fy + (lane + 4) * FY_STRIDE + FY_X0 - 4 : (pl ? fv : fu) + (j + 4) * FC_STRIDE + FC_X0 - 4;
    // chroma lanes read 8 bytes past their 12-pixel line (in-bounds LDS: the
    // next row, or the tile that follows); they are never written back
    uint32_t w[5];
#pragma unroll
    for (int k = 0; k < 5; k++) w[k] = *reinterpret_cast<const uint32_t*>(rowp + 4 * k);
    int v[20];
#pragma unroll
    for (int k = 0; k < 20; k++) v[k] = byte_of(w[k >> 2], k & 3);
    rf_line<COMPLEX>(v, left, inner, luma, limit, ilevel, hev_t);
#pragma unroll
    for (int k = 0; k < 3; k++)
      *reinterpret_cast<uint32_t*>(rowp + 4 * k) = pack4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    if (luma) {
      *reinterpret_cast<uint32_t*>(rowp + 12) = pack4(v[12], v[13], v[14], v[15]);
      *reinterpret_cast<uint32_t*>(rowp + 16) = pack4(v[16], v[17], v[18], v[19]);
    }
  }
  __syncthreads();
  if (active) {
    uint8_t* col = luma ? fy + FY_X0 + lane : (pl ? fv : fu) + FC_X0 + j;
    const int st = luma ? FY_STRIDE : FC_STRIDE;
    int v[20];
#pragma unroll
    for (int k = 0; k < 20; k++) v[k] = col[k * st];
    rf_line<COMPLEX>(v, top, inner, luma, limit, ilevel, hev_t);
#pragma unroll
    for (int k = 1; k < 12; k++) col[k * st] = (uint8_t)v[k];
    if (luma) {
#pragma unroll
      for (int k = 12; k < 20; k++) col[k * st] = (uint8_t)v[k];
    }
  }
  __syncthreads();
}

// threadIdx.x through an opaque move, re-read at every phase of the MB loop:
// stops the compiler from hoisting each phase's lane-derived LDS / global
// addresses out of the loop, where they would pin ~60 VGPRs for the whole
// kernel and cut the resident workgroups per CU.
__device__ __forceinline__ int opaque_lane() {
  int l;
  asm volatile("v_mov_b32 %0, %1" : "=v"(l) : "v"((int)threadIdx.x));
  return l;
}

constexpr uint64_t SPIN_TICKS = 200000000ull;  // 2 s of the 100 MHz s_memrealtime clock per wait

__global__ __launch_bounds__(64) void k_decode_rows(DecArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t wb[WB_SIZE];
  // prefetch landing zone: coefficients (48 x 16 B) then the wg_mb_info (2 x 16 B)
  __shared__ __attribute__((aligned(16))) int4 stage[50];
  int16_t* const cof = reinterpret_cast<int16_t*>(stage);
  // filter tiles Y | U | V, then slack that chroma lanes of filter_mb read
  // (never write) when they run the 20-pixel luma code path
  __shared__ __attribute__((aligned(16))) uint8_t ftiles[20 * FY_STRIDE + 2 * 12 * FC_STRIDE + 8 * FC_STRIDE];
  uint8_t* const fy = ftiles;
  uint8_t* const fu = ftiles + 20 * FY_STRIDE;
  uint8_t* const fv = fu + 12 * FC_STRIDE;
  __shared__ int sh_word;

  int lane = threadIdx.x;
  const int mbw = a.mbw, mbh = a.mbh;
  const int total_rows = a.n_img * mbh;
  const int ys = 16 * mbw, uvs = 8 * mbw;
  const bool luma_only = a.filter_type == 1;
  STAMP_DECL;

  for (;;) {
    if (lane == 0) sh_word = __hip_atomic_fetch_add(&a.ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int row = __builtin_amdgcn_readfirstlane(sh_word);
    __syncthreads();
    if (row >= total_rows) break;
    const int mby = row / a.n_img, img = row % a.n_img;
    uint8_t* top = a.top + (int64_t)img * mbw * TOP_BYTES;
    int* prog_above = a.progress + (int64_t)img * mbh + mby - 1;
    int* prog_mine = a.progress + (int64_t)img * mbh + mby;
    uint8_t* Yp = a.Y + (int64_t)img * ys * 16 * mbh;
    uint8_t* Up = a.U + (int64_t)img * uvs * 8 * mbh;
    uint8_t* Vp = a.V + (int64_t)img * uvs * 8 * mbh;

    // row start: left border 129, top-left 129 (127 on the first row) -- decode_frame.go:93-110
    if (lane < 16) wb[LY - 1 + lane * WG_BPS] = 129;
    else if (lane < 24) wb[LU - 1 + (lane - 16) * WG_BPS] = 129;
    else if (lane < 32) wb[LV - 1 + (lane - 24) * WG_BPS] = 129;
    else if (lane < 35) wb[(lane == 32 ? LY : lane == 33 ? LU : LV) - WG_BPS - 1] = mby > 0 ? 129 : 127;
    int seen = 0;  // progress of the row above observed so far
    // Register prefetch of the next macroblock's coefficients + info (lanes
    // 0-47 / 48-49): issued once the current MB's hand-off loads are consumed,
    // so it overlaps the MB's compute (loads retire in order: issuing it
    // earlier would make every wait on a hand-off load wait for it too).
    const int64_t row_mb0 = ((int64_t)img * mbh + mby) * mbw;
    int4 pf = make_int4(0, 0, 0, 0);
    if (lane < 48) pf = reinterpret_cast<const int4*>(a.coeffs + row_mb0 * 384)[lane];
    else if (lane < 50) pf = reinterpret_cast<const int4*>(a.mb + row_mb0)[lane - 48];

    for (int mbx = 0; mbx < mbw; mbx++) {
      const int64_t mbi = ((int64_t)img * mbh + mby) * mbw + mbx;
      STAMP(0);
      // ---- dependency on the row above ----
      if (mby > 0) {
        const int need = min(mbx + 2, mbw);
        if (seen < need) {
          int v = 0;
          if (lane == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (uint32_t it = 0;; it++) {
              v = __hip_atomic_load(prog_above, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if (v >= need) break;
              // never hang the GPU: after SPIN_TICKS (or once any row has timed out)
              // flag the error and carry on with whatever is in memory
              if ((it & 63) == 63 &&
                  (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS ||
                   __hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
                __hip_atomic_fetch_or(&a.ctl[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v = mbw;
                break;
              }
              __builtin_amdgcn_s_sleep(2);
            }
          }
          seen = __shfl(v, 0, 64);
        }
      }
      STAMP(1);
      lane = opaque_lane();
      // ---- loads: macroblock info (scalar), coefficients -> LDS, top context, filter rows above ----
      if (lane < 50) stage[lane] = pf;
      // rotate the filter tile: the left MB's final columns 12..15 become columns -4..-1
      if (mbx > 0) {
        if (lane < 16) {
          uint8_t* r = fy + (lane + 4) * FY_STRIDE + FY_X0;
          *reinterpret_cast<uint32_t*>(r - 4) = lds32(r + 12);
        } else if (lane < 32) {
          const int j = (lane - 16) & 7;
          uint8_t* r = ((lane < 24) ? fu : fv) + (j + 4) * FC_STRIDE + FC_X0;
          *reinterpret_cast<uint32_t*>(r - 4) = lds32(r + 4);
        }
      }
      if (mby > 0) {
        const uint8_t* tc = top + mbx * TOP_BYTES;
        if (lane >= 48 && lane < 52) {  // unfiltered top context Y16 U8 V8
          const uint64_t w = ld_sc1_64(tc + 8 * (lane - 48));
          const int k = lane - 48;
          uint8_t* dst = k < 2 ? wb + LY - WG_BPS + 8 * k : (k == 2 ? wb + LU - WG_BPS : wb + LV - WG_BPS);
          *reinterpret_cast<uint64_t*>(dst) = w;
        } else if (lane >= 52 && lane < 60) {  // filtered frame rows 16y-4..16y-1 (Y)
          const int k = lane - 52, rr = k >> 1, half = k & 1;
          const uint64_t w = ld_sc1_64(Yp + (int64_t)(16 * mby - 4 + rr) * ys + 16 * mbx + 8 * half);
          *reinterpret_cast<uint64_t*>(fy + rr * FY_STRIDE + FY_X0 + 8 * half) = w;
        } else if (lane >= 60) {  // U rows 8y-4..8y-1
          const int rr = lane - 60;
          *reinterpret_cast<uint64_t*>(fu + rr * FC_STRIDE + FC_X0) =
              ld_sc1_64(Up + (int64_t)(8 * mby - 4 + rr) * uvs + 8 * mbx);
        } else if (lane >= 44) {  // V rows (lanes 44..47)
          const int rr = lane - 44;
          *reinterpret_cast<uint64_t*>(fv + rr * FC_STRIDE + FC_X0) =
              ld_sc1_64(Vp + (int64_t)(8 * mby - 4 + rr) * uvs + 8 * mbx);
        }
        if (lane == 0) {  // top-right: next MB's top context, or replicate top[15] at the right edge
          uint32_t tr;
          if (mbx < mbw - 1) tr = (uint32_t)ld_sc1_64(tc + TOP_BYTES);
          else tr = 0x01010101u * (uint32_t)(ld_sc1_64(tc + 8) >> 56);
          *reinterpret_cast<uint32_t*>(wb + LY - WG_BPS + 16) = tr;
        }
      } else {  // first row: everything above is 127 (decode_frame.go:104-108)
        if (lane < 21) wb[LY - WG_BPS + lane - 1] = 127;
        else if (lane < 30) wb[LU - WG_BPS + lane - 22] = 127;
        else if (lane < 39) wb[LV - WG_BPS + lane - 31] = 127;
      }
      __syncthreads();
      if (mbx + 1 < mbw) {  // prefetch the next MB (see above)
        if (lane < 48) pf = reinterpret_cast<const int4*>(a.coeffs + (mbi + 1) * 384)[lane];
        else if (lane < 50) pf = reinterpret_cast<const int4*>(a.mb + mbi + 1)[lane - 48];
      }
      const uint32_t* iw = reinterpret_cast<const uint32_t*>(stage + 48);  // wg_mb_info words
      const uint32_t nz_y = __builtin_amdgcn_readfirstlane(iw[0]), nz_uv = __builtin_amdgcn_readfirstlane(iw[1]);
      const uint32_t im0 = __builtin_amdgcn_readfirstlane(iw[2]);
      const uint32_t w6 = __builtin_amdgcn_readfirstlane(iw[6]), w7 = __builtin_amdgcn_readfirstlane(iw[7]);
      const int is_i4 = w6 & 0xff, uv_mode = (w6 >> 8) & 0xff;
      const int f_limit = w7 & 0xff, ilevel = (w7 >> 8) & 0xff, f_inner = (w7 >> 16) & 0xff, hev_t = w7 >> 24;
      const uint8_t* imodes = reinterpret_cast<const uint8_t*>(stage + 48) + 8;
      if (is_i4 && lane < 12) {  // replicate top-right down to rows 3, 7, 11 (:155-160)
        const int r = 4 * (lane / 4 + 1) - 1, i = lane & 3;
        wb[LY + r * WG_BPS + 16 + i] = wb[LY - WG_BPS + 16 + i];
      }
      __syncthreads();

      STAMP(2);
      lane = opaque_lane();
      // ---- luma prediction + residual ----
      {
        const int blk = lane >> 2, r = lane & 3, bx = blk & 3, by = blk >> 2;
        const int off = LY + (4 * by + r) * WG_BPS + 4 * bx;
        const int code = (nz_y >> (30 - 2 * blk)) & 3;
        int res[4];
        dec_residual_row(cof + blk * 16, code, r, res);
        if (!is_i4) {
          const int mode = check_mode(mbx, mby, im0 & 0xff);
          const int dc = predsq_dc(mode, wb + LY, 16);
          const uint32_t pred = predsq_row4(mode, wb + LY, 4 * bx, 4 * by + r, dc);
          *reinterpret_cast<uint32_t*>(wb + off) =
              pack4(clip8(byte_of(pred, 0) + res[0]), clip8(byte_of(pred, 1) + res[1]),
                    clip8(byte_of(pred, 2) + res[2]), clip8(byte_of(pred, 3) + res[3]));
        } else {
          const int my_step = bx + 2 * by;  // in-MB dependency wavefront
          const int mode = imodes[blk];
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
      STAMP(3);
      lane = opaque_lane();
      // ---- chroma prediction + residual (doUVTransform :47-68) ----
      if (lane < 32) {
        const int pl = lane >> 4, cblk = (lane >> 2) & 3, r = lane & 3;
        const int cbx = cblk & 1, cby = cblk >> 1;
        const int base = pl ? LV : LU;
        const int mode = check_mode(mbx, mby, uv_mode);
        const int dc = predsq_dc(mode, wb + base, 8);
        const uint32_t pred = predsq_row4(mode, wb + base, 4 * cbx, 4 * cby + r, dc);
        const uint32_t bits = nz_uv >> (8 * pl);
        const int16_t* bco = cof + (16 + 4 * pl + cblk) * 16;
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

      STAMP(4);
      lane = opaque_lane();
      // ---- unfiltered top context for the row below (:190-194) + MB into the filter tiles ----
      if (mby < mbh - 1 && lane >= 32 && lane < 36) {
        const int k = lane - 32;
        const uint8_t* src =
            k < 2 ? wb + LY + 15 * WG_BPS + 8 * k : (k == 2 ? wb + LU + 7 * WG_BPS : wb + LV + 7 * WG_BPS);
        st_sc1_64(top + mbx * TOP_BYTES + 8 * k, lds64(src));
      }
      if (lane < 16) {
        *reinterpret_cast<uint4*>(fy + (lane + 4) * FY_STRIDE + FY_X0) =
            *reinterpret_cast<const uint4*>(wb + LY + lane * WG_BPS);
      } else if (lane < 32) {
        const int pl = lane >= 24, j = (lane - 16) & 7;
        *reinterpret_cast<uint64_t*>((pl ? fv : fu) + (j + 4) * FC_STRIDE + FC_X0) =
            lds64(wb + (pl ? LV : LU) + j * WG_BPS);
      }
      __syncthreads();

      STAMP(5);
      lane = opaque_lane();
      // ---- loop filter (doFilter :293-342): H edges (left MB edge, inner x=4,8,12), then V edges ----
      const bool do_filter = a.filter_type > 0 && f_limit > 0;
      const bool inner = f_inner != 0;
      if (do_filter) {
        if (a.filter_type == 2) filter_mb<true>(fy, fu, fv, lane, true, mbx > 0, mby > 0, inner, f_limit, ilevel, hev_t);
        else filter_mb<false>(fy, fu, fv, lane, false, mbx > 0, mby > 0, inner, f_limit, ilevel, hev_t);
      }

      STAMP(6);
      lane = opaque_lane();
      // ---- stores (all sc1: the row below reads them) ----
      if (lane < 32) {  // Y rows, 2 x 8 B
        const int j = lane >> 1, half = lane & 1;
        st_sc1_64(Yp + (int64_t)(16 * mby + j) * ys + 16 * mbx + 8 * half,
                  lds64(fy + (j + 4) * FY_STRIDE + FY_X0 + 8 * half));
      } else if (lane < 48) {  // U, V rows
        const int pl = lane >= 40, j = (lane - 32) & 7;
        st_sc1_64((pl ? Vp : Up) + (int64_t)(8 * mby + j) * uvs + 8 * mbx,
                  lds64((pl ? fv : fu) + (j + 4) * FC_STRIDE + FC_X0));
      }
      if (do_filter) {
        if (mbx > 0) {  // the 3 columns of the left MB modified by our left-edge filter
          if (lane >= 48) {
            st_sc1_32(Yp + (int64_t)(16 * mby + lane - 48) * ys + 16 * mbx - 4,
                      lds32(fy + (lane - 48 + 4) * FY_STRIDE + FY_X0 - 4));
          } else if (!luma_only && lane < 16) {
            const int pl = lane >= 8, j = lane & 7;
            st_sc1_32((pl ? Vp : Up) + (int64_t)(8 * mby + j) * uvs + 8 * mbx - 4,
                      lds32((pl ? fv : fu) + (j + 4) * FC_STRIDE + FC_X0 - 4));
          }
        }
        if (mby > 0) {  // the 3 rows of the MB above modified by our top-edge filter
          if (lane >= 16 && lane < 22) {
            const int k = lane - 16, rr = 1 + (k >> 1), half = k & 1;
            st_sc1_64(Yp + (int64_t)(16 * mby - 4 + rr) * ys + 16 * mbx + 8 * half,
                      lds64(fy + rr * FY_STRIDE + FY_X0 + 8 * half));
          } else if (!luma_only && lane >= 22 && lane < 28) {
            const int k = lane - 22, pl = k >= 3, rr = 1 + (k % 3);
            st_sc1_64((pl ? Vp : Up) + (int64_t)(8 * mby - 4 + rr) * uvs + 8 * mbx,
                      lds64((pl ? fv : fu) + rr * FC_STRIDE + FC_X0));
          }
        }
      }
      // ---- rotate the reconstruction context for the next MB (:118-126) ----
      if (lane < 16) wb[LY - 1 + lane * WG_BPS] = wb[LY + 15 + lane * WG_BPS];
      else if (lane < 24) wb[LU - 1 + (lane - 16) * WG_BPS] = wb[LU + 7 + (lane - 16) * WG_BPS];
      else if (lane < 32) wb[LV - 1 + (lane - 24) * WG_BPS] = wb[LV + 7 + (lane - 24) * WG_BPS];
      else if (lane == 32) wb[LY - WG_BPS - 1] = wb[LY - WG_BPS + 15];
      else if (lane == 33) wb[LU - WG_BPS - 1] = wb[LU - WG_BPS + 7];
      else if (lane == 34) wb[LV - WG_BPS - 1] = wb[LV - WG_BPS + 7];
      __syncthreads();
      STAMP(7);
      lane = opaque_lane();
      // ---- publish: every store of this MB is complete before the flag ----
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(prog_mine, mbx + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      STAMP(8);
    }
  }
  STAMP_FLUSH();
}

int g_num_cus = 0;
int g_rows_per_cu = 0;  // resident workgroups per CU (occupancy)

}  // namespace

#ifdef WG_STAMPS
extern "C" int wg_debug_phases(unsigned long long* host, int n) {
  hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * n);
  unsigned long long z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)) == hipSuccess ? 0 : -2;
}
#endif

extern "C" size_t wg_decode_work_bytes(int32_t mbw, int32_t mbh, int32_t n_images) {
  if (mbw <= 0 || mbh <= 0 || n_images <= 0) return 0;
  return (size_t)n_images * mbw * TOP_BYTES + sizeof(int) * ((size_t)n_images * mbh + 4);
}

extern "C" int wg_decode_frames(const wg_mb_info* mb, const int16_t* coeffs, int32_t filter_type, int32_t mbw,
                                int32_t mbh, int32_t n_images, uint8_t* y, uint8_t* u, uint8_t* v, void* work,
                                void* stream) {
  WG_REQUIRE(mb && coeffs && y && u && v && work);
  WG_REQUIRE(mbw > 0 && mbh > 0 && n_images > 0);
  WG_REQUIRE(filter_type >= 0 && filter_type <= 2);
  WG_REQUIRE(((reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(v)) &
              7) == 0 &&
             (reinterpret_cast<uintptr_t>(coeffs) & 15) == 0 && (reinterpret_cast<uintptr_t>(mb) & 15) == 0 && (reinterpret_cast<uintptr_t>(work) & 15) == 0);
  DecArgs a;
  a.mb = mb;
  a.coeffs = coeffs;
  a.Y = y;
  a.U = u;
  a.V = v;
  a.top = static_cast<uint8_t*>(work);
  a.ctl = reinterpret_cast<int*>(a.top + (size_t)n_images * mbw * TOP_BYTES);
  a.progress = a.ctl + 4;
  a.filter_type = filter_type;
  a.mbw = mbw;
  a.mbh = mbh;
  a.n_img = n_images;
  hipStream_t s = wg::as_stream(stream);
  if (g_num_cus == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0 ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_decode_rows, 64, 0) != hipSuccess || per_cu <= 0)
      return wg::check_launch("decode occupancy query");
    g_num_cus = cus;
    g_rows_per_cu = per_cu;
    if (const char* e = getenv("WG_DECODE_WG_PER_CU")) g_rows_per_cu = atoi(e) > 0 ? atoi(e) : per_cu;  // tuning
  }
  if (hipMemsetAsync(a.ctl, 0, sizeof(int) * ((size_t)n_images * mbh + 4), s) != hipSuccess)
    return wg::check_launch("hipMemsetAsync(decode ctl)");
  const int rows = n_images * mbh;
  const int grid = rows < g_rows_per_cu * g_num_cus ? rows : g_rows_per_cu * g_num_cus;
  hipLaunchKernelGGL(k_decode_rows, dim3((unsigned)grid), dim3(64), 0, s, a);
  return wg::check_launch("k_decode_rows");
}

extern "C" int wg_decode_status(const void* work, int32_t mbw, int32_t n_images, void* stream) {
  WG_REQUIRE(work && mbw > 0 && n_images > 0);
  const int* ctl =
      reinterpret_cast<const int*>(static_cast<const uint8_t*>(work) + (size_t)n_images * mbw * TOP_BYTES);
  int flag = 0;
  hipStream_t s = wg::as_stream(stream);
  if (hipMemcpyAsync(&flag, ctl + 1, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return wg::check_launch("wg_decode_status");
  if (flag) {
    wg::set_error("decode: a row dependency wait timed out (output invalid)");
    return WG_EHIP;
  }
  return WG_OK;
}
