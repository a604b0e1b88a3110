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
#include <cstring>

#include <mutex>

#include "wg_common.h"
#include "wg_dsp.h"
#include "wg_instr.h"

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
// Filter tiles: Y col c at byte FY_X0 + c, U / V col c at FC_X0 + c.  The
// columns left of the MB hold the MBs to its left (two for Y, four for U / V),
// so the frame rows leave in 32-B pieces -- whole 32-B sectors of an L2 line --
// once those MBs are final.
constexpr int FY_STRIDE = 48, FY_X0 = 32;
constexpr int FC_STRIDE = 40, FC_X0 = 32;

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
// one 16-B write-through store (a bottom-row record leaves as 8 x 16 B, one 128-B line).
// The s_nop: a store of more than 8 bytes reads its data VGPRs after issue,
// and a VALU write to them in the next cycle corrupts the stored bytes; the
// compiler's hazard recognizer does not look inside the asm (round 6: a
// variant of k_decode_split got its next address computation into the data
// registers right after the store, and stored address bits)
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_sc1_128(uint8_t* p, uint4 w) {
  const u32x4_t v = {w.x, w.y, w.z, w.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
// Coefficients are read exactly once: non-temporal loads, so the stream
// (2 B / coefficient, the kernel's largest input) does not push the frame's
// partly written output lines out of L2 before their other pieces arrive.
__device__ __forceinline__ int4 ld_stream(const int4* p) {
  typedef int v4i __attribute__((ext_vector_type(4)));
  const v4i v = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(p));
  return make_int4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint64_t lds64(const uint8_t* p) { return *reinterpret_cast<const uint64_t*>(p); }

// (WG_DEC_SKIPW / WG_BOUNDS builds, wg_instr.h: DEC_SITE(bit) drops a store
// site of k_decode_bands, WG_IN checks an access against its buffer)
// k_decode_bands' frame stores
__device__ __forceinline__ void frame_st16(uint8_t* p, uint4 w) {
  *reinterpret_cast<uint4*>(p) = w;
}
__device__ __forceinline__ void frame_st8(uint8_t* p, uint64_t w) {
  *reinterpret_cast<uint64_t*>(p) = w;
}
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
  uint8_t* bot;   // [n_img][mbw][BOT_BYTES] (k_decode_split): final rows 12..15 of a band's last row, for the next band
  int* progress;  // [n_img][mbh]: macroblocks completed (reconstructed + filtered + stored)
  int* ctl;       // [0] row dequeue counter, [1] error flag (wait timeout)
  int* diag;      // wg::diag_words + DIAG_DECODE
  int filter_type, mbw, mbh, n_img;
};

// (WG_STAMPS builds, wg_instr.h) cycles spent per phase, summed over all macroblocks
WG_IF_STAMPS(__device__ unsigned long long g_phase[16];)

// wave-level LDS ordering: this wave's LDS accesses retire before what follows
// (the LDS unit executes one wave's DS instructions in issue order, so a
// read after a write of the same wave -- or another wave's read after this
// wave's later flag store -- sees the write without draining the queue; the
// drain cost C3 3.6%: 4.75 -> 4.58 ms.)
__device__ __forceinline__ void lds_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

template <bool COMPLEX>
__device__ __forceinline__ void filter_mb_rows(uint8_t* fy, uint8_t* fu, uint8_t* fv, int lane, bool chroma, bool left,
                                               bool inner, int limit, int ilevel, int hev_t) {
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
  lds_sync();
}
template <bool COMPLEX>
__device__ __forceinline__ void filter_mb_cols(uint8_t* fy, uint8_t* fu, uint8_t* fv, int lane, bool chroma, bool top,
                                               bool inner, int limit, int ilevel, int hev_t) {
  const bool luma = lane < 16;
  const bool active = luma || (chroma && lane < 32);
  const int pl = lane >= 24, j = (lane - 16) & 7;
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
  lds_sync();
}
// Loop filter of one MB on the LDS tiles (doFilter, decode_frame.go:293-342):
// lanes 0-15 luma line 0-15, lanes 16-31 chroma line 0-7 of U / V.  A line is
// 20 (luma) / 12 (chroma) pixels: 4 of the left / upper neighbour, then the
// MB.  Each lane filters all edges of its line in registers (rf_line); the
// row pass (H edges) completes before the column pass (V edges).  One wave:
// the passes are ordered with wave-level LDS syncs.
template <bool COMPLEX>
__device__ __forceinline__ void filter_mb(uint8_t* fy, uint8_t* fu, uint8_t* fv, int lane, bool chroma, bool left,
                                          bool top, bool inner, int limit, int ilevel, int hev_t) {
  filter_mb_rows<COMPLEX>(fy, fu, fv, lane, chroma, left, inner, limit, ilevel, hev_t);
  filter_mb_cols<COMPLEX>(fy, fu, fv, lane, chroma, top, inner, limit, ilevel, hev_t);
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

// Rows per workgroup (one wave each) and the depth of the intra-band LDS rings.
constexpr int DW = 4;
constexpr int RING = 8;
constexpr int BOT_BYTES = 128;  // final rows 12..15 of an MB: Y 4 x 16, U 4 x 8, V 4 x 8

// bounded spin on a progress word (LDS or agent-scope global) by lane 0
template <bool GLOBAL>
__device__ __forceinline__ int wait_progress(const int* p, int need, int* err_flag, int give_up, int* diag) {
  const uint64_t t0 = wg::wait_clock();
  for (uint32_t it = 0;; it++) {
    int v;
    if (GLOBAL) v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else v = __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);  // pairs with the tprog release
    if (v >= need) return v;
    // never hang the GPU: after SPIN_TICKS (or once any wait has timed out)
    // flag the error and carry on with whatever is in memory
    if ((it & 63) == 63 && (wg::wait_clock() - t0 > SPIN_TICKS ||
                            __hip_atomic_load(err_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
      __hip_atomic_fetch_or(err_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      wg::note_timeout(diag, need, v, GLOBAL ? 1 : 0, (int)(wg::wait_clock() - t0), (int)blockIdx.x,
                       (int)(threadIdx.x >> 6));
      return give_up;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// The I4 blocks' steps inside one macroblock (decode_frame.go:148-170's raster
// order, run as a wavefront).  Block (bx, by) reads the finished pixels of
// its left and top neighbours (and, through them, the top-left one), and
// the top-right neighbour's bottom row only in the modes that read T[4..7]:
// VE4, LD4, VL4 (wg_dsp.h pred4_row; the right column's top-right comes
// from the MB above-right instead, see top_right_step).  Each block runs at
// the first step after its dependencies: bx + by steps when no mode reads
// an in-MB top-right, up to the static bx + 2 by.  Returns the 16 steps as
// 4-bit fields (block b at bits 4b..4b+3); modes are uniform, so this is
// scalar work.
__device__ __forceinline__ uint64_t i4_schedule(uint32_t im0, uint32_t im1, uint32_t im2, uint32_t im3) {
  const uint32_t im[4] = {im0, im1, im2, im3};
  int st[16];
  uint64_t packed = 0;
#pragma unroll
  for (int b = 0; b < 16; b++) {
    const int bx = b & 3, by = b >> 2;
    const uint32_t m = (im[by] >> (8 * bx)) & 0xff;
    int v = bx > 0 ? st[b - 1] + 1 : 0;
    if (by > 0) v = max(v, st[b - 4] + 1);
    if (by > 0 && bx < 3 && (m == 2 || m == 6 || m == 7)) v = max(v, st[b - 3] + 1);
    st[b] = v;
    packed |= (uint64_t)v << (4 * b);
  }
  return packed;
}

// Band schedule: a workgroup of DW waves dequeues a band of DW consecutive
// macroblock rows of one image (ordered counter over (band, image)); wave r
// walks row DW*band + r.  Wave 0 depends on the previous band's last row
// through global memory exactly as a lone row would (sc1 hand-off, progress
// counter); waves r > 0 depend on wave r-1 through LDS: a RING-deep ring per
// wave of the unfiltered top context (32 B) and the final bottom rows 12..15
// (128 B) of each finished MB, and an LDS progress word.  The bottom rows of
// an MB are final once the MB to its right has run its left-edge filter, so,
// as across bands, the consumer waits for MB x+1 of the row above.  Across
// bands the same rows travel as one 128-B write-through record per MB column
// (a.bot, as in k_decode_split), drained before the progress flag.  Writes
// to the frame never overlap: a producer leaves its rows 13..15 (Y) / 5..7
// (U, V) to the row below, which stores them after its top-edge filter
// (changed or not), so every frame byte is written once.
__global__ __launch_bounds__(64 * DW) void k_decode_bands(DecArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t wb_all[DW][WB_SIZE];
  // prefetch landing zone: coefficients (48 x 16 B) then the wg_mb_info (2 x 16 B)
  __shared__ __attribute__((aligned(16))) int4 stage_all[DW][50];
  // filter tiles Y | U | V, then slack that chroma lanes of filter_mb read
  // (never write) when they run the 20-pixel luma code path
  constexpr int FT_BYTES = 20 * FY_STRIDE + 2 * 12 * FC_STRIDE + 8 * FC_STRIDE;
  __shared__ __attribute__((aligned(16))) uint8_t ftiles_all[DW][FT_BYTES];
  __shared__ __attribute__((aligned(16))) uint8_t top_ring[DW][RING][TOP_BYTES];
  __shared__ __attribute__((aligned(16))) uint8_t bot_ring[DW][RING][BOT_BYTES];
  __shared__ int prog_lds[DW];
  __shared__ int sh_word;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  uint8_t* const wb = wb_all[wave];
  int16_t* const cof = reinterpret_cast<int16_t*>(stage_all[wave]);
  int4* const stage = stage_all[wave];
  uint8_t* const fy = ftiles_all[wave];
  uint8_t* const fu = fy + 20 * FY_STRIDE;
  uint8_t* const fv = fu + 12 * FC_STRIDE;
  const int mbw = a.mbw, mbh = a.mbh;
  const int bands = (mbh + DW - 1) / DW;
  const int total = a.n_img * bands;
  const int ys = 16 * mbw, uvs = 8 * mbw;
  const bool luma_only = a.filter_type == 1;
  STAMP_DECL;
  // (WG_BOUNDS) the buffers' extents
  [[maybe_unused]] const int64_t n_mb = (int64_t)a.n_img * mbh * mbw, y_size = n_mb * 256, uv_size = n_mb * 64,
                                 top_size = (int64_t)a.n_img * mbw * TOP_BYTES, bot_size = (int64_t)a.n_img * mbw * BOT_BYTES;

  for (;;) {
    if (threadIdx.x == 0) sh_word = __hip_atomic_fetch_add(&a.ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) prog_lds[wave] = 0;
    __syncthreads();
    const int idx = __builtin_amdgcn_readfirstlane(sh_word);
    __syncthreads();
    if (idx >= total) break;
    const int band = idx / a.n_img, img = idx % a.n_img;
    const int mby = band * DW + wave;
    const int last_wave = min(DW, mbh - band * DW) - 1;  // the band's last row
    if (wave <= last_wave) {
      const bool from_lds = wave > 0;           // the row above is in this band
      const bool to_lds = wave < last_wave;      // the row below is in this band
      uint8_t* top = a.top + (int64_t)img * mbw * TOP_BYTES;
      int* prog_above = a.progress + (int64_t)img * mbh + mby - 1;
      int* prog_mine = a.progress + (int64_t)img * mbh + mby;
      uint8_t* Yp = a.Y + (int64_t)img * ys * 16 * mbh;
      uint8_t* Up = a.U + (int64_t)img * uvs * 8 * mbh;
      uint8_t* Vp = a.V + (int64_t)img * uvs * 8 * mbh;
      // a band's last row hands the next band each MB's final rows 12..15 as
      // one 128-B record (Y 4 x 16 B, U 4 x 8, V 4 x 8; bot_ring's layout)
      uint8_t* const bot_img = a.bot + (int64_t)img * mbw * BOT_BYTES;
      const bool hand = !to_lds && mby < mbh - 1;

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
      if (lane < 48) {
        const int4* pp = reinterpret_cast<const int4*>(a.coeffs + row_mb0 * 384) + lane;
        if (WG_IN(pp, 16, a.coeffs, n_mb * 768, &a.ctl[1])) pf = ld_stream(pp);
      } else if (lane < 50) {
        const int4* pp = reinterpret_cast<const int4*>(a.mb + row_mb0) + (lane - 48);
        if (WG_IN(pp, 16, a.mb, n_mb * 32, &a.ctl[1])) pf = *pp;
      }

      for (int mbx = 0; mbx < mbw; mbx++) {
        const int64_t mbi = ((int64_t)img * mbh + mby) * mbw + mbx;
        const int slot = mbx & (RING - 1);
        STAMP(0);
        // ---- dependency on the row above (and ring space in the row below) ----
        if (mby > 0) {
          const int need = min(mbx + 2, mbw);
          if (seen < need) {
            int v = 0;
            if (lane == 0)
              v = from_lds ? wait_progress<false>(&prog_lds[wave - 1], need, &a.ctl[1], mbw, a.diag)
                           : wait_progress<true>(prog_above, need, &a.ctl[1], mbw, a.diag);
            seen = __shfl(v, 0, 64);
          }
        }
        if (to_lds && mbx >= RING - 1) {  // ring slot `slot` must have been read by the row below
          if (lane == 0) wait_progress<false>(&prog_lds[wave + 1], mbx - RING + 2, &a.ctl[1], mbw, a.diag);
          lds_sync();
        }
        STAMP(1);
        lane = opaque_lane() & 63;
        // ---- loads: macroblock info (scalar), coefficients -> LDS, top context, filter rows above ----
        if (lane < 50) stage[lane] = pf;
        // rotate the filter tiles: the MBs to the left move one MB further left
        // (our left-edge filter then finishes the left MB's columns 13..15)
        if (mbx > 0) {  // shift every tile row left by one MB (all loads before all stores)
          uint4 y0 = make_uint4(0, 0, 0, 0);
          uint64_t c[2] = {0, 0};
          if (lane < 40) y0 = *reinterpret_cast<const uint4*>(fy + (lane >> 1) * FY_STRIDE + FY_X0 - 16 + 16 * (lane & 1));
#pragma unroll
          for (int h = 0; h < 2; h++) {  // U, V: 24 rows x 4 words
            const int i = lane + 64 * h;
            if (i < 96) {
              const int row = i >> 2, pl = row >= 12;
              c[h] = lds64((pl ? fv : fu) + (row - 12 * pl) * FC_STRIDE + FC_X0 - 24 + 8 * (i & 3));
            }
          }
          lds_sync();
          if (lane < 40) *reinterpret_cast<uint4*>(fy + (lane >> 1) * FY_STRIDE + FY_X0 - 32 + 16 * (lane & 1)) = y0;
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const int i = lane + 64 * h;
            if (i < 96) {
              const int row = i >> 2, pl = row >= 12;
              *reinterpret_cast<uint64_t*>((pl ? fv : fu) + (row - 12 * pl) * FC_STRIDE + FC_X0 - 32 + 8 * (i & 3)) = c[h];
            }
          }
        }
        if (mby > 0 && from_lds) {
          const uint8_t* tc = top_ring[wave - 1][slot];
          const uint8_t* bt = bot_ring[wave - 1][slot];
          if (lane >= 48 && lane < 52) {  // unfiltered top context Y16 U8 V8
            const int k = lane - 48;
            uint8_t* dst = k < 2 ? wb + LY - WG_BPS + 8 * k : (k == 2 ? wb + LU - WG_BPS : wb + LV - WG_BPS);
            *reinterpret_cast<uint64_t*>(dst) = lds64(tc + 8 * k);
          } else if (lane >= 52 && lane < 60) {  // final rows 12..15 of the MB above (Y)
            const int k = lane - 52, rr = k >> 1, half = k & 1;
            *reinterpret_cast<uint64_t*>(fy + rr * FY_STRIDE + FY_X0 + 8 * half) = lds64(bt + 16 * rr + 8 * half);
          } else if (lane >= 60) {  // U rows 4..7
            const int rr = lane - 60;
            *reinterpret_cast<uint64_t*>(fu + rr * FC_STRIDE + FC_X0) = lds64(bt + 64 + 8 * rr);
          } else if (lane >= 44) {  // V rows (lanes 44..47)
            const int rr = lane - 44;
            *reinterpret_cast<uint64_t*>(fv + rr * FC_STRIDE + FC_X0) = lds64(bt + 96 + 8 * rr);
          }
          if (lane == 0) {  // top-right: next MB's top context, or replicate top[15] at the right edge
            uint32_t tr;
            if (mbx < mbw - 1) tr = lds32(top_ring[wave - 1][(mbx + 1) & (RING - 1)]);
            else tr = 0x01010101u * (uint32_t)tc[15];
            *reinterpret_cast<uint32_t*>(wb + LY - WG_BPS + 16) = tr;
          }
        } else if (mby > 0) {
          const uint8_t* tc = top + mbx * TOP_BYTES;
          if (lane >= 48 && lane < 52) {  // unfiltered top context Y16 U8 V8
            const uint64_t w = WG_IN(tc + 8 * (lane - 48), 8, a.top, top_size, &a.ctl[1]) ? ld_sc1_64(tc + 8 * (lane - 48)) : 0;
            const int k = lane - 48;
            uint8_t* dst = k < 2 ? wb + LY - WG_BPS + 8 * k : (k == 2 ? wb + LU - WG_BPS : wb + LV - WG_BPS);
            *reinterpret_cast<uint64_t*>(dst) = w;
          } else if (lane >= 52 && lane < 60) {  // the previous band's record: Y rows 16y-4..16y-1
            const int k = lane - 52, rr = k >> 1, half = k & 1;
            const uint8_t* bp = bot_img + mbx * BOT_BYTES + 16 * rr + 8 * half;
            const uint64_t w = WG_IN(bp, 8, a.bot, bot_size, &a.ctl[1]) ? ld_sc1_64(bp) : 0;
            *reinterpret_cast<uint64_t*>(fy + rr * FY_STRIDE + FY_X0 + 8 * half) = w;
          } else if (lane >= 60) {  // U rows 8y-4..8y-1
            const int rr = lane - 60;
            const uint8_t* bp = bot_img + mbx * BOT_BYTES + 64 + 8 * rr;
            *reinterpret_cast<uint64_t*>(fu + rr * FC_STRIDE + FC_X0) = WG_IN(bp, 8, a.bot, bot_size, &a.ctl[1]) ? ld_sc1_64(bp) : 0;
          } else if (lane >= 44) {  // V rows (lanes 44..47)
            const int rr = lane - 44;
            const uint8_t* bp = bot_img + mbx * BOT_BYTES + 96 + 8 * rr;
            *reinterpret_cast<uint64_t*>(fv + rr * FC_STRIDE + FC_X0) = WG_IN(bp, 8, a.bot, bot_size, &a.ctl[1]) ? ld_sc1_64(bp) : 0;
          }
          if (lane == 0) {  // top-right: next MB's top context, or replicate top[15] at the right edge
            uint32_t tr;
            if (mbx < mbw - 1) tr = WG_IN(tc + TOP_BYTES, 8, a.top, top_size, &a.ctl[1]) ? (uint32_t)ld_sc1_64(tc + TOP_BYTES) : 0u;
            else tr = 0x01010101u * (uint32_t)((WG_IN(tc + 8, 8, a.top, top_size, &a.ctl[1]) ? ld_sc1_64(tc + 8) : 0ull) >> 56);
            *reinterpret_cast<uint32_t*>(wb + LY - WG_BPS + 16) = tr;
          }
        } else {  // first row: everything above is 127 (decode_frame.go:104-108)
          if (lane < 21) wb[LY - WG_BPS + lane - 1] = 127;
          else if (lane < 30) wb[LU - WG_BPS + lane - 22] = 127;
          else if (lane < 39) wb[LV - WG_BPS + lane - 31] = 127;
        }
        lds_sync();
        if (mbx + 1 < mbw) {  // prefetch the next MB (see above)
          if (lane < 48) {
            const int4* pp = reinterpret_cast<const int4*>(a.coeffs + (mbi + 1) * 384) + lane;
            if (WG_IN(pp, 16, a.coeffs, n_mb * 768, &a.ctl[1])) pf = ld_stream(pp);
          } else if (lane < 50) {
            const int4* pp = reinterpret_cast<const int4*>(a.mb + mbi + 1) + (lane - 48);
            if (WG_IN(pp, 16, a.mb, n_mb * 32, &a.ctl[1])) pf = *pp;
          }
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
        lds_sync();

        STAMP(2);
        lane = opaque_lane() & 63;
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
            const uint64_t sched = i4_schedule(im0, __builtin_amdgcn_readfirstlane(iw[3]),
                                               __builtin_amdgcn_readfirstlane(iw[4]),
                                               __builtin_amdgcn_readfirstlane(iw[5]));
            const int my_step = (int)(sched >> (4 * blk)) & 15;  // in-MB dependency wavefront
            const int n_steps = (int)(sched >> 60) + 1;           // block 15 is last
            const int mode = imodes[blk];
            for (int s = 0; s < n_steps; s++) {
              if (s == my_step) {
                int X, T[8], L[4];
                pred4_ctx(wb, LY + 4 * by * WG_BPS + 4 * bx, X, T, L);
                const uint32_t pred = pred4_row(mode, r, X, T, L);
                *reinterpret_cast<uint32_t*>(wb + off) =
                    pack4(clip8(byte_of(pred, 0) + res[0]), clip8(byte_of(pred, 1) + res[1]),
                          clip8(byte_of(pred, 2) + res[2]), clip8(byte_of(pred, 3) + res[3]));
              }
              lds_sync();
            }
          }
        }
        STAMP(3);
        lane = opaque_lane() & 63;
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
        lds_sync();

        STAMP(4);
        lane = opaque_lane() & 63;
        // ---- unfiltered top context for the row below (:190-194) + MB into the filter tiles ----
        if (mby < mbh - 1 && lane >= 32 && lane < 36) {
          const int k = lane - 32;
          const uint8_t* src =
              k < 2 ? wb + LY + 15 * WG_BPS + 8 * k : (k == 2 ? wb + LU + 7 * WG_BPS : wb + LV + 7 * WG_BPS);
          if (to_lds) {
            *reinterpret_cast<uint64_t*>(top_ring[wave][slot] + 8 * k) = lds64(src);
          } else if (k < 2) {  // the record as two 16-B write-through stores (Y | U V): one 32-B write
            uint4 w;
            if (k == 0) {
              w = *reinterpret_cast<const uint4*>(wb + LY + 15 * WG_BPS);
            } else {
              const uint64_t u = lds64(wb + LU + 7 * WG_BPS), v = lds64(wb + LV + 7 * WG_BPS);
              w = make_uint4((uint32_t)u, (uint32_t)(u >> 32), (uint32_t)v, (uint32_t)(v >> 32));
            }
            if (DEC_SITE(1) && WG_IN(top + mbx * TOP_BYTES + 16 * k, 16, a.top, top_size, &a.ctl[1]))
              st_sc1_128(top + mbx * TOP_BYTES + 16 * k, w);
          }
        }
        if (lane < 16) {
          *reinterpret_cast<uint4*>(fy + (lane + 4) * FY_STRIDE + FY_X0) =
              *reinterpret_cast<const uint4*>(wb + LY + lane * WG_BPS);
        } else if (lane < 32) {
          const int pl = lane >= 24, j = (lane - 16) & 7;
          *reinterpret_cast<uint64_t*>((pl ? fv : fu) + (j + 4) * FC_STRIDE + FC_X0) =
              lds64(wb + (pl ? LV : LU) + j * WG_BPS);
        }
        lds_sync();

        STAMP(5);
        lane = opaque_lane() & 63;
        // ---- loop filter (doFilter :293-342): H edges (left MB edge, inner x=4,8,12), then V edges ----
        const bool do_filter = a.filter_type > 0 && f_limit > 0;
        const bool inner = f_inner != 0;
        if (do_filter) {
          if (a.filter_type == 2) filter_mb<true>(fy, fu, fv, lane, true, mbx > 0, mby > 0, inner, f_limit, ilevel, hev_t);
          else filter_mb<false>(fy, fu, fv, lane, false, mbx > 0, mby > 0, inner, f_limit, ilevel, hev_t);
        }

        STAMP(6);
        lane = opaque_lane() & 63;
        // ---- stores ----
        // An MB's pixels are final once the MB to its right has run its
        // left-edge filter, except rows 13..15 (Y) / 5..7 (U, V), which the
        // row below finishes with its top-edge filter.  Rows leave in 32-B
        // pieces (two Y MBs, four U / V MBs) once every MB of the piece is
        // final, and the rest at the row's end: every frame byte is written
        // once, by the wave that finalises it, as whole 32-B sectors; rows
        // 13..15 / 5..7 are the row below's to store, in this band or the
        // next.  Only the next band's filter context is written through
        // (sc1): a band's last row hands it MB x - 1's final rows 12..15 (at
        // the row's end this MB's too) as one 128-B record per MB.
        if (hand) {
          const int which = lane >> 3, k = lane & 7, x = mbx - 1 + which;
          if (lane < 16 && (which == 0 ? mbx > 0 : mbx == mbw - 1)) {
            uint4 w;
            if (k < 4) {
              w = *reinterpret_cast<const uint4*>(fy + (16 + k) * FY_STRIDE + FY_X0 + 16 * (x - mbx));
            } else {  // U rows 4,5 | 6,7, V rows 4,5 | 6,7
              const uint8_t* src = ((k >= 6) ? fv : fu) + (8 + 2 * (k & 1)) * FC_STRIDE + FC_X0 + 8 * (x - mbx);
              const uint64_t a0 = lds64(src), a1 = lds64(src + FC_STRIDE);
              w = make_uint4((uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1, (uint32_t)(a1 >> 32));
            }
            if (DEC_SITE(2) && WG_IN(bot_img + x * BOT_BYTES + 16 * k, 16, a.bot, bot_size, &a.ctl[1]))
              st_sc1_128(bot_img + x * BOT_BYTES + 16 * k, w);
          }
        }
        {
          const bool last = mbx == mbw - 1;
          // Y: MBs [y0, y1] leave now (tile column of MB m: 16 (m - mbx)).
          // Pieces go out at even mbx for the two MBs before it; at the row's
          // end everything not yet stored (up to 3 MBs) does.
          int y0 = -1, y1 = -1;
          if (last) {
            y0 = mbx > 0 ? (mbx - 1) & ~1 : 0;
            y1 = mbx;
          } else if (mbx >= 2 && (mbx & 1) == 0) {
            y0 = mbx - 2;
            y1 = mbx - 1;
          }
          int c0 = -1, c1 = -1;  // U, V: likewise, 4-MB pieces (up to 5 MBs at the end)
          if (last) {
            c0 = mbx > 0 ? (mbx - 1) & ~3 : 0;
            c1 = mbx;
          } else if (mbx >= 4 && (mbx & 3) == 0) {
            c0 = mbx - 4;
            c1 = mbx - 1;
          }
          // rows below ylim / clim are this wave's; the rest the row below
          // stores (the image's last row stores all; with the simple filter
          // chroma is never filtered, so its rows are all this wave's)
          const int ylim = to_lds || hand ? 13 : 16, clim = to_lds || (hand && !luma_only) ? 5 : 8;
          if (lane < 48) {  // Y: row lane & 15, MB y0 + (lane >> 4)
            const int j = lane & 15, x = y0 + (lane >> 4);
            if (DEC_SITE(4) && y0 >= 0 && j < ylim && x <= y1) {
              const uint4 w = *reinterpret_cast<const uint4*>(fy + (j + 4) * FY_STRIDE + FY_X0 + 16 * (x - mbx));
              if (WG_IN(Yp + (int64_t)(16 * mby + j) * ys + 16 * x, 16, a.Y, y_size, &a.ctl[1]))
                frame_st16(Yp + (int64_t)(16 * mby + j) * ys + 16 * x, w);
            }
          }
#pragma unroll
          for (int h = 0; h < 2; h++) {  // U, V: row (i & 15), MB c0 + (i >> 4)
            const int i = lane + 64 * h, pl = (i >> 3) & 1, j = i & 7, x = c0 + (i >> 4);
            if (DEC_SITE(8) && c0 >= 0 && i < 80 && j < clim && x <= c1 &&
                WG_IN((pl ? Vp : Up) + (int64_t)(8 * mby + j) * uvs + 8 * x, 8, pl ? a.V : a.U, uv_size, &a.ctl[1]))
              frame_st8((pl ? Vp : Up) + (int64_t)(8 * mby + j) * uvs + 8 * x,
                        lds64((pl ? fv : fu) + (j + 4) * FC_STRIDE + FC_X0 + 8 * (x - mbx)));
          }
          if (mby > 0) {
            // rows 13..15 / 5..7 of the MBs above, final after our top-edge
            // filter (tile rows 1..3): 32-B pieces of the MBs above up to this
            // one, whether or not the filter ran on each (a piece spans MBs;
            // an unfiltered row rewrites the bytes it was loaded with).
            // Nobody reads them again in this launch: plain stores.
            int t0 = -1, t1 = -1;
            if ((mbx & 1) == 1 || last) {
              t0 = mbx & ~1;
              t1 = mbx;
            }
            int u0 = -1, u1 = -1;
            if ((mbx & 3) == 3 || last) {
              u0 = mbx & ~3;
              u1 = mbx;
            }
            if (lane < 6) {
              const int rr = 1 + (lane >> 1), part = lane & 1, x = t0 + part;
              if (DEC_SITE(16) && t0 >= 0 && x <= t1 && WG_IN(Yp + (int64_t)(16 * mby - 4 + rr) * ys + 16 * x, 16, a.Y, y_size, &a.ctl[1]))
                frame_st16(Yp + (int64_t)(16 * mby - 4 + rr) * ys + 16 * x,
                           *reinterpret_cast<const uint4*>(fy + rr * FY_STRIDE + FY_X0 + 16 * (x - mbx)));
            } else if ((from_lds || !luma_only) && lane >= 8 && lane < 32) {
              const int k = lane - 8, pl = k >= 12, rr = 1 + (k % 12) / 4, q = k & 3, x = u0 + q;
              if (DEC_SITE(32) && u0 >= 0 && x <= u1 &&
                  WG_IN((pl ? Vp : Up) + (int64_t)(8 * mby - 4 + rr) * uvs + 8 * x, 8, pl ? a.V : a.U, uv_size, &a.ctl[1]))
                frame_st8((pl ? Vp : Up) + (int64_t)(8 * mby - 4 + rr) * uvs + 8 * x,
                          lds64((pl ? fv : fu) + rr * FC_STRIDE + FC_X0 + 8 * (x - mbx)));
            }
          }
        }
        if (to_lds) {
          // final rows 12..15 of this MB for the row below, and the left MB's
          // columns 12..15 of those rows as our left-edge filter left them
          uint8_t* bt = bot_ring[wave][slot];
          if (lane < 8) {
            const int rr = lane >> 1, half = lane & 1;
            *reinterpret_cast<uint64_t*>(bt + 16 * rr + 8 * half) = lds64(fy + (16 + rr) * FY_STRIDE + FY_X0 + 8 * half);
          } else if (lane < 16) {
            const int k = lane - 8, pl = k >= 4, rr = k & 3;
            *reinterpret_cast<uint64_t*>(bt + 64 + 32 * pl + 8 * rr) =
                lds64((pl ? fv : fu) + (8 + rr) * FC_STRIDE + FC_X0);
          } else if (mbx > 0 && do_filter && lane < 28) {
            uint8_t* bl = bot_ring[wave][(mbx - 1) & (RING - 1)];
            const int k = lane - 16;
            if (k < 4) {
              *reinterpret_cast<uint32_t*>(bl + 16 * k + 12) = lds32(fy + (16 + k) * FY_STRIDE + FY_X0 - 4);
            } else if (!luma_only) {
              const int pl = k >= 8, rr = k & 3;
              *reinterpret_cast<uint32_t*>(bl + 64 + 32 * pl + 8 * rr + 4) =
                  lds32((pl ? fv : fu) + (8 + rr) * FC_STRIDE + FC_X0 - 4);
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
        lds_sync();
        STAMP(7);
        lane = opaque_lane() & 63;
        // ---- publish ----
        if (to_lds) {
          // the rings are written (lds_sync above); the frame stores of a band's
          // rows never overlap, so no drain is needed before the LDS flag
          if (lane == 0) __hip_atomic_store(&prog_lds[wave], mbx + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
          // every store of this MB is complete before the flag
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (lane == 0 && WG_IN(prog_mine, 4, a.progress, (int64_t)a.n_img * mbh * 4, &a.ctl[1]))
            __hip_atomic_store(prog_mine, mbx + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (from_lds && lane == 0) {
          // our progress is also what the row above's ring waits on
          __hip_atomic_store(&prog_lds[wave], mbx + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        STAMP(8);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // the band's LDS rings are reused by the next band
  }
  STAMP_FLUSH();
}

// ---------------------------------------------------------------------------
// Table-driven 4x4 intra prediction of one row (k_decode_split, round 6).
// Every pixel of the ten modes (pred4_row, predict_lossy.go:185-424) is one
// value of a small per-row pool: with E = L3 L2 L1 L0 X T0..T7 (E[-1] = L3,
// E[13..] = T7), A3[i] = avg3(E[i-1], E[i], E[i+1]) for i < 16 and
// A2[i] = avg2(E[i], E[i+1]) for i < 12 -- DC, TM and the left column raw
// aside.  The block's four lanes (a DPP quad: lane = 4 block + row) load its
// context as seven dwords between them, build E packed with v_perm /
// v_alignbyte, take A3 four at a time as two v_lerp_u8 (avg3(a, b, c) =
// (((a + c) >> 1) + b + 1) >> 1: a floor then a rounding byte average) and A2
// as one, write the pool (40 B) to the lane's LDS slot and read the row's
// four bytes back by the mode's code word: no branch on the mode, where
// pred4_row's switch runs every mode present in the step one after another.
// Pool: bytes 0-15 A3, 16-27 A2, 28-31 E[0..3], 32-35 DC, 36-39 TM's row.
// kI4Code[mode][row]: the pool byte of pixel x in byte x (checked against
// pred4_row on random and saturated contexts, all modes and rows).
constexpr uint32_t i4c(int a, int b, int c, int d) { return (uint32_t)a | (uint32_t)b << 8 | (uint32_t)c << 16 | (uint32_t)d << 24; }
__constant__ uint32_t kI4Code[40] = {
    i4c(32, 33, 34, 35), i4c(32, 33, 34, 35), i4c(32, 33, 34, 35), i4c(32, 33, 34, 35),  // DC
    i4c(36, 37, 38, 39), i4c(36, 37, 38, 39), i4c(36, 37, 38, 39), i4c(36, 37, 38, 39),  // TM
    i4c(5, 6, 7, 8), i4c(5, 6, 7, 8), i4c(5, 6, 7, 8), i4c(5, 6, 7, 8),                  // VE
    i4c(3, 3, 3, 3), i4c(2, 2, 2, 2), i4c(1, 1, 1, 1), i4c(0, 0, 0, 0),                  // HE
    i4c(4, 5, 6, 7), i4c(3, 4, 5, 6), i4c(2, 3, 4, 5), i4c(1, 2, 3, 4),                  // RD
    i4c(20, 21, 22, 23), i4c(4, 5, 6, 7), i4c(3, 20, 21, 22), i4c(2, 4, 5, 6),          // VR
    i4c(6, 7, 8, 9), i4c(7, 8, 9, 10), i4c(8, 9, 10, 11), i4c(9, 10, 11, 12),            // LD
    i4c(21, 22, 23, 24), i4c(6, 7, 8, 9), i4c(22, 23, 24, 10), i4c(7, 8, 9, 11),         // VL
    i4c(19, 4, 5, 6), i4c(18, 3, 19, 4), i4c(17, 2, 18, 3), i4c(16, 1, 17, 2),           // HD
    i4c(18, 2, 17, 1), i4c(17, 1, 16, 0), i4c(16, 0, 28, 28), i4c(28, 28, 28, 28)};     // HU
template <int K>
__device__ __forceinline__ uint32_t quad_b(uint32_t v) {  // lane K of the quad to all four (quad_perm [K,K,K,K])
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xf, 0xf, false);
}
// (code: the lane's kI4Code word from LDS; pool: its 48-B LDS slot)
__device__ __forceinline__ uint32_t pred4_row_tab(const uint8_t* wb, int off, int rr, uint32_t cw, uint32_t* pool) {
  const uint8_t* d = wb + off;
  // lane rr: its row's left dword (L[rr] in byte 3); lanes 0 / 1 / 2 the top
  // row's two dwords and the dword ending in X
  const uint32_t ld = lds32(d - 4 + rr * WG_BPS);
  const uint32_t q = lds32(d + (rr == 1 ? 4 - WG_BPS : (rr == 2 ? -4 - WG_BPS : -WG_BPS)));
  const uint32_t l0 = quad_b<0>(ld), l1 = quad_b<1>(ld), l2 = quad_b<2>(ld), l3 = quad_b<3>(ld);
  const uint32_t tlo = quad_b<0>(q), thi = quad_b<1>(q), xd = quad_b<2>(q);
  const uint32_t e0 = __builtin_amdgcn_perm(l2, l3, 0x0c0c0703u) | __builtin_amdgcn_perm(l0, l1, 0x07030c0cu);  // L3 L2 L1 L0
  const uint32_t e1 = __builtin_amdgcn_alignbyte(tlo, xd, 3);                                                    // X T0 T1 T2
  const uint32_t e2 = __builtin_amdgcn_alignbyte(thi, tlo, 3);                                                   // T3 .. T6
  const uint32_t e3 = __builtin_amdgcn_perm(thi, thi, 0x07070707u);                                              // T7 x 4
  const uint32_t lf0 = __builtin_amdgcn_perm(e0, e0, 0x02010000u), lf1 = __builtin_amdgcn_alignbyte(e1, e0, 3);
  const uint32_t lf2 = __builtin_amdgcn_alignbyte(e2, e1, 3), lf3 = __builtin_amdgcn_alignbyte(e3, e2, 3);
  const uint32_t rt0 = __builtin_amdgcn_alignbyte(e1, e0, 1), rt1 = __builtin_amdgcn_alignbyte(e2, e1, 1);
  const uint32_t rt2 = __builtin_amdgcn_alignbyte(e3, e2, 1);
  constexpr uint32_t UP = 0x01010101u;
  auto a3 = [](uint32_t l, uint32_t c, uint32_t r) { return __builtin_amdgcn_lerp(__builtin_amdgcn_lerp(l, r, 0u), c, UP); };
  const uint32_t dc = (__builtin_amdgcn_sad_u8(tlo, 0u, __builtin_amdgcn_sad_u8(e0, 0u, 4u)) >> 3) * UP;
  // TM: clip(L[rr] - X + T[x]) on 16-bit pairs
  const int base = (int)(ld >> 24) - (int)(xd >> 24);
  const wg::s16x2_t b2 = {(short)base, (short)base};
  wg::s16x2_t tl = __builtin_bit_cast(wg::s16x2_t, __builtin_amdgcn_perm(0u, tlo, 0x0c010c00u)) + b2;
  wg::s16x2_t th = __builtin_bit_cast(wg::s16x2_t, __builtin_amdgcn_perm(0u, tlo, 0x0c030c02u)) + b2;
  const wg::s16x2_t z = {0, 0}, m = {255, 255};
  tl = __builtin_elementwise_min(__builtin_elementwise_max(tl, z), m);
  th = __builtin_elementwise_min(__builtin_elementwise_max(th, z), m);
  const uint32_t tm = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, th), __builtin_bit_cast(uint32_t, tl), 0x06040200u);
  uint4* pv = reinterpret_cast<uint4*>(pool);
  pv[0] = make_uint4(a3(lf0, e0, rt0), a3(lf1, e1, rt1), a3(lf2, e2, rt2), a3(lf3, e3, e3));
  pv[1] = make_uint4(__builtin_amdgcn_lerp(e0, rt0, UP), __builtin_amdgcn_lerp(e1, rt1, UP), __builtin_amdgcn_lerp(e2, rt2, UP), e0);
  pv[2] = make_uint4(dc, tm, 0u, 0u);
  const uint8_t* pb = reinterpret_cast<const uint8_t*>(pool);
  return (uint32_t)pb[cw & 0xff] | (uint32_t)pb[(cw >> 8) & 0xff] << 8 | (uint32_t)pb[(cw >> 16) & 0xff] << 16 |
         (uint32_t)pb[cw >> 24] << 24;
}

// ---------------------------------------------------------------------------
// k_decode_split: the same work as k_decode_bands with reconstruction and loop
// filtering on two waves per macroblock row.  Intra prediction reads
// UNFILTERED pixels (the top context is saved before filtering,
// decode_frame.go:190-194), so the reconstruction chain never waits for the
// filter: a workgroup takes a band of SW rows with a reconstruction wave (R)
// and a filter wave (F) per row.
//   R(y) walks row y: it waits for R(y-1) to have finished MB x (x + 1 when
//     this MB's I4 blocks on the right column read the top-right pixels:
//     modes VE / LD / VL), reconstructs, hands the unfiltered top context to
//     R(y+1) (LDS ring, or the global top records across bands) and the
//     unfiltered MB (+ its filter parameters) to F(y) through an LDS ring.
//   F(y) takes MB x from that ring, waits for F(y-1) to have finished MB
//     x + 1 (its top-edge filter writes the rows above, which are final only
//     once the MB above-right has run its left-edge filter), filters and
//     stores exactly as k_decode_bands does.
// The reconstruction chain -- the critical path of one image -- is then the
// loads, prediction and residuals alone, and its slope is one MB per row
// wherever the MB above-right is not needed.  Cross-band hand-off: R by
// progress_r + the top records, F by progress_f + the frame rows (sc1 stores,
// drained before the flag), as in k_decode_bands.
constexpr int SW = 4;  // rows per band (one R and one F wave each; round 6, C3 real: 2 / 4 / 8 -> 3.96 / 3.72-3.75 / 4.67-4.68 ms)
constexpr int RING_M = 4; // R -> F ring depth (R's work buffers of unfiltered MBs; round 6, C3 real: 8 -> 3.43-3.46 ms against 3.42-3.43)

// The first I4 wavefront step (i4_schedule) that reads the MB above-right,
// or 99: blocks 3, 7, 11, 15 read it in VE4 / LD4 / VL4 (wg_dsp.h pred4_row).
__device__ __forceinline__ int top_right_step(uint32_t is_i4, uint32_t right_modes, uint64_t sched) {
  // right_modes: the modes of blocks 3, 7, 11, 15, one byte each
  if (!is_i4) return 99;
  int st = 99;
#pragma unroll
  for (int k = 3; k >= 0; k--) {
    const uint32_t m = (right_modes >> (8 * k)) & 0xff;
    if (m == 2 || m == 6 || m == 7) st = (int)(sched >> (4 * (3 + 4 * k))) & 15;
  }
  return st;
}

__global__ __launch_bounds__(128 * SW) void k_decode_split(DecArgs a) {
  // R reconstructs MB x in wb_all[row][x % RING_M]; F filters it from there
  __shared__ __attribute__((aligned(16))) uint8_t wb_all[SW][RING_M][WB_SIZE];
  __shared__ __attribute__((aligned(16))) int4 stage_all[SW][50];
  constexpr int FT_BYTES = 20 * FY_STRIDE + 2 * 12 * FC_STRIDE + 8 * FC_STRIDE;
  __shared__ __attribute__((aligned(16))) uint8_t ftiles_all[SW][FT_BYTES];
  __shared__ __attribute__((aligned(16))) uint8_t top_ring[SW][RING][TOP_BYTES];
  __shared__ __attribute__((aligned(16))) uint8_t bot_ring[SW][RING][BOT_BYTES];
  __shared__ __attribute__((aligned(16))) uint8_t info_ring[SW][RING_M][32];  // each MB's wg_mb_info, R -> F
  // prog_f: MBs F finished; bot_f: MBs whose final bottom rows are in bot_ring
  // (MB x's once MB x + 1's left-edge filter, in its row pass, has run)
  __shared__ int prog_r[SW], prog_f[SW], cons_f[SW], bot_f[SW];
  // tprog: 4 x (MBs done) + (blocks of the current MB done) of the luma
  // bottom row in top_ring: block 12 + k's last row (px 4k..4k+3 of row 15)
  // is final at block 12 + k's I4 step (i4_schedule).  R(y+1) waits on it for its top-right (block
  // 12 of MB x + 1 above) instead of on the whole MB.  (Waiting block by
  // block for the top row as well measured slower: C3 4.19 -> 4.34 ms.)
  __shared__ int tprog[SW];
  __shared__ int sh_word;
  __shared__ __attribute__((aligned(16))) uint32_t i4pool[SW][64][12];  // pred4_row_tab's per-lane pools
  __shared__ uint32_t i4code[40];

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool is_f = wave >= SW;
  const int r = is_f ? wave - SW : wave;  // row of the band
  int lane = threadIdx.x & 63;
  const int mbw = a.mbw, mbh = a.mbh;
  const int bands = (mbh + SW - 1) / SW;
  const int total = a.n_img * bands;
  const int ys = 16 * mbw, uvs = 8 * mbw;
  const bool luma_only = a.filter_type == 1;
  int* const progress_f = a.progress + (int64_t)a.n_img * mbh;
  // (WG_BOUNDS) the buffers' extents from wg_decode_frames' shapes
  [[maybe_unused]] const int64_t n_mb = (int64_t)a.n_img * mbh * mbw, top_size = n_mb / mbh * TOP_BYTES,
                                 bot_size = n_mb / mbh * BOT_BYTES, prog_size = 8ll * a.n_img * mbh,
                                 y_size = n_mb * 256, uv_size = n_mb * 64;
  STAMP_DECL;
  for (int i = threadIdx.x; i < 40; i += blockDim.x) i4code[i] = kI4Code[i];  // (ordered by the loop's barrier)

  for (;;) {
    if (threadIdx.x == 0) sh_word = __hip_atomic_fetch_add(&a.ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) {
      if (is_f) {
        prog_f[r] = 0;
        cons_f[r] = 0;
        bot_f[r] = 0;
      } else {
        prog_r[r] = 0;
        tprog[r] = 0;
      }
    }
    __syncthreads();
    const int idx = __builtin_amdgcn_readfirstlane(sh_word);
    __syncthreads();
    if (idx >= total) break;
    const int band = idx / a.n_img, img = idx % a.n_img;
    const int mby = band * SW + r;
    const int last_row = min(SW, mbh - band * SW) - 1;
    const bool from_lds = r > 0, to_lds = r < last_row;
    uint8_t* top = a.top + (int64_t)img * mbw * TOP_BYTES;
    if (r <= last_row && !is_f) {
      // ============================ R: reconstruction ============================
      int16_t* const cof = reinterpret_cast<int16_t*>(stage_all[r]);
      int4* const stage = stage_all[r];
      int* prog_above = a.progress + (int64_t)img * mbh + mby - 1;
      int* prog_mine = a.progress + (int64_t)img * mbh + mby;
      int seen = 0;
      int seen_t = 0;  // lane 0 only: tprog of the row above (in the band)
      const int64_t row_mb0 = ((int64_t)img * mbh + mby) * mbw;
      int4 pf = make_int4(0, 0, 0, 0);
      if (lane < 48) {
        if (WG_IN(reinterpret_cast<const int4*>(a.coeffs + row_mb0 * 384) + lane, 16, a.coeffs, n_mb * 768, &a.ctl[1]))
          pf = ld_stream(reinterpret_cast<const int4*>(a.coeffs + row_mb0 * 384) + lane);
      } else if (lane < 50) {
        if (WG_IN(reinterpret_cast<const int4*>(a.mb + row_mb0) + lane - 48, 16, a.mb, n_mb * 32, &a.ctl[1]))
          pf = reinterpret_cast<const int4*>(a.mb + row_mb0)[lane - 48];
      }
      for (int mbx = 0; mbx < mbw; mbx++) {
        const int64_t mbi = row_mb0 + mbx;
        const int slot = mbx & (RING - 1), mslot = mbx & (RING_M - 1);
        STAMP(0);
        lane = opaque_lane() & 63;
        if (lane < 50) stage[lane] = pf;
        // the MB's wg_mb_info words straight from the prefetch registers
        // (lanes 48, 49), not back from LDS: nz masks, modes, flags
        const uint32_t nz_y = (uint32_t)__builtin_amdgcn_readlane(pf.x, 48);
        const uint32_t nz_uv = (uint32_t)__builtin_amdgcn_readlane(pf.y, 48);
        const uint32_t im0 = (uint32_t)__builtin_amdgcn_readlane(pf.z, 48);
        const uint32_t im1 = (uint32_t)__builtin_amdgcn_readlane(pf.w, 48);
        const uint32_t im2 = (uint32_t)__builtin_amdgcn_readlane(pf.x, 49);
        const uint32_t im3 = (uint32_t)__builtin_amdgcn_readlane(pf.y, 49);
        const uint32_t w6 = (uint32_t)__builtin_amdgcn_readlane(pf.z, 49);
        lds_sync();
        // the residuals need this MB's coefficients only: made here, before
        // the waits for the row above, off the wavefront's chain
        int lres[4], cres[4] = {0, 0, 0, 0};
        {
          const int blk = lane >> 2, rr = lane & 3;
          dec_residual_row(cof + blk * 16, (nz_y >> (30 - 2 * blk)) & 3, rr, lres);
          if (lane < 32) {
            const int pl = lane >> 4, cblk = (lane >> 2) & 3;
            const uint32_t bits = nz_uv >> (8 * pl);
            const int16_t* bco = cof + (16 + 4 * pl + cblk) * 16;
            if (bits & 0xff) {
              if (bits & 0xaa) dec_residual_row(bco, 3, rr, cres);
              else if (bco[0] != 0) dec_residual_row(bco, 1, rr, cres);
            }
          }
        }
        const uint8_t* imodes = reinterpret_cast<const uint8_t*>(stage + 48) + 8;
        // the step before which R waits for MB x + 1 above (its bottom row is
        // the top-right context); 99: never
        const uint64_t sched = i4_schedule(im0, im1, im2, im3);
        const int tr_step =
            mby > 0 && mbx + 1 < mbw
                ? top_right_step(w6 & 0xff, (im0 >> 24) | (im1 >> 24) << 8 | (im2 >> 24) << 16 | (im3 >> 24) << 24,
                                 sched)
                : 99;
        // ---- dependency on the row above; ring space below (top ring) and in F's ring ----
        // The whole MB x above: through prog_r in the band, through the row
        // above's progress word (its top record) across bands.  Only the
        // top-right wait of an I4 block (tr_step below) goes block by block
        // (tprog).
        if (mby > 0) {
          const int need = mbx + 1;
          if (seen < need) {
            int v = 0;
            if (lane == 0)
              v = from_lds ? wait_progress<false>(&prog_r[r - 1], need, &a.ctl[1], mbw, a.diag)
                           : wait_progress<true>(prog_above, need, &a.ctl[1], mbw, a.diag);
            seen = __shfl(v, 0, 64);
          }
        }
        if (lane == 0) {
          if (to_lds && mbx >= RING - 1) wait_progress<false>(&prog_r[r + 1], mbx - RING + 2, &a.ctl[1], mbw, a.diag);
          if (mbx >= RING_M) wait_progress<false>(&cons_f[r], mbx - RING_M + 1, &a.ctl[1], mbw, a.diag);
        }
        // ---- this MB's work buffer: left context from the previous MB's (:118-126), or the row start (:93-110) ----
        uint8_t* const wb = wb_all[r][mslot];
        // (left context and, in the band, top context and F's info record:
        // every read first, then the writes -- one LDS round trip)
        const bool l_lane = lane < 35, t_lane = from_lds && lane >= 48 && lane < 52;  // (U, V: before the chroma)
        // left: lanes 0-15 / 16-23 / 24-31 the Y / U / V column, 32-34 the
        // top-left corners, one byte a lane with select-computed addresses
        const int l_pl = lane < 16 ? 0 : (lane < 24 ? 1 : (lane < 32 ? 2 : lane - 32));
        const int l_row = lane < 16 ? lane : (lane < 24 ? lane - 16 : (lane < 32 ? lane - 24 : -1));
        const int l_o = (l_pl == 0 ? LY : (l_pl == 1 ? LU : LV)) + l_row * WG_BPS;
        // top (unfiltered): lanes 48-51 Y 0..7 / Y 8..15 / U / V
        const int t_k = lane - 48;
        uint8_t* const t_dst = t_k < 2 ? wb + LY - WG_BPS + 8 * t_k : (t_k == 2 ? wb + LU - WG_BPS : wb + LV - WG_BPS);
        uint8_t lv = l_row < 0 && mby == 0 ? 127 : 129;
        uint64_t tv = 0;
        if (l_lane && mbx > 0) lv = wb_all[r][(mbx - 1) & (RING_M - 1)][l_o + (l_pl ? 7 : 15)];
        if (t_lane) tv = lds64(top_ring[r - 1][slot] + 8 * t_k);
        if (l_lane) wb[l_o - 1] = lv;
        if (t_lane) *reinterpret_cast<uint64_t*>(t_dst) = tv;
        if (lane >= 48 && lane < 50) *reinterpret_cast<int4*>(info_ring[r][mslot] + 16 * (lane - 48)) = pf;
        if (from_lds && mbx == mbw - 1) {
          // the top-right of the row's last MB repeats its top[15] (the
          // others' comes in the I4 steps, once MB x + 1 above has it)
          const uint32_t t15 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(tv >> 32), 49) >> 24;
          if (lane == 0) *reinterpret_cast<uint32_t*>(wb + LY - WG_BPS + 16) = 0x01010101u * t15;
        }
        STAMP(1);
        // ---- top context across bands / on the first row ----
        if (!from_lds && mby > 0) {
          const uint8_t* tc = top + mbx * TOP_BYTES;
          if (lane >= 48 && lane < 52) {
            const uint64_t w = WG_IN(tc + 8 * (lane - 48), 8, a.top, top_size, &a.ctl[1]) ? ld_sc1_64(tc + 8 * (lane - 48)) : 0;
            const int k = lane - 48;
            uint8_t* dst = k < 2 ? wb + LY - WG_BPS + 8 * k : (k == 2 ? wb + LU - WG_BPS : wb + LV - WG_BPS);
            *reinterpret_cast<uint64_t*>(dst) = w;
          }
          if (lane == 0) {
            uint32_t tr;
            if (mbx < mbw - 1) tr = WG_IN(tc + TOP_BYTES, 8, a.top, top_size, &a.ctl[1]) ? (uint32_t)ld_sc1_64(tc + TOP_BYTES) : 0u;
            else tr = 0x01010101u * (uint32_t)((WG_IN(tc + 8, 8, a.top, top_size, &a.ctl[1]) ? ld_sc1_64(tc + 8) : 0ull) >> 56);
            *reinterpret_cast<uint32_t*>(wb + LY - WG_BPS + 16) = tr;
          }
        } else if (mby == 0) {
          if (lane < 21) wb[LY - WG_BPS + lane - 1] = 127;
          else if (lane < 30) wb[LU - WG_BPS + lane - 22] = 127;
          else if (lane < 39) wb[LV - WG_BPS + lane - 31] = 127;
        }
        lds_sync();
        if (mbx + 1 < mbw) {  // prefetch the next MB
          if (lane < 48) {
            if (WG_IN(reinterpret_cast<const int4*>(a.coeffs + (mbi + 1) * 384) + lane, 16, a.coeffs, n_mb * 768, &a.ctl[1]))
              pf = ld_stream(reinterpret_cast<const int4*>(a.coeffs + (mbi + 1) * 384) + lane);
          } else if (lane < 50) {
            if (WG_IN(reinterpret_cast<const int4*>(a.mb + mbi + 1) + lane - 48, 16, a.mb, n_mb * 32, &a.ctl[1]))
              pf = reinterpret_cast<const int4*>(a.mb + mbi + 1)[lane - 48];
          }
        }
        const int is_i4 = w6 & 0xff, uv_mode = (w6 >> 8) & 0xff;
        // replicate the top-right down to rows 3, 7, 11 (:155-160) where it is
        // known already: the first row (127) and a row's last MB (its top[15]);
        // elsewhere it comes at tr_step, or no block reads it
        if (is_i4 && tr_step == 99 && (mby == 0 || mbx == mbw - 1) && lane < 12) {
          const int rr = 4 * (lane / 4 + 1) - 1, i = lane & 3;
          wb[LY + rr * WG_BPS + 16 + i] = wb[LY - WG_BPS + 16 + i];
        }
        lds_sync();
        STAMP(2);
        lane = opaque_lane() & 63;
        // ---- luma prediction + residual ----
        {
          const int blk = lane >> 2, rr = lane & 3, bx = blk & 3, by = blk >> 2;
          const int off = LY + (4 * by + rr) * WG_BPS + 4 * bx;
          const int* const res = lres;
          // the last rows of blocks 12..15 (row 15) are the next row's top
          // context: in the band each goes to R(y+1) as soon as it is made
          const bool top_lane = to_lds && by == 3 && rr == 3;
          if (!is_i4) {
            const int mode = check_mode(mbx, mby, im0 & 0xff);
            const int dc = predsq_dc(mode, wb + LY, 16);
            const uint32_t pred = predsq_row4(mode, wb + LY, 4 * bx, 4 * by + rr, dc);
            const uint32_t row = pack4(clip8(byte_of(pred, 0) + res[0]), clip8(byte_of(pred, 1) + res[1]),
                                       clip8(byte_of(pred, 2) + res[2]), clip8(byte_of(pred, 3) + res[3]));
            *reinterpret_cast<uint32_t*>(wb + off) = row;
            if (top_lane) {
              *reinterpret_cast<uint32_t*>(top_ring[r][slot] + 4 * bx) = row;
              asm volatile("" ::: "memory");  // (one wave's DS ops complete in order)
              // (a workgroup-scope release: the top-ring row is visible to R(y+1)
              // before the count that announces it, by the memory model, not
              // only by the LDS unit's in-order execution)
              if (bx == 3) __hip_atomic_store(&tprog[r], 4 * mbx + 4, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
          } else {
            const int my_step = (int)(sched >> (4 * blk)) & 15;
            const int n_steps = (int)(sched >> 60) + 1;  // block 15 is last
            const uint32_t cw = i4code[4 * imodes[blk] + rr];  // (pred4_row_tab's code word)
            for (int st = 0; st < n_steps; st++) {
              if (st == tr_step) {
                // the first block that reads the top-right: only now wait for
                // MB x + 1 above (in the band: its block 12 only), then its
                // bottom row's first 4 px, copied beside rows 3, 7, 11 as well
                int v = 0;
                if (lane == 0) {
                  uint32_t tr;
                  if (from_lds) {
                    const int need = 4 * (mbx + 1) + 1;
                    if (seen_t < need) seen_t = wait_progress<false>(&tprog[r - 1], need, &a.ctl[1], 4 * mbw + 8, a.diag);
                    tr = lds32(top_ring[r - 1][(mbx + 1) & (RING - 1)]);
                    v = seen;  // (unused in the band)
                  } else {
                    v = seen < mbx + 2 ? wait_progress<true>(prog_above, mbx + 2, &a.ctl[1], mbw, a.diag) : seen;
                    tr = WG_IN(top + (mbx + 1) * TOP_BYTES, 8, a.top, top_size, &a.ctl[1])
                             ? (uint32_t)ld_sc1_64(top + (mbx + 1) * TOP_BYTES) : 0u;
                  }
#pragma unroll
                  for (int k = 0; k < 4; k++) *reinterpret_cast<uint32_t*>(wb + LY + (4 * k - 1) * WG_BPS + 16) = tr;
                }
                seen = __shfl(v, 0, 64);
                lds_sync();
              }
              if (st == my_step) {
                const uint32_t pred = pred4_row_tab(wb, LY + 4 * by * WG_BPS + 4 * bx, rr, cw, i4pool[r][lane]);
                const uint32_t row = pack4(clip8(byte_of(pred, 0) + res[0]), clip8(byte_of(pred, 1) + res[1]),
                                           clip8(byte_of(pred, 2) + res[2]), clip8(byte_of(pred, 3) + res[3]));
                *reinterpret_cast<uint32_t*>(wb + off) = row;
                if (top_lane) {  // (blocks 12..15 run in order, one a step or more apart)
                  *reinterpret_cast<uint32_t*>(top_ring[r][slot] + 4 * bx) = row;
                  asm volatile("" ::: "memory");
                  __hip_atomic_store(&tprog[r], 4 * mbx + bx + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
              }
              lds_sync();
            }
          }
        }
        STAMP(3);
        lane = opaque_lane() & 63;
        // ---- chroma prediction + residual (doUVTransform :47-68) ----
        if (lane < 32) {
          const int pl = lane >> 4, cblk = (lane >> 2) & 3, rr = lane & 3;
          const int cbx = cblk & 1, cby = cblk >> 1;
          const int base = pl ? LV : LU;
          const int mode = check_mode(mbx, mby, uv_mode);
          const int dc = predsq_dc(mode, wb + base, 8);
          const uint32_t pred = predsq_row4(mode, wb + base, 4 * cbx, 4 * cby + rr, dc);
          const int* const res = cres;
          const uint32_t crow = pack4(clip8(byte_of(pred, 0) + res[0]), clip8(byte_of(pred, 1) + res[1]),
                                      clip8(byte_of(pred, 2) + res[2]), clip8(byte_of(pred, 3) + res[3]));
          *reinterpret_cast<uint32_t*>(wb + base + (4 * cby + rr) * WG_BPS + 4 * cbx) = crow;
          // the bottom row (row 7) is the next row's top context: in the band
          // straight into the top ring
          if (to_lds && cby == 1 && rr == 3) *reinterpret_cast<uint32_t*>(top_ring[r][slot] + 16 + 8 * pl + 4 * cbx) = crow;
        }
        lds_sync();
        STAMP(4);
        lane = opaque_lane() & 63;
        // ---- hand-offs: unfiltered top context for R(y+1), the MB and its info for F(y) ----
        if (!to_lds && mby < mbh - 1 && lane >= 32 && lane < 36) {  // (in the band the rows are out already)
          const int k = lane - 32;
          const uint8_t* src =
              k < 2 ? wb + LY + 15 * WG_BPS + 8 * k : (k == 2 ? wb + LU + 7 * WG_BPS : wb + LV + 7 * WG_BPS);
          if (to_lds) {
            *reinterpret_cast<uint64_t*>(top_ring[r][slot] + 8 * k) = lds64(src);
          } else if (k < 2) {  // the record as two 16-B write-through stores (Y | U V): one 32-B write
            uint4 w;
            if (k == 0) {
              w = *reinterpret_cast<const uint4*>(wb + LY + 15 * WG_BPS);
            } else {
              const uint64_t u = lds64(wb + LU + 7 * WG_BPS), v = lds64(wb + LV + 7 * WG_BPS);
              w = make_uint4((uint32_t)u, (uint32_t)(u >> 32), (uint32_t)v, (uint32_t)(v >> 32));
            }
            if (WG_IN(top + mbx * TOP_BYTES + 16 * k, 16, a.top, top_size, &a.ctl[1])) st_sc1_128(top + mbx * TOP_BYTES + 16 * k, w);
          }
        }
        lds_sync();
        STAMP(5);
        // ---- publish: LDS for F(y) and R(y+1) in the band; global for the next band ----
        if (!to_lds && mby < mbh - 1) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the top record is out before the flag
          if (lane == 0 && WG_IN(prog_mine, 4, a.progress, prog_size, &a.ctl[1]))
            __hip_atomic_store(prog_mine, mbx + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) __hip_atomic_store(&prog_r[r], mbx + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        STAMP(6);
      }
    } else if (r <= last_row) {
      // ============================ F: loop filter + frame stores ============================
      uint8_t* const fy = ftiles_all[r];
      uint8_t* const fu = fy + 20 * FY_STRIDE;
      uint8_t* const fv = fu + 12 * FC_STRIDE;
      int* prog_above = progress_f + (int64_t)img * mbh + mby - 1;
      int* prog_mine = progress_f + (int64_t)img * mbh + mby;
      uint8_t* const bot_img = a.bot + (int64_t)img * mbw * BOT_BYTES;
      const bool hand = !to_lds && mby < mbh - 1;  // a band's last row with a band below
      uint8_t* Yp = a.Y + (int64_t)img * ys * 16 * mbh;
      uint8_t* Up = a.U + (int64_t)img * uvs * 8 * mbh;
      uint8_t* Vp = a.V + (int64_t)img * uvs * 8 * mbh;
      int seen = 0, have = 0;
      for (int mbx = 0; mbx < mbw; mbx++) {
        const int slot = mbx & (RING - 1), mslot = mbx & (RING_M - 1);
        STAMP(0);
        lane = opaque_lane() & 63;
        // ---- this row's MB from R, ring space below (the row above: before the column pass) ----
        if (lane == 0) {
          if (have < mbx + 1) have = wait_progress<false>(&prog_r[r], mbx + 1, &a.ctl[1], mbw, a.diag);
          if (to_lds && mbx >= RING - 1) wait_progress<false>(&prog_f[r + 1], mbx - RING + 2, &a.ctl[1], mbw, a.diag);
        }
        lds_sync();
        STAMP(7);
        // rotate the filter tiles (the MBs to the left move one MB further
        // left), then the MB into the tiles (rows 4..): every read of both
        // first, then the writes (one LDS round trip; the rotation reads the
        // columns the copy-in and the rotation itself overwrite, so all reads
        // precede all writes)
        const bool rot = mbx > 0;
        uint4 y0 = make_uint4(0, 0, 0, 0);
        uint64_t c[2] = {0, 0};
        if (rot) {
          if (lane < 40) y0 = *reinterpret_cast<const uint4*>(fy + (lane >> 1) * FY_STRIDE + FY_X0 - 16 + 16 * (lane & 1));
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const int i = lane + 64 * h;
            if (i < 96) {
              const int row = i >> 2, pl = row >= 12;
              c[h] = lds64((pl ? fv : fu) + (row - 12 * pl) * FC_STRIDE + FC_X0 - 24 + 8 * (i & 3));
            }
          }
        }
        const uint8_t* ms = wb_all[r][mslot];
        const bool y_lane = lane < 16, c_lane = lane >= 16 && lane < 32;
        const int c_pl = lane >= 24, c_j = (lane - 16) & 7;
        uint4 yv = make_uint4(0, 0, 0, 0);
        uint64_t cv = 0;
        if (y_lane) yv = *reinterpret_cast<const uint4*>(ms + LY + lane * WG_BPS);
        if (c_lane) cv = lds64(ms + (c_pl ? LV : LU) + c_j * WG_BPS);
        const uint32_t w7v = reinterpret_cast<const uint32_t*>(info_ring[r][mslot])[7];
        asm volatile("" ::: "memory");  // (reads above, writes below)
        if (rot) {
          if (lane < 40) *reinterpret_cast<uint4*>(fy + (lane >> 1) * FY_STRIDE + FY_X0 - 32 + 16 * (lane & 1)) = y0;
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const int i = lane + 64 * h;
            if (i < 96) {
              const int row = i >> 2, pl = row >= 12;
              *reinterpret_cast<uint64_t*>((pl ? fv : fu) + (row - 12 * pl) * FC_STRIDE + FC_X0 - 32 + 8 * (i & 3)) = c[h];
            }
          }
        }
        if (y_lane) *reinterpret_cast<uint4*>(fy + (lane + 4) * FY_STRIDE + FY_X0) = yv;
        if (c_lane) *reinterpret_cast<uint64_t*>((c_pl ? fv : fu) + (c_j + 4) * FC_STRIDE + FC_X0) = cv;
        const uint32_t w7 = __builtin_amdgcn_readfirstlane(w7v);
        lds_sync();
        if (lane == 0) __hip_atomic_store(&cons_f[r], mbx + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int f_limit = w7 & 0xff, ilevel = (w7 >> 8) & 0xff, f_inner = (w7 >> 16) & 0xff, hev_t = w7 >> 24;
        STAMP(8);
        lane = opaque_lane() & 63;
        // ---- loop filter (doFilter :293-342) ----
        const bool do_filter = a.filter_type > 0 && f_limit > 0;
        const bool inner = f_inner != 0;
        if (do_filter) {
          if (a.filter_type == 2) filter_mb_rows<true>(fy, fu, fv, lane, true, mbx > 0, inner, f_limit, ilevel, hev_t);
          else filter_mb_rows<false>(fy, fu, fv, lane, false, mbx > 0, inner, f_limit, ilevel, hev_t);
        }
        if (to_lds && mbx > 0) {
          // the left MB's bottom rows are final now (our left-edge filter was
          // the last to touch them): its columns 12..15 into its bot_ring slot
          // (lanes 16-19 Y rows 12..15, 20-27 U / V rows 4..7; addresses by
          // selects: one LDS read + write)
          if (do_filter && lane >= 16 && lane < (luma_only ? 20 : 28)) {
            uint8_t* bl = bot_ring[r][(mbx - 1) & (RING - 1)];
            const int k = lane - 16, pl = k >= 8, rr = k & 3;
            const int dst = k < 4 ? 16 * k + 12 : 64 + 32 * pl + 8 * rr + 4;
            const uint8_t* src = k < 4 ? fy + (16 + k) * FY_STRIDE + FY_X0 - 4 : (pl ? fv : fu) + (8 + rr) * FC_STRIDE + FC_X0 - 4;
            *reinterpret_cast<uint32_t*>(bl + dst) = lds32(src);
          }
          lds_sync();
          if (lane == 0) __hip_atomic_store(&bot_f[r], mbx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        // ---- the row above: only now (round 6) ----
        // The rotation, the copy-in and the row pass touch this row's tile
        // rows 4.. and the MBs to the left; the column pass (the top edge)
        // and the stores of the rows above need the row above's MB x final:
        // in the band its bottom rows (bot_f, published once MB x + 1 above
        // has run its row pass); across bands the frame rows, final once the
        // row above has finished MB x + 1.  Waiting here instead of before
        // the tiles takes the copy-in and the row pass off the rows' chain
        // (C3 real 3.66-3.67 -> 3.42 ms).  They go into the tile rows 0..3
        // from bot_ring / the cross-band record (same layout): lanes 52-59 Y
        // rows 0..3 in 8-B halves, 60-63 U, 44-47 V.
        if (mby > 0) {
          if (lane == 0) {
            const int need = from_lds ? mbx + 1 : min(mbx + 2, mbw);
            if (seen < need)
              seen = from_lds ? wait_progress<false>(&bot_f[r - 1], need, &a.ctl[1], mbw, a.diag)
                              : wait_progress<true>(prog_above, need, &a.ctl[1], mbw, a.diag);
          }
          lds_sync();
          const int bk = lane - 52;
          const int b_src = lane >= 60 ? 64 + 8 * (lane - 60) : (lane >= 52 ? 16 * (bk >> 1) + 8 * (bk & 1) : 96 + 8 * (lane - 44));
          uint8_t* const b_dst = lane >= 60 ? fu + (lane - 60) * FC_STRIDE + FC_X0
                                            : (lane >= 52 ? fy + (bk >> 1) * FY_STRIDE + FY_X0 + 8 * (bk & 1)
                                                          : fv + (lane - 44) * FC_STRIDE + FC_X0);
          if (lane >= 52 || (lane >= 44 && lane < 48)) {
            const uint64_t bv = from_lds ? lds64(bot_ring[r - 1][slot] + b_src)
                                         : (WG_IN(bot_img + mbx * BOT_BYTES + b_src, 8, a.bot, bot_size, &a.ctl[1])
                                                ? ld_sc1_64(bot_img + mbx * BOT_BYTES + b_src) : 0ull);
            *reinterpret_cast<uint64_t*>(b_dst) = bv;
          }
          lds_sync();
        }
        if (do_filter) {
          if (a.filter_type == 2) filter_mb_cols<true>(fy, fu, fv, lane, true, mby > 0, inner, f_limit, ilevel, hev_t);
          else filter_mb_cols<false>(fy, fu, fv, lane, false, mby > 0, inner, f_limit, ilevel, hev_t);
        }
        STAMP(9);
        lane = opaque_lane() & 63;
        // ---- stores ----
        // A band's last row first hands the next band MB x - 1's bottom rows
        // 12..15 (final after this MB's left-edge filter; at the row's end this
        // MB's too) as one 128-B write-through record per MB, and publishes.
        // Every frame byte is then stored once, by the wave that finalises
        // it, with plain (write-back) stores that L2 merges into whole lines:
        // rows 13..15 are the next band's to store after its top-edge filter.
        if (hand) {
          const int which = lane >> 3, k = lane & 7, x = mbx - 1 + which;
          if (lane < 16 && (which == 0 ? mbx > 0 : mbx == mbw - 1)) {
            uint4 w;
            if (k < 4) {
              w = *reinterpret_cast<const uint4*>(fy + (16 + k) * FY_STRIDE + FY_X0 + 16 * (x - mbx));
            } else {  // U rows 4,5 | 6,7, V rows 4,5 | 6,7
              const uint8_t* src = ((k >= 6) ? fv : fu) + (8 + 2 * (k & 1)) * FC_STRIDE + FC_X0 + 8 * (x - mbx);
              const uint64_t a0 = lds64(src), a1 = lds64(src + FC_STRIDE);
              w = make_uint4((uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1, (uint32_t)(a1 >> 32));
            }
            if (WG_IN(bot_img + x * BOT_BYTES + 16 * k, 16, a.bot, bot_size, &a.ctl[1])) st_sc1_128(bot_img + x * BOT_BYTES + 16 * k, w);
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the record is out before the flag
          if (lane == 0 && WG_IN(prog_mine, 4, a.progress, prog_size, &a.ctl[1]))
            __hip_atomic_store(prog_mine, mbx + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        {
          const bool last = mbx == mbw - 1;
          int y0 = -1, y1 = -1;
          if (last) {
            y0 = mbx > 0 ? (mbx - 1) & ~1 : 0;
            y1 = mbx;
          } else if (mbx >= 2 && (mbx & 1) == 0) {
            y0 = mbx - 2;
            y1 = mbx - 1;
          }
          int c0 = -1, c1 = -1;
          if (last) {
            c0 = mbx > 0 ? (mbx - 1) & ~3 : 0;
            c1 = mbx;
          } else if (mbx >= 4 && (mbx & 3) == 0) {
            c0 = mbx - 4;
            c1 = mbx - 1;
          }
          // rows below ylim / clim are this wave's; the rest the row below
          // stores (the image's last row stores all; with the simple filter
          // chroma is never filtered, so its rows are all this wave's)
          const int ylim = to_lds || hand ? 13 : 16, clim = to_lds || (hand && !luma_only) ? 5 : 8;
          int t0 = -1, t1 = -1, u0 = -1, u1 = -1;
          if (mby > 0) {
            if ((mbx & 1) == 1 || last) {
              t0 = mbx & ~1;
              t1 = mbx;
            }
            if ((mbx & 3) == 3 || last) {
              u0 = mbx & ~3;
              u1 = mbx;
            }
          }
          // every piece's LDS read first, then the stores (one LDS round trip):
          //   ym: Y rows of MBs y0..y1 (lane = 16 MB + row)
          //   cm0 / cm1: U / V rows of MBs c0..c1 (i = lane, lane + 64)
          //   yt / ct: the rows above this row's top-edge filter rewrote
          //     (Y rows 13..15 of MBs t0..t1: lanes 0-5; U / V rows 5..7 of
          //     MBs u0..u1: lanes 8-31)
          //   bb: this MB's bottom rows for the row below (bot_ring)
          const int yj = lane & 15, yx = y0 + (lane >> 4);
          const bool sy = lane < 48 && y0 >= 0 && yj < ylim && yx <= y1;
          const int ci0 = lane, ci1 = lane + 64;
          const int cx0 = c0 + (ci0 >> 4), cx1 = c0 + (ci1 >> 4);
          const bool sc0 = c0 >= 0 && (ci0 & 7) < clim && cx0 <= c1;
          const bool sc1 = c0 >= 0 && ci1 < 80 && (ci1 & 7) < clim && cx1 <= c1;
          const int tr_ = 1 + (lane >> 1), tx = t0 + (lane & 1);
          const bool syt = lane < 6 && t0 >= 0 && tx <= t1;
          const int ck = lane - 8, cpl = ck >= 12, crr = 1 + (ck % 12) / 4, cx = u0 + (ck & 3);
          const bool sct = (from_lds || !luma_only) && lane >= 8 && lane < 32 && u0 >= 0 && cx <= u1;
          const bool sb = to_lds && lane < 16;
          const int bpl = lane >= 12, brr = lane & 3;
          uint4 ym = make_uint4(0, 0, 0, 0), yt = make_uint4(0, 0, 0, 0);
          uint64_t cm0 = 0, cm1 = 0, ct = 0, bb = 0;
          if (sy) ym = *reinterpret_cast<const uint4*>(fy + (yj + 4) * FY_STRIDE + FY_X0 + 16 * (yx - mbx));
          if (sc0) cm0 = lds64(((ci0 >> 3) & 1 ? fv : fu) + ((ci0 & 7) + 4) * FC_STRIDE + FC_X0 + 8 * (cx0 - mbx));
          if (sc1) cm1 = lds64(((ci1 >> 3) & 1 ? fv : fu) + ((ci1 & 7) + 4) * FC_STRIDE + FC_X0 + 8 * (cx1 - mbx));
          if (syt) yt = *reinterpret_cast<const uint4*>(fy + tr_ * FY_STRIDE + FY_X0 + 16 * (tx - mbx));
          if (sct) ct = lds64((cpl ? fv : fu) + crr * FC_STRIDE + FC_X0 + 8 * (cx - mbx));
          if (sb)
            bb = lds64(lane < 8 ? fy + (16 + (lane >> 1)) * FY_STRIDE + FY_X0 + 8 * (lane & 1)
                                : (bpl ? fv : fu) + (8 + brr) * FC_STRIDE + FC_X0);
#define DEC_ST(cond, T, p, v, base, size) \
  if (cond) {                               \
    uint8_t* const q_ = (p);                \
    if (WG_IN(q_, (int)sizeof(T), (base), (size), &a.ctl[1])) *reinterpret_cast<T*>(q_) = (v); \
  }
          DEC_ST(sy, uint4, Yp + (int64_t)(16 * mby + yj) * ys + 16 * yx, ym, a.Y, y_size)
          DEC_ST(sc0, uint64_t, ((ci0 >> 3) & 1 ? Vp : Up) + (int64_t)(8 * mby + (ci0 & 7)) * uvs + 8 * cx0, cm0,
                 (ci0 >> 3) & 1 ? a.V : a.U, uv_size)
          DEC_ST(sc1, uint64_t, ((ci1 >> 3) & 1 ? Vp : Up) + (int64_t)(8 * mby + (ci1 & 7)) * uvs + 8 * cx1, cm1,
                 (ci1 >> 3) & 1 ? a.V : a.U, uv_size)
          DEC_ST(syt, uint4, Yp + (int64_t)(16 * mby - 4 + tr_) * ys + 16 * tx, yt, a.Y, y_size)
          DEC_ST(sct, uint64_t, (cpl ? Vp : Up) + (int64_t)(8 * mby - 4 + crr) * uvs + 8 * cx, ct, cpl ? a.V : a.U, uv_size)
#undef DEC_ST
          if (sb)
            *reinterpret_cast<uint64_t*>(bot_ring[r][slot] + (lane < 8 ? 16 * (lane >> 1) + 8 * (lane & 1) : 64 + 32 * bpl + 8 * brr)) = bb;
        }
        lds_sync();
        lane = opaque_lane() & 63;
        if (lane == 0) {
          __hip_atomic_store(&prog_f[r], mbx + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (mbx == mbw - 1) __hip_atomic_store(&bot_f[r], mbw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        STAMP(10);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // the band's LDS rings are reused by the next band
  }
  STAMP_FLUSH();
}

// launch configuration, read once per process (under the mutex: host
// threads may call wg_decode_frames concurrently)
struct DecConfig {
  int num_cus = 0;
  int rows_per_cu = 0;   // resident k_decode_bands workgroups per CU (occupancy)
  int split_per_cu = 0;  // resident k_decode_split workgroups per CU
  int max_wg = 0;        // grid cap (0: every resident slot; WG_DECODE_MAX_WG)
  int force = 0;         // WG_DECODE_KERNEL=split / bands forces one kernel (A/B); 0: by batch size
};
std::mutex g_dec_cfg_mu;
DecConfig g_dec_cfg;

int dec_config(DecConfig* out) {
  std::lock_guard<std::mutex> lock(g_dec_cfg_mu);
  DecConfig& c = g_dec_cfg;
  if (c.num_cus == 0) {
    int dev = 0, cus = 0, per_cu = 0, per_cu_s = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0 ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_decode_bands, 64 * DW, 0) != hipSuccess || per_cu <= 0 ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_s, k_decode_split, 128 * SW, 0) != hipSuccess ||
        per_cu_s <= 0)
      return wg::check_launch("decode occupancy query");
    c.rows_per_cu = per_cu;
    c.split_per_cu = per_cu_s;
    if (const char* e = getenv("WG_DECODE_WG_PER_CU")) c.rows_per_cu = atoi(e) > 0 ? atoi(e) : per_cu;  // tuning
    if (const char* e = getenv("WG_DECODE_KERNEL")) c.force = strcmp(e, "bands") == 0 ? 2 : (strcmp(e, "split") == 0 ? 1 : 0);
    if (const char* e = getenv("WG_DECODE_MAX_WG")) c.max_wg = atoi(e) > 0 ? atoi(e) : 0;  // tuning: cap the grid
    c.num_cus = cus;
  }
  *out = c;
  return WG_OK;
}

// the switch between the two kernels (see wg_decode_frames)
bool use_split(const DecConfig& cfg, int32_t mbh, int32_t n_images) {
  return cfg.force ? cfg.force == 1 : (int64_t)n_images * mbh <= (int64_t)2 * cfg.split_per_cu * cfg.num_cus * SW;
}

}  // namespace

WG_IF_STAMPS(extern "C" int wg_debug_phases(unsigned long long* host, int n) {
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * n);
  unsigned long long z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)) == hipSuccess ? 0 : -2;
})

extern "C" size_t wg_decode_work_bytes(int32_t mbw, int32_t mbh, int32_t n_images) {
  if (mbw <= 0 || mbh <= 0 || n_images <= 0) return 0;
  // top records | ctl[4] | progress (reconstruction) | progress_f (filter, k_decode_split) | bottom records (16-B aligned)
  const size_t head = (size_t)n_images * mbw * TOP_BYTES + sizeof(int) * (2 * (size_t)n_images * mbh + 4);
  return ((head + 15) & ~(size_t)15) + (size_t)n_images * mbw * BOT_BYTES;
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
  {
    const size_t head = (size_t)n_images * mbw * TOP_BYTES + sizeof(int) * (2 * (size_t)n_images * mbh + 4);
    a.bot = static_cast<uint8_t*>(work) + ((head + 15) & ~(size_t)15);
  }
  a.filter_type = filter_type;
  a.mbw = mbw;
  a.mbh = mbh;
  a.n_img = n_images;
  hipStream_t s = wg::as_stream(stream);
  a.diag = wg::diag_words(s);
  if (!a.diag) return WG_EHIP;
  a.diag += wg::DIAG_DECODE;
  DecConfig cfg;
  if (const int e = dec_config(&cfg)) return e;
  if (hipMemsetAsync(a.ctl, 0, sizeof(int) * (2 * (size_t)n_images * mbh + 4), s) != hipSuccess)
    return wg::check_launch("hipMemsetAsync(decode ctl)");
  // k_decode_split (two waves a row: reconstruction and loop filter apart)
  // shortens a row's macroblock time, which is what bounds a batch of few
  // long rows (C3's one 4096^2 image: 3.8 ms against 5.1 ms with one wave a
  // row; 16 x 4096^2: 5.0 against 8.2 ms).  A batch with many more rows than
  // the chip holds at once is bound by throughput instead, and there the
  // split kernel's second wave per row only holds wave slots -- beside the
  // encoder (the bench's pipeline), the encoder's: k_decode_bands (64 x
  // 1080p: whole-path median 6,495 -> 7,065 MPix/s, decode side alone 77.4k
  // -> 76.1k).  The switch is at twice the rows of the resident
  // split workgroups (a heuristic between those two measured points).
  if (use_split(cfg, mbh, n_images)) {
    const int bands = n_images * ((mbh + SW - 1) / SW);
    int grid = bands < cfg.split_per_cu * cfg.num_cus ? bands : cfg.split_per_cu * cfg.num_cus;
    if (cfg.max_wg > 0 && grid > cfg.max_wg) grid = cfg.max_wg;
    hipLaunchKernelGGL(k_decode_split, dim3((unsigned)grid), dim3(128 * SW), 0, s, a);
    return wg::check_launch("k_decode_split");
  }
  const int bands = n_images * ((mbh + DW - 1) / DW);
  const int grid = bands < cfg.rows_per_cu * cfg.num_cus ? bands : cfg.rows_per_cu * cfg.num_cus;
  hipLaunchKernelGGL(k_decode_bands, dim3((unsigned)grid), dim3(64 * DW), 0, s, a);
  return wg::check_launch("k_decode_bands");
}

extern "C" int wg_decode_kernel(int32_t mbh, int32_t n_images) {
  WG_REQUIRE(mbh > 0 && n_images > 0);
  DecConfig cfg;
  if (const int e = dec_config(&cfg)) return e;
  return use_split(cfg, mbh, n_images) ? 1 : 2;
}

extern "C" int wg_decode_status(const void* work, int32_t mbw, int32_t n_images, void* stream) {
  WG_REQUIRE(work && mbw > 0 && n_images > 0);
  const int* ctl =
      reinterpret_cast<const int*>(static_cast<const uint8_t*>(work) + (size_t)n_images * mbw * TOP_BYTES);
  return wg::wait_status(ctl + 1, wg::DIAG_DECODE, wg::as_stream(stream), "wg_decode_status: decode row",
                         "needed, seen, global, ticks, block, wave");
}
