// alpha.hip -- alpha-plane filters and alpha processing on gfx950
// (SURVEY.md 8(f)#4).
//
//   k_alpha_filter      alphaFilterHorizontal / Vertical / Gradient
//                       (internal/lossy/alpha.go:387-454): one thread per pixel
//   unfilters           alphaUnfilterHorizontal / Vertical / Gradient (:128-203),
//                       in place:
//     horizontal        value(y, x) = sum_{k<=y} d(k, 0) + sum_{1<=i<=x} d(y, i)
//                       (mod 256): a scan of column 0, then one wave per row
//                       scanning 64 columns at a time
//     vertical          a scan of row 0, then one thread per column walking down
//     gradient          row 0 scanned; the rows below are a 2-D recurrence
//                       (left, top, top-left, clamped): one wave per 64-row band
//                       walks it diagonally (lane k does x = s - k of row
//                       band*64 + k; the row above comes from lane k-1 by a lane
//                       shift); bands hand their last row down 64 columns at a
//                       time (plain stores, vmcnt(0) + release fence, then a
//                       relaxed progress counter)
//   k_alpha_meanwalk    estimateBestFilter (:321-385), the "none" bin: one lane per
//                       sampled row (the running mean is serial along the row)
//   k_alpha_stats       the horizontal / vertical / gradient bins and
//                       getNumColors (:302-317): one thread per 16 bytes; the
//                       4 x 16 "seen" bins are OR-ed into one 64-bit word per
//                       image, the colours into a 256-bit set
//   premultiply         ApplyAlphaMultiply, MultARGBRow, ApplyAlphaMultiply4444
//                       (internal/dsp/alpha_proc.go:13-135): one thread per pixel
//   dispatch / extract  DispatchAlpha / ExtractAlpha (:140-176) with their
//                       any-transparent / all-opaque results
// Bit-exact with oracle/alpha.c.
#include "wg_common.h"
#include "wg_instr.h"

namespace {

__device__ __forceinline__ int clip255(int v) { return min(max(v, 0), 255); }

// -------------------------------------------------------------- filters
// one thread per 16 pixels of a row: the 16 bytes, the row above's 16 and the
// byte left of each (16-B accesses when rows are 16-B aligned)
__global__ __launch_bounds__(256) void k_alpha_filter(int filter, const uint8_t* in, uint8_t* out, int w, int h,
                                                      int64_t pitch, int groups, int64_t total, int fast) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int g = (int)(i % groups);
  const int64_t ry = i / groups;
  const int y = (int)(ry % h);
  const int64_t img = ry / h;
  const int x0 = g * 16;
  const uint8_t* row = in + img * pitch + (int64_t)y * w;
  uint8_t* dst = out + img * pitch + (int64_t)y * w;
  uint8_t cur[16], up[16];
  const int n = min(16, w - x0);
  if (fast) {
    *reinterpret_cast<uint4*>(cur) = *reinterpret_cast<const uint4*>(row + x0);
    if (y > 0) *reinterpret_cast<uint4*>(up) = *reinterpret_cast<const uint4*>(row - w + x0);
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++) {
      cur[k] = k < n ? row[x0 + k] : 0;
      up[k] = (y > 0 && k < n) ? row[x0 + k - w] : 0;
    }
  }
  const int left0 = x0 > 0 ? row[x0 - 1] : 0;
  const int upleft0 = (x0 > 0 && y > 0) ? row[x0 - 1 - w] : 0;
  uint8_t res[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int x = x0 + k;
    const int v = cur[k];
    const int left = k > 0 ? cur[k - 1] : left0;
    int pred = 0;
    if (filter != 0) {
      if (y == 0) {
        pred = x > 0 ? left : 0;
      } else if (filter == 2 || x == 0) {
        pred = up[k];
      } else {
        const int ul = k > 0 ? up[k - 1] : upleft0;
        pred = filter == 1 ? left : clip255(left + up[k] - ul);
      }
    }
    res[k] = (uint8_t)(v - pred);
  }
  if (fast) {
    *reinterpret_cast<uint4*>(dst + x0) = *reinterpret_cast<const uint4*>(res);
  } else {
    for (int k = 0; k < n; k++) dst[x0 + k] = res[k];
  }
}

// inclusive scan (mod 256, carried in int) of v over the 64 lanes
__device__ __forceinline__ int wave_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// scan of n bytes at p, stride `step` (in place): one wave.  Lane k owns a
// run of ceil(n/64) consecutive elements: its run's sum (independent loads),
// an exclusive wave scan of the sums, then the run re-walked with the offset.
__device__ __forceinline__ void scan_line(uint8_t* p, int64_t step, int n, int lane) {
  const int len = (n + 63) >> 6;
  const int i0 = min(lane * len, n), i1 = min(i0 + len, n);
  int sum = 0;
  for (int i = i0; i < i1; i++) sum += p[i * step];
  int acc = wave_scan(sum, lane) - sum;
  for (int i = i0; i < i1; i++) {
    acc += p[i * step];
    p[i * step] = (uint8_t)acc;
  }
}

// one wave per (image, line): kind 0 = column 0 of the image, kind 1 = row 0
__global__ __launch_bounds__(64) void k_alpha_scan_edge(uint8_t* data, int w, int h, int64_t pitch, int kind) {
  uint8_t* img = data + (int64_t)blockIdx.x * pitch;
  if (kind == 0)
    scan_line(img, w, h, threadIdx.x);
  else
    scan_line(img, 1, w, threadIdx.x);
}

// horizontal unfilter, rows: one wave per (image, row); column 0 already holds
// its prefix, x >= 1 add the row's running sum.  Fast path (16-B rows): lane
// = 16 bytes, an in-lane prefix, then a wave scan of the lane totals.
__global__ __launch_bounds__(64) void k_alpha_hrows(uint8_t* data, int w, int h, int64_t pitch, int fast) {
  const int lane = threadIdx.x;
  const int img = blockIdx.x / h, y = blockIdx.x % h;
  uint8_t* row = data + img * pitch + (int64_t)y * w;
  if (fast) {
    int carry = 0;  // sum of the row up to the current 1 KB block (column 0's prefix included)
    for (int c0 = 0; c0 < w; c0 += 1024) {
      const int x0 = c0 + 16 * lane;
      uint8_t b[16];
      if (x0 < w) *reinterpret_cast<uint4*>(b) = *reinterpret_cast<const uint4*>(row + x0);
      int run[16], acc = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        acc += x0 < w ? b[k] : 0;
        run[k] = acc;
      }
      const int excl = wave_scan(acc, lane) - acc + carry;
#pragma unroll
      for (int k = 0; k < 16; k++) b[k] = (uint8_t)(run[k] + excl);
      if (x0 < w) *reinterpret_cast<uint4*>(row + x0) = *reinterpret_cast<const uint4*>(b);
      carry = __shfl(excl + acc, 63, 64);
    }
    return;
  }
  int carry = row[0];
  for (int c0 = 1; c0 < w; c0 += 64) {
    const int i = c0 + lane;
    const int v = i < w ? row[i] : 0;
    const int s = wave_scan(v, lane) + carry;
    if (i < w) row[i] = (uint8_t)s;
    carry = __shfl(s, 63, 64);
  }
}

// vertical unfilter below row 0: one thread per column
__global__ __launch_bounds__(256) void k_alpha_vcols(uint8_t* data, int w, int h, int64_t pitch, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t img = i / w;
  const int x = (int)(i % w);
  uint8_t* p = data + img * pitch + x;
  int acc = p[0];
  for (int y = 1; y < h; y++) {
    acc += p[(int64_t)y * w];
    p[(int64_t)y * w] = (uint8_t)acc;
  }
}

// vertical unfilter below row 0, dword columns (w % 4 == 0, aligned rows):
// a 1024-thread workgroup owns a strip of 64 dword columns; wave g walks the
// g-th of 16 row segments.  Pass 1 sums each segment (per-byte adds, mod 256,
// packed four to a dword), the segment prefixes are combined through LDS, and
// pass 2 re-walks the segment writing the running sums.
__device__ __forceinline__ uint32_t padd8(uint32_t a, uint32_t b) {
  return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ ((a ^ b) & 0x80808080u);
}

__global__ __launch_bounds__(1024) void k_alpha_vseg(uint8_t* data, int w, int h, int64_t pitch, int strips) {
  __shared__ uint32_t seg_sum[16][64];
  const int col = threadIdx.x & 63, seg = threadIdx.x >> 6;
  const int img = blockIdx.x / strips, strip = blockIdx.x % strips;
  const int wd = w >> 2;
  const int q = strip * 64 + col;
  const int n = h - 1, len = (n + 15) / 16;
  const int r0 = 1 + seg * len, r1 = min(r0 + len, h);
  uint32_t* base = reinterpret_cast<uint32_t*>(data + img * pitch) + q;
  uint32_t sum = 0;
  if (q < wd) {
#pragma unroll 8
    for (int r = r0; r < r1; r++) sum = padd8(sum, base[(int64_t)r * wd]);
  }
  seg_sum[seg][col] = sum;
  __syncthreads();
  if (q >= wd) return;
  uint32_t acc = base[0];  // row 0, already unfiltered
  for (int g = 0; g < seg; g++) acc = padd8(acc, seg_sum[g][col]);
#pragma unroll 8
  for (int r = r0; r < r1; r++) {
    acc = padd8(acc, base[(int64_t)r * wd]);
    base[(int64_t)r * wd] = acc;
  }
}

struct GArgs {
  uint8_t* data;
  int* ctl;       // [0] band dequeue, [1] error
  int* diag;      // wg::diag_words + DIAG_ALPHA
  int* progress;  // [n_img][bands]
  int64_t pitch;
  int w, h, bands, n_img;
};
constexpr uint64_t SPIN_TICKS = 200000000ull;  // 2 s of s_memrealtime

// gradient unfilter below row 0 (row 0 already scanned).  Rows 1.. are cut
// into bands of 64; band b holds rows 1 + 64b .. 64 + 64b, one wave each.
// Lane k owns row 1 + 64b + k and walks it one pixel per step, lane k at
// x = s - k (a diagonal), so the row above (lane k-1's newest and previous
// outputs) comes by a lane shift.  The band's pixels are staged through LDS
// in 64-column chunks, a two-chunk ring per lane (row stride 132 B): at step
// 64m the wave stores chunk m-2 back (every lane is past it) and loads chunk
// m with 16-B global accesses, so the per-step work is LDS-only.  The band
// above hands its last row down as before: lane `last_lane` also stores each
// output byte straight to global and publishes progress every 64 columns
// (vmcnt(0), agent release, relaxed counter); the band below reads it with
// agent-scope dword loads into up_buf.
constexpr int GB_STRIDE = 132;

__device__ __forceinline__ void gb_chunk_io(uint8_t* ring_row, uint8_t* row, int c0, int w, bool fast, bool store) {
  uint8_t* slot = ring_row + (c0 & 127);
  if (fast && c0 + 64 <= w) {
    uint4* g = reinterpret_cast<uint4*>(row + c0);
    uint32_t* l = reinterpret_cast<uint32_t*>(slot);
    if (store) {
#pragma unroll
      for (int q = 0; q < 4; q++) g[q] = make_uint4(l[4 * q], l[4 * q + 1], l[4 * q + 2], l[4 * q + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint4 v = g[q];
        l[4 * q] = v.x, l[4 * q + 1] = v.y, l[4 * q + 2] = v.z, l[4 * q + 3] = v.w;
      }
    }
    return;
  }
  const int n = min(64, w - c0);
  for (int i = 0; i < n; i++) {
    if (store)
      row[c0 + i] = slot[i];
    else
      slot[i] = row[c0 + i];
  }
}

__global__ __launch_bounds__(64) void k_alpha_gbands(GArgs a) {
  __shared__ uint8_t up_buf[65];  // the band above's last row, columns c0-1 .. c0+63
  __shared__ __attribute__((aligned(16))) uint8_t ring[64 * GB_STRIDE];
  __shared__ int sh_band;
  const int lane = threadIdx.x;
  const int w = a.w;
  const int total = a.bands * a.n_img;
  const bool fast = ((w & 15) == 0) && ((a.pitch & 15) == 0) && ((reinterpret_cast<uintptr_t>(a.data) & 15) == 0);
  uint8_t* my_ring = ring + lane * GB_STRIDE;
  for (;;) {
    if (lane == 0) sh_band = __hip_atomic_fetch_add(&a.ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int idx = __builtin_amdgcn_readfirstlane(sh_band);
    __syncthreads();
    if (idx >= total) break;
    const int band = idx / a.n_img, img = idx % a.n_img;
    const int y = 1 + band * 64 + lane;
    const bool live = y < a.h;
    uint8_t* d = a.data + img * a.pitch;
    uint8_t* my_row = d + (int64_t)y * w;
    const int* prog_above = a.progress + img * a.bands + band - 1;
    int* prog_mine = a.progress + img * a.bands + band;
    const int last_lane = min(63, a.h - 2 - band * 64);
    const int chunks = (w + 63) >> 6;
    int o1 = 0, o2 = 0;  // this lane's outputs at x-1, x-2 (o2: the value before o1)
    int first = 0;       // row above's value at x = 0 for lane 0 is read with the rest
    const int steps = w + last_lane;
    for (int s = 0; s < steps; s++) {
      const int x = s - lane;
      if ((s & 63) == 0 && s < w) {  // chunk m = s / 64 starts for lane 0
        const int c0 = s;
        if (live && c0 >= 128) gb_chunk_io(my_ring, my_row, c0 - 128, w, fast, true);  // chunk m-2 is done
        if (live) gb_chunk_io(my_ring, my_row, c0, w, fast, false);
        // next 64 columns of the row above this band
        if (band > 0) {
          const int need = min(s + 64, w);
          if (lane == 0) {
            const uint64_t t0 = wg::wait_clock();
            for (uint32_t it = 0;; it++) {
              const int seen = __hip_atomic_load(prog_above, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if (seen >= need) break;
              if ((it & 63) == 63 && (wg::wait_clock() - t0 > SPIN_TICKS ||
                                      __hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                __hip_atomic_fetch_or(&a.ctl[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                wg::note_timeout(a.diag, need, seen, (int)(wg::wait_clock() - t0), (int)blockIdx.x, 0, 0);
                break;
              }
              __builtin_amdgcn_s_sleep(2);
            }
          }
        }
        const uint8_t* up = d + (int64_t)(band * 64) * w;  // row band*64 (row 0 for band 0)
        const int c = s + lane;
        if (c < w) {
          // the aligned dword holding the byte, read around L1 (same page as the byte)
          const uintptr_t addr = reinterpret_cast<uintptr_t>(up + c);
          const uint32_t word = __hip_atomic_load(reinterpret_cast<const uint32_t*>(addr & ~uintptr_t(3)),
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          up_buf[lane + 1] = (uint8_t)(word >> (8 * (addr & 3)));
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __syncthreads();
      }
      // row above at x (lane k-1's newest output) and x-1 (its previous one),
      // by a whole-wave DPP shift (wave_shr:1) rather than an LDS permute
      int top = __builtin_amdgcn_update_dpp(0, o1, 0x138, 0xf, 0xf, false);
      int top_left = __builtin_amdgcn_update_dpp(0, o2, 0x138, 0xf, 0xf, false);
      if (lane == 0 && x < w) {
        const int k = x - (s & ~63);  // x - c0
        top = up_buf[k + 1];
        top_left = k > 0 ? up_buf[k] : (x > 0 ? first : top);
      }
      if (live && x >= 0 && x < w) {
        // x == 0: left = top_left = top (alpha.go:177-181)
        const int left = x == 0 ? top : o1;
        const int tl = x == 0 ? top : top_left;
        uint8_t* cell = my_ring + (x & 127);
        const int v = (*cell + clip255(left + top - tl)) & 0xff;
        o2 = o1;
        o1 = v;
        *cell = (uint8_t)v;
        if (!fast && lane == last_lane) my_row[x] = (uint8_t)v;  // hand-off copy for the band below
      } else {
        o2 = o1;
        o1 = 0;
      }
      if (lane == 0 && (s & 63) == 63) first = up_buf[64];  // column c0+63 for the next chunk's x-1
      // publish the band's last row every 64 columns (and at its end)
      const int xl = s - last_lane;
      if (band + 1 < a.bands && xl >= 0 && ((xl & 63) == 63 || xl == w - 1)) {
        if (fast) {
          // the chunk of the last row, from the last lane's ring, as 4-byte
          // write-through (sc1) stores: no L2 write-back fence per chunk (a
          // release fence here cost microseconds every 64 steps)
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_wave_barrier();
          const int c0 = xl & ~63, n = xl - c0 + 1;
          if (4 * lane < n) {
            const uint32_t word = *reinterpret_cast<const uint32_t*>(ring + last_lane * GB_STRIDE + ((c0 + 4 * lane) & 127));
            __hip_atomic_store(reinterpret_cast<uint32_t*>(d + (int64_t)(1 + band * 64 + last_lane) * w + c0 + 4 * lane), word,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (lane == 0) __hip_atomic_store(prog_mine, xl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          if (lane == last_lane) __hip_atomic_store(prog_mine, xl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    // the last two chunks (or one) have not been stored yet
    if (live)
      for (int m = max(0, chunks - 2); m < chunks; m++) gb_chunk_io(my_ring, my_row, m * 64, w, fast, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // the ring is reused by the next band this wave dequeues
  }
}

// Gradient unfilter below row 0, fast path (w % 16 == 0, w >= 64, 16-B
// aligned rows and images).  The same band / diagonal walk as
// k_alpha_gbands (lane k owns row 1 + 64b + k at x = s - k; the row above by
// a whole-wave DPP shift), with the per-step work in registers:
//  - each lane's residual bytes come in 16-step chunks as one 32-B aligned
//    load pair, two chunks ahead, and are cut to the lane's 16-byte window
//    (offset (-k) & 15, fixed per lane) with selects + v_alignbyte, so a step
//    reads no memory;
//  - lane 0's row above (the band above's last row) arrives as 4-pixel
//    granules {pixels, tag} that the band above's last lane stores with one
//    8-B write-through store each, as soon as it has made them (no progress
//    counter, no store drain); lane 0 loads a chunk's five granules two
//    chunks ahead and re-polls only if a tag is still clear;
//  - outputs go to the LDS ring (one byte store a step, off the chain) and
//    back to the frame 64 columns at a time, as in k_alpha_gbands.
// Band 0's row above is row 0 (already unfiltered by k_alpha_scan_edge).
constexpr int GD_CH = 16;  // steps per chunk

struct GdArgs {
  uint8_t* data;
  int* ctl;        // [0] band dequeue, [1] error
  int* diag;       // wg::diag_words + DIAG_ALPHA
  uint64_t* hand;  // [n_img][bands + 1][w / 4] granules {4 pixels, tag}: row 0, then each band's last row
  int64_t pitch;
  int w, h, bands, n_img;
};

__device__ __forceinline__ int byte_at(uint32_t v, int i) { return (int)((v >> (8 * i)) & 0xff); }
// 64 columns of a lane's ring back to its row, as 16-B pieces (w % 16 == 0:
// a piece is either inside the row or past its end); no loop with a
// run-time count, so the compiler keeps its load-wait bookkeeping exact
// (data / data_n: the batch's planes and their extent, for WG_BOUNDS builds)
__device__ __forceinline__ void gd_store_block(const uint8_t* ring_row, uint8_t* row, int c0, int w, const uint8_t* data,
                                               int64_t data_n) {
  const uint32_t* l = reinterpret_cast<const uint32_t*>(ring_row + (c0 & 127));
#pragma unroll
  for (int q = 0; q < 4; q++)
    if (c0 + 16 * q < w && WG_CHK(row + c0 + 16 * q, 16, data, data_n, "k_alpha_gdiag row store"))
      *reinterpret_cast<uint4*>(row + c0 + 16 * q) = make_uint4(l[4 * q], l[4 * q + 1], l[4 * q + 2], l[4 * q + 3]);
}

// row 0 (already unfiltered) as band 0's row above: granule g = {pixels
// 4g .. 4g + 3, tag 1}
__global__ __launch_bounds__(256) void k_alpha_row0_granules(GdArgs a) {
  const int gw = a.w >> 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)gw * a.n_img) return;
  const int img = (int)(i / gw), g = (int)(i % gw);
  const uint8_t* src = a.data + img * a.pitch + 4 * g;
  uint64_t* const dst = a.hand + (int64_t)img * (a.bands + 1) * gw + g;
  if (!WG_CHK(src, 4, a.data, a.n_img * a.pitch, "k_alpha_row0_granules data") ||
      !WG_CHK(dst, 8, a.hand, 8ll * a.n_img * (a.bands + 1) * gw, "k_alpha_row0_granules hand"))
    return;
  const uint32_t px = *reinterpret_cast<const uint32_t*>(src);
  *dst = 1ull << 32 | px;
}

__global__ __launch_bounds__(64) void k_alpha_gdiag(GdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[64 * GB_STRIDE];
  __shared__ int sh_band;
  const int lane = threadIdx.x;
  const int w = a.w, gw = w >> 2;
  const int total = a.bands * a.n_img;
  uint8_t* my_ring = ring + lane * GB_STRIDE;
  // (WG_BOUNDS) the buffers' extents from the entry point's shapes
  [[maybe_unused]] const int64_t data_n = a.n_img * a.pitch, hand_n = 8ll * a.n_img * (a.bands + 1) * gw;
  // the lane's window within a 16-B aligned 32-B load: chunk starts are
  // multiples of 16, so (s0 - k) & 15 = (-k) & 15
  const int o = (-lane) & 15, q = o >> 2, rsh = o & 3;
  const uint32_t mq1 = (q & 1) ? ~0u : 0u, mq2 = (q & 2) ? ~0u : 0u;
  // m ? a1 : a0, bitwise (one v_bitop3_b32 / v_bfi_b32; as inline asm the
  // compiler put an s_nop on each side of it)
  auto bfi = [](uint32_t m, uint32_t a1, uint32_t a0) { return (m & a1) | (~m & a0); };
  for (;;) {
    if (lane == 0) sh_band = __hip_atomic_fetch_add(&a.ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int idx = __builtin_amdgcn_readfirstlane(sh_band);
    __syncthreads();
    if (idx >= total) break;
    const int band = idx / a.n_img, img = idx % a.n_img;
    const int y = 1 + band * 64 + lane;
    const bool live = y < a.h;
    uint8_t* d = a.data + img * a.pitch;
    uint8_t* my_row = d + (int64_t)min(y, a.h - 1) * w;
    const int last_lane = min(63, a.h - 2 - band * 64);
    const uint64_t* hand_above = a.hand + ((int64_t)img * (a.bands + 1) + band) * gw;  // (band 0: row 0)
    uint64_t* hand_mine = a.hand + ((int64_t)img * (a.bands + 1) + band + 1) * gw;
    const bool hands_off = band + 1 < a.bands;
    const int nch = (w + last_lane + GD_CH - 1) / GD_CH;
    // residual bytes of chunk s0: the 32 aligned bytes holding x = s0 - k ..
    // s0 - k + 15 (rows >= 1, w >= 64: the start is inside the image; the
    // end is clamped, and only x >= w can read the clamped bytes)
    auto ld_res = [&](int s0, uint4& lo, uint4& hi) {
      const int a16 = s0 - lane - o;
      const uint8_t *p0 = my_row + min(a16, w - 16), *p1 = my_row + min(a16 + 16, w - 16);
      lo = WG_CHK(p0, 16, a.data, data_n, "k_alpha_gdiag residuals") ? *reinterpret_cast<const uint4*>(p0)
                                                                       : make_uint4(0, 0, 0, 0);
      hi = WG_CHK(p1, 16, a.data, data_n, "k_alpha_gdiag residuals") ? *reinterpret_cast<const uint4*>(p1)
                                                                       : make_uint4(0, 0, 0, 0);
    };
    // (x < 0 residuals read as 0: every output left of column 0 is then 0,
    // which makes x == 0's left = top_left = top rule hold with no select)
    auto window = [&](int s0, const uint4& lo, const uint4& hi, uint32_t R[4]) {
      const uint32_t D[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      // S[i] = D[i + q] by bit-field inserts on per-lane masks (a ternary on
      // the lane-varying q compiled to exec-masked branches)
      uint32_t S[5];
#pragma unroll
      for (int i = 0; i < 5; i++) S[i] = bfi(mq2, bfi(mq1, D[i + 3], D[i + 2]), bfi(mq1, D[i + 1], D[i]));
#pragma unroll
      for (int j = 0; j < 4; j++) R[j] = __builtin_amdgcn_alignbyte(S[j + 1], S[j], rsh);
      if (s0 < 64) {  // bytes u with s0 + u - k < 0 (the band's first chunks)
        const int t = lane - s0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int sh = t - 4 * j;  // the first kept byte of dword j
          R[j] = sh <= 0 ? R[j] : (sh >= 4 ? 0u : R[j] & (0xffffffffu << (8 * sh)));
        }
      }
    };
    // lane 0's row above for chunk s0: columns s0 - 4 .. s0 + 15, five
    // granules (one load form for every band: row 0's granules are written
    // before the launch, k_alpha_row0_granules)
    auto ld_up = [&](int s0, uint64_t U[5]) {
#pragma unroll
      for (int t = 0; t < 5; t++) {
        const uint64_t* g = hand_above + min(max((s0 >> 2) - 1 + t, 0), gw - 1);
        U[t] = WG_CHK(g, 8, a.hand, hand_n, "k_alpha_gdiag hand load")
                   ? __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : 0ull;
      }
    };
    // Prefetch three chunks ahead in three register sets that the unrolled
    // chunk loop rotates by role, never by copying (a copy of a register a
    // load is still filling makes the compiler wait for the load there).
    uint32_t R[4];
    {
      uint4 lo0, hi0;
      ld_res(0, lo0, hi0);
      window(0, lo0, hi0, R);
    }
    uint4 rX[2], rY[2], rZ[2];  // raw residuals of chunks m + 1, m + 2, m + 3
    ld_res(GD_CH, rX[0], rX[1]);
    ld_res(2 * GD_CH, rY[0], rY[1]);
    ld_res(3 * GD_CH, rZ[0], rZ[1]);
    uint64_t UA[5], UB[5], UC[5];  // the row above for chunks m, m + 1, m + 2
    ld_up(0, UA);
    ld_up(GD_CH, UB);
    ld_up(2 * GD_CH, UC);
    int o1 = 0, o2 = 0;  // this lane's outputs at x - 1, x - 2
    int pub = 0;         // granules of the band's last row published
    // chunk m: consumes R and Uc (its row above), then windows raw (chunk
    // m + 1) into R and refills raw with chunk m + 4 and Uc with chunk m + 3
    auto chunk = [&](int m, uint64_t (&Uc)[5], uint4 (&raw)[2]) {
      const int s0 = m * GD_CH;
      if ((s0 & 63) == 0 && s0 >= 128 && live) gd_store_block(my_ring, my_row, s0 - 128, w, a.data, data_n);  // every lane is past it
      {  // the row above: re-poll the granules whose tag is still clear
        bool ready = true;
#pragma unroll
        for (int t = 0; t < 5; t++) ready &= __builtin_amdgcn_readfirstlane((int)(Uc[t] >> 32)) != 0;
        if (!ready) {  // (re-polled into other registers: a load into Uc here would make every
                       // chunk's first use of its Uc wait for all loads in flight)
          const uint64_t t0 = wg::wait_clock();
          uint64_t T[5];
          for (uint32_t it = 0;; it++) {
            __builtin_amdgcn_s_sleep(1);
            ld_up(s0, T);
            ready = true;
#pragma unroll
            for (int t = 0; t < 5; t++) ready &= __builtin_amdgcn_readfirstlane((int)(T[t] >> 32)) != 0;
            if (ready) break;
            // (the timeout alone ends the wait: a vector load of the error flag
            // here made the compiler treat the chunk buffers as just loaded)
            if ((it & 15) == 15 && wg::wait_clock() - t0 > SPIN_TICKS) {
              if (lane == 0) {
                __hip_atomic_fetch_or(&a.ctl[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                wg::note_timeout(a.diag, s0, band, (int)(wg::wait_clock() - t0), (int)blockIdx.x, 0, 0);
              }
              break;
            }
          }
#pragma unroll
          for (int t = 0; t < 5; t++) Uc[t] = T[t];
        }
      }
      uint32_t UP[5];
#pragma unroll
      for (int t = 0; t < 5; t++) UP[t] = (uint32_t)Uc[t];
      if (s0 == 0) UP[0] = 0;  // column -1 (x == 0's top_left is its top: 0 - 0 cancels)
      // x == 0: left = top_left = top (alpha.go:177-181).  Outputs left of
      // column 0 are 0 (zero residuals, zero row above: see window), so there
      // left - top_left = 0 and the plain formula gives top.
      const int xb = s0 - lane;
      if (s0 + GD_CH <= w) {  // every lane's x < w: the ring takes every byte (x < 0 ones are rewritten later)
#pragma unroll
        for (int u = 0; u < GD_CH; u++) {
          const int res = byte_at(R[u >> 2], u & 3);
          // row above at x and x - 1: lane k - 1's newest and previous outputs
          // (wave_shr:1); lane 0 keeps the band above's row (update_dpp's old)
          const int top = __builtin_amdgcn_update_dpp(byte_at(UP[1 + (u >> 2)], u & 3), o1, 0x138, 0xf, 0xf, false);
          const int tl = __builtin_amdgcn_update_dpp(byte_at(UP[(u + 3) >> 2], (u + 3) & 3), o2, 0x138, 0xf, 0xf, false);
          const int v = (res + clip255(o1 + top - tl)) & 0xff;
          o2 = o1;
          o1 = v;
          my_ring[(xb + u) & 127] = (uint8_t)v;
        }
      } else {  // the band's last chunks: bytes past the row end go to the pad byte
#pragma unroll
        for (int u = 0; u < GD_CH; u++) {
          const int res = byte_at(R[u >> 2], u & 3);
          const int top = __builtin_amdgcn_update_dpp(byte_at(UP[1 + (u >> 2)], u & 3), o1, 0x138, 0xf, 0xf, false);
          const int tl = __builtin_amdgcn_update_dpp(byte_at(UP[(u + 3) >> 2], (u + 3) & 3), o2, 0x138, 0xf, 0xf, false);
          const int v = (res + clip255(o1 + top - tl)) & 0xff;
          o2 = o1;
          o1 = v;
          my_ring[xb + u < w ? (xb + u) & 127 : 128] = (uint8_t)v;
        }
      }
      // the band's last row, 4 pixels at a time, for the band below
      // (a chunk moves the last lane on by 16 columns: at most 4 granules)
      if (hands_off) {
        const int done = min(max((s0 + GD_CH - last_lane) >> 2, 0), gw);
#pragma unroll
        for (int j = 0; j < GD_CH / 4; j++) {
          const int g = pub + j;
          if (g < done && lane == last_lane && WG_CHK(hand_mine + g, 8, a.hand, hand_n, "k_alpha_gdiag hand store")) {
            const uint32_t px = *reinterpret_cast<const uint32_t*>(my_ring + ((4 * g) & 127));
            __hip_atomic_store(hand_mine + g, 1ull << 32 | px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
        pub = max(pub, done);
      }
      window(s0 + GD_CH, raw[0], raw[1], R);
      ld_res(s0 + 4 * GD_CH, raw[0], raw[1]);
      ld_up(s0 + 3 * GD_CH, Uc);
      // (the loads stay here, three chunks ahead of their use: sunk to the
      // loop latch they would be the newest in flight at the next use)
      asm volatile("" ::: "memory");
    };
    for (int m = 0; m < nch; m += 3) {
      chunk(m, UA, rX);
      if (m + 1 >= nch) break;
      chunk(m + 1, UB, rY);
      if (m + 2 >= nch) break;
      chunk(m + 2, UC, rZ);
    }
    // the last two 64-column blocks (or one) have not been stored yet
    const int chunks = (w + 63) >> 6;
    if (live) {
      if (chunks >= 2) gd_store_block(my_ring, my_row, (chunks - 2) * 64, w, a.data, data_n);
      gd_store_block(my_ring, my_row, (chunks - 1) * 64, w, a.data, data_n);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // the ring is reused by the next band this wave dequeues
  }
}

// -------------------------------------------------------------- estimate
// estimateBestFilter's bins split by dependence: the "none" bin follows a
// running mean along each sampled row (serial per row: one lane per row,
// k_alpha_meanwalk); the horizontal / vertical / gradient bins and the colour
// set are per pixel (k_alpha_stats: one thread per 16 bytes of a row, a 2-D
// grid so a block never straddles images).  Bins are 16 bits per filter in one
// 64-bit word per image; every |diff| >> 4 is < 16, so each sets a bit.
__global__ __launch_bounds__(256) void k_alpha_stats(const uint8_t* data, int w, int h, int64_t pitch, int groups,
                                                     int fast, unsigned long long* bins, uint32_t* sets) {
  __shared__ uint32_t set[8];
  __shared__ unsigned long long bin;
  if (threadIdx.x < 8) set[threadIdx.x] = 0;
  if (threadIdx.x == 0) bin = 0;
  __syncthreads();
  const int img = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  unsigned long long seen = 0;
  if (i < (int64_t)groups * h) {
    const int y = (int)(i / groups), x0 = (int)(i % groups) * 16;
    const uint8_t* row = data + img * pitch + (int64_t)y * w;
    const int n = min(16, w - x0);
    uint8_t cur[16];
    if (fast) {
      *reinterpret_cast<uint4*>(cur) = *reinterpret_cast<const uint4*>(row + x0);
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++) cur[k] = k < n ? row[x0 + k] : 0;
    }
    uint32_t local[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; k++)
      if (k < n) {
#pragma unroll
        for (int b = 0; b < 8; b++)
          if ((cur[k] >> 5) == b) local[b] |= 1u << (cur[k] & 31);
      }
#pragma unroll
    for (int b = 0; b < 8; b++)
      if (local[b]) atomicOr(&set[b], local[b]);
    // sampled positions: rows j = 2, 4, .. < h-1; columns i = 2, 4, .. < w-1
    if (y >= 2 && (y & 1) == 0 && y < h - 1) {
      uint8_t up[16];
      if (fast) {
        *reinterpret_cast<uint4*>(up) = *reinterpret_cast<const uint4*>(row - w + x0);
      } else {
#pragma unroll
        for (int k = 0; k < 16; k++) up[k] = k < n ? row[x0 + k - w] : 0;
      }
      // x0 is a multiple of 16, so the sampled columns are the even k; their left
      // neighbours (odd k) are inside the group
#pragma unroll
      for (int k = 0; k < 16; k += 2) {
        const int x = x0 + k;
        if (x >= 2 && x < w - 1) {
          const int c = cur[k], l = cur[k - 1 < 0 ? 0 : k - 1], t = up[k], tl = up[k - 1 < 0 ? 0 : k - 1];
          const int lft = k > 0 ? l : row[x - 1], tlf = k > 0 ? tl : row[x - 1 - w];
          const int g = clip255(lft + t - tlf);
          seen |= 1ull << (16 + (abs(c - lft) >> 4));
          seen |= 1ull << (32 + (abs(c - t) >> 4));
          seen |= 1ull << (48 + (abs(c - g) >> 4));
        }
      }
    }
  }
  // OR over the wave, then the block
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) seen |= __shfl_xor(seen, o, 64);
  if ((threadIdx.x & 63) == 0 && seen) atomicOr(&bin, seen);
  __syncthreads();
  if (threadIdx.x < 8 && set[threadIdx.x]) atomicOr(&sets[img * 8 + threadIdx.x], set[threadIdx.x]);
  if (threadIdx.x == 0 && bin) atomicOr(&bins[img], bin);
}

// the "none" bin: lane = sampled row j = 2 + 2t, the running mean walked over
// its even columns (estimateBestFilter :343-375), rows read 64 B at a time
__global__ __launch_bounds__(64) void k_alpha_meanwalk(const uint8_t* data, int w, int h, int64_t pitch, int rows,
                                                       int fast, unsigned long long* bins) {
  const int img = blockIdx.y;
  const int t = blockIdx.x * 64 + threadIdx.x;
  unsigned long long seen = 0;
  if (t < rows) {
    const uint8_t* p = data + img * pitch + (int64_t)(2 + 2 * t) * w;
    int mean = p[0];
    const int end = w - 1;  // i < w - 1
    if (fast) {
      // 64-byte blocks; i even in [2, end)
      const uint4* q = reinterpret_cast<const uint4*>(p);
      const int blocks = (end + 63) >> 6;
      uint4 nxt[4];
#pragma unroll
      for (int k = 0; k < 4; k++) nxt[k] = (k < (w >> 4)) ? q[k] : make_uint4(0, 0, 0, 0);
      for (int b = 0; b < blocks; b++) {
        uint4 cb[4];
#pragma unroll
        for (int k = 0; k < 4; k++) cb[k] = nxt[k];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int qi = 4 * (b + 1) + k;
          nxt[k] = qi < (w >> 4) ? q[qi] : make_uint4(0, 0, 0, 0);
        }
        const uint32_t* wd = reinterpret_cast<const uint32_t*>(cb);
#pragma unroll
        for (int k = 0; k < 32; k++) {
          const int i = 64 * b + 2 * k;
          const int cur = (wd[k >> 1] >> (16 * (k & 1))) & 0xff;
          if (i >= 2 && i < end) {
            seen |= 1ull << (abs(cur - mean) >> 4);
            mean = (3 * mean + cur + 2) >> 2;
          }
        }
      }
    } else {
      for (int i = 2; i < end; i += 2) {
        const int cur = p[i];
        seen |= 1ull << (abs(cur - mean) >> 4);
        mean = (3 * mean + cur + 2) >> 2;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) seen |= __shfl_xor(seen, o, 64);
  if (threadIdx.x == 0 && seen) atomicOr(&bins[img], seen);
}

__global__ void k_alpha_finalize(const unsigned long long* bins, const uint32_t* sets, int n_img, int32_t* best,
                                 int32_t* colors) {
  const int img = blockIdx.x * blockDim.x + threadIdx.x;
  if (img >= n_img) return;
  const unsigned long long b = bins[img];
  int bf = 0, bs = 0x7fffffff;
  for (int f = 0; f < 4; f++) {
    int score = 0;
    for (int i = 0; i < 16; i++)
      if ((b >> (16 * f + i)) & 1) score += i;
    if (score < bs) {
      bs = score;
      bf = f;
    }
  }
  int nc = 0;
  for (int k = 0; k < 8; k++) nc += __popc(sets[img * 8 + k]);
  best[img] = bf;
  colors[img] = nc;
}

// -------------------------------------------------------------- premultiply
__device__ __forceinline__ uint32_t a_mult(uint32_t x, uint32_t mult) { return (x * mult + (1u << 23)) >> 24; }
__device__ __forceinline__ uint32_t a_scale(uint32_t a, int inverse) {
  return inverse ? (255u << 24) / a : a * ((1u << 24) / 255);
}

__global__ __launch_bounds__(256) void k_alpha_multiply(uint8_t* rgba, int alpha_first, int w, int h, int stride,
                                                        int64_t pitch, int inverse, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t per = (int64_t)w * h;
  const int64_t img = i / per, r = i - img * per;
  uint8_t* p = rgba + img * pitch + (r / w) * stride + 4 * (r % w);
  const uint32_t word = *reinterpret_cast<const uint32_t*>(p);
  const int ao = alpha_first ? 0 : 3, ro = alpha_first ? 1 : 0;
  const uint32_t a = (word >> (8 * ao)) & 0xff;
  if (a == 255) return;
  uint32_t out = word & (0xffu << (8 * ao));
  if (a != 0) {
    const uint32_t s = a_scale(a, inverse);
#pragma unroll
    for (int c = 0; c < 3; c++) out |= (a_mult((word >> (8 * (ro + c))) & 0xff, s) & 0xff) << (8 * (ro + c));
  }
  *reinterpret_cast<uint32_t*>(p) = out;
}

__global__ __launch_bounds__(256) void k_mult_argb(uint32_t* argb, int64_t n, int inverse) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = argb[i];
  if (p >= 0xff000000u) return;
  if (p <= 0x00ffffffu) {
    argb[i] = 0;
    return;
  }
  const uint32_t s = a_scale((p >> 24) & 0xff, inverse);
  argb[i] = (p & 0xff000000u) | (a_mult(p & 0xff, s) & 0xff) | (a_mult((p >> 8) & 0xff, s) & 0xff) << 8 |
            (a_mult((p >> 16) & 0xff, s) & 0xff) << 16;
}

__global__ __launch_bounds__(256) void k_alpha_4444(uint8_t* data, int w, int h, int stride, int64_t pitch,
                                                    int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t per = (int64_t)w * h;
  const int64_t img = i / per, r = i - img * per;
  uint8_t* p = data + img * pitch + (r / w) * stride + 2 * (r % w);
  const int rg = p[0], ba = p[1], a = ba & 0x0f;
  if (a == 0x0f) return;
  if (a == 0) {
    p[0] = p[1] = 0;
    return;
  }
  const int rr = (((rg >> 4) & 0x0f) * a + 7) / 15, gg = ((rg & 0x0f) * a + 7) / 15, bb = (((ba >> 4) & 0x0f) * a + 7) / 15;
  p[0] = (uint8_t)(rr << 4 | gg);
  p[1] = (uint8_t)(bb << 4 | a);
}

// -------------------------------------------------------------- dispatch / extract
__global__ __launch_bounds__(256) void k_dispatch_alpha(const uint8_t* alpha, int alpha_stride, int w, int h,
                                                        uint8_t* dst, int dst_stride, int alpha_off, int* any_transparent) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool in = i < (int64_t)w * h;
  int v = 0xff;
  if (in) {
    const int y = (int)(i / w), x = (int)(i % w);
    v = alpha[(int64_t)y * alpha_stride + x];
    dst[(int64_t)y * dst_stride + 4 * x + alpha_off] = (uint8_t)v;
  }
  if (__ballot(v != 0xff) && (threadIdx.x & 63) == 0) atomicOr(any_transparent, 1);
}

__global__ __launch_bounds__(256) void k_extract_alpha(const uint8_t* src, int src_stride, int w, int h, uint8_t* alpha,
                                                       int alpha_stride, int alpha_off, int* and_mask) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool in = i < (int64_t)w * h;
  int v = 0xff;
  if (in) {
    const int y = (int)(i / w), x = (int)(i % w);
    v = src[(int64_t)y * src_stride + 4 * x + alpha_off];
    alpha[(int64_t)y * alpha_stride + x] = (uint8_t)v;
  }
  if (__ballot(v != 0xff) && (threadIdx.x & 63) == 0) atomicAnd(and_mask, 0);
}

// -------------------------------------------------------------- small row helpers (alpha_proc.go:178-238)
// HasAlpha8b / HasAlpha32b: any byte at i * step (i < n) other than 0xff
__global__ __launch_bounds__(256) void k_has_alpha(const uint8_t* src, int64_t n, int step, int* any) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool hit = i < n && src[i * step] != 0xff;
  if (__ballot(hit) && (threadIdx.x & 63) == 0) atomicOr(any, 1);
}

__global__ __launch_bounds__(256) void k_alpha_replace(uint32_t* argb, int64_t n, uint32_t color) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n && (argb[i] >> 24) == 0) argb[i] = color;
}

__global__ __launch_bounds__(256) void k_alpha_to_green(const uint8_t* alpha, int alpha_stride, int w, int h,
                                                        uint32_t* dst, int dst_stride) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)w * h) return;
  const int y = (int)(i / w), x = (int)(i % w);
  dst[(int64_t)y * dst_stride + x] = (uint32_t)alpha[(int64_t)y * alpha_stride + x] << 8;
}

__global__ __launch_bounds__(256) void k_extract_green(const uint32_t* argb, uint8_t* alpha, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) alpha[i] = (uint8_t)(argb[i] >> 8);
}

__global__ __launch_bounds__(256) void k_pack_rgb(const uint8_t* r, const uint8_t* g, const uint8_t* b, int64_t n,
                                                  int step, uint32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t o = i * step;
  out[i] = 0xff000000u | (uint32_t)r[o] << 16 | (uint32_t)g[o] << 8 | (uint32_t)b[o];
}

unsigned grid_of(int64_t total, int block) { return (unsigned)((total + block - 1) / block); }

}  // namespace

extern "C" int wg_alpha_filter(int32_t filter, const uint8_t* in, uint8_t* out, int32_t width, int32_t height,
                               int64_t pitch, int32_t n_images, void* stream) {
  WG_REQUIRE(in && out && width > 0 && height > 0 && n_images > 0 && filter >= 0 && filter <= 3);
  WG_REQUIRE(pitch >= (int64_t)width * height);
  const int groups = (width + 15) / 16;
  const int64_t total = (int64_t)groups * height * n_images;
  const int fast = (width & 15) == 0 && (pitch & 15) == 0 && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  hipLaunchKernelGGL(k_alpha_filter, dim3(grid_of(total, 256)), dim3(256), 0, wg::as_stream(stream), (int)filter, in, out,
                     (int)width, (int)height, pitch, groups, total, fast);
  return wg::check_launch("k_alpha_filter");
}

// work: ctl[4] | progress[n_img * bands] (k_alpha_gbands) | hand-off granules
// [n_img][bands + 1][width / 4] (k_alpha_gdiag: row 0, then each band's last
// row), 16-B aligned
static size_t gd_hand_offset(int32_t height, int32_t n_images) {
  const int bands = (height - 1 + 63) / 64;
  return (sizeof(int) * (4 + (size_t)n_images * (bands > 0 ? bands : 1)) + 15) & ~(size_t)15;
}
extern "C" size_t wg_alpha_unfilter_work_bytes(int32_t width, int32_t height, int32_t n_images) {
  if (width <= 0 || height <= 0 || n_images <= 0) return 0;
  const int bands = (height - 1 + 63) / 64;
  return gd_hand_offset(height, n_images) + sizeof(uint64_t) * (size_t)n_images * (bands + 1) * ((width + 3) / 4);
}

extern "C" int wg_alpha_unfilter(int32_t filter, uint8_t* data, int32_t width, int32_t height, int64_t pitch,
                                 int32_t n_images, void* work, void* stream) {
  WG_REQUIRE(data && width > 0 && height > 0 && n_images > 0 && filter >= 0 && filter <= 3);
  WG_REQUIRE(pitch >= (int64_t)width * height);
  hipStream_t s = wg::as_stream(stream);
  if (filter == 0) return WG_OK;
  if (filter == 1) {
    hipLaunchKernelGGL(k_alpha_scan_edge, dim3(n_images), dim3(64), 0, s, data, (int)width, (int)height, pitch, 0);
    int rc = wg::check_launch("k_alpha_scan_edge");
    if (rc != WG_OK) return rc;
    const int fast = (width & 15) == 0 && (pitch & 15) == 0 && (reinterpret_cast<uintptr_t>(data) & 15) == 0;
    hipLaunchKernelGGL(k_alpha_hrows, dim3((unsigned)((int64_t)height * n_images)), dim3(64), 0, s, data, (int)width,
                       (int)height, pitch, fast);
    return wg::check_launch("k_alpha_hrows");
  }
  hipLaunchKernelGGL(k_alpha_scan_edge, dim3(n_images), dim3(64), 0, s, data, (int)width, (int)height, pitch, 1);
  int rc = wg::check_launch("k_alpha_scan_edge");
  if (rc != WG_OK || height == 1) return rc;
  if (filter == 2 && (width & 3) == 0 && (pitch & 3) == 0 && (reinterpret_cast<uintptr_t>(data) & 3) == 0) {
    const int strips = (width / 4 + 63) / 64;
    hipLaunchKernelGGL(k_alpha_vseg, dim3((unsigned)(strips * n_images)), dim3(1024), 0, s, data, (int)width,
                       (int)height, pitch, strips);
    return wg::check_launch("k_alpha_vseg");
  }
  if (filter == 2) {
    const int64_t total = (int64_t)width * n_images;
    hipLaunchKernelGGL(k_alpha_vcols, dim3(grid_of(total, 256)), dim3(256), 0, s, data, (int)width, (int)height, pitch,
                       total);
    return wg::check_launch("k_alpha_vcols");
  }
  WG_REQUIRE(work);
  WG_REQUIRE((reinterpret_cast<uintptr_t>(work) & 15) == 0);
  if (hipMemsetAsync(work, 0, wg_alpha_unfilter_work_bytes(width, height, n_images), s) != hipSuccess)
    return wg::check_launch("hipMemsetAsync(alpha work)");
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return wg::check_launch("device query");
  const int bands = (height - 1 + 63) / 64;
  const int total = bands * n_images;
  const int grid = total < 4 * cus ? total : 4 * cus;
  if ((width & 15) == 0 && width >= 64 && (pitch & 15) == 0 && (reinterpret_cast<uintptr_t>(data) & 15) == 0 &&
      !getenv("WG_ALPHA_GBANDS")) {
    GdArgs g;
    g.data = data;
    g.ctl = static_cast<int*>(work);
    g.diag = wg::diag_words(s);
    if (!g.diag) return WG_EHIP;
    g.diag += wg::DIAG_ALPHA;
    g.hand = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(work) + gd_hand_offset(height, n_images));
    g.pitch = pitch;
    g.w = width;
    g.h = height;
    g.bands = bands;
    g.n_img = n_images;
    hipLaunchKernelGGL(k_alpha_row0_granules, dim3(wg::blocks_for((int64_t)(width / 4) * n_images, 256)), dim3(256), 0, s, g);
    if ((rc = wg::check_launch("k_alpha_row0_granules")) != WG_OK) return rc;
    hipLaunchKernelGGL(k_alpha_gdiag, dim3(grid), dim3(64), 0, s, g);
    return wg::check_launch("k_alpha_gdiag");
  }
  GArgs a;
  a.data = data;
  a.ctl = static_cast<int*>(work);
  a.diag = wg::diag_words(s);
  if (!a.diag) return WG_EHIP;
  a.diag += wg::DIAG_ALPHA;
  a.progress = a.ctl + 4;
  a.pitch = pitch;
  a.w = width;
  a.h = height;
  a.bands = bands;
  a.n_img = n_images;
  hipLaunchKernelGGL(k_alpha_gbands, dim3(grid), dim3(64), 0, s, a);
  return wg::check_launch("k_alpha_gbands");
}

extern "C" int wg_alpha_unfilter_status(const void* work, void* stream) {
  WG_REQUIRE(work);
  return wg::wait_status(static_cast<const int*>(work) + 1, wg::DIAG_ALPHA, wg::as_stream(stream),
                         "wg_alpha_unfilter_status: alpha unfilter band", "needed, seen, ticks, block, -, -");
}

extern "C" size_t wg_alpha_estimate_work_bytes(int32_t n_images) {
  return n_images > 0 ? (size_t)n_images * (sizeof(unsigned long long) + 8 * sizeof(uint32_t)) : 0;
}

extern "C" int wg_alpha_estimate_filter(const uint8_t* data, int32_t width, int32_t height, int64_t pitch,
                                        int32_t n_images, int32_t* best_filter, int32_t* num_colors, void* work,
                                        void* stream) {
  WG_REQUIRE(data && best_filter && num_colors && work && width > 0 && height > 0 && n_images > 0);
  WG_REQUIRE(pitch >= (int64_t)width * height);
  hipStream_t s = wg::as_stream(stream);
  unsigned long long* bins = static_cast<unsigned long long*>(work);
  uint32_t* sets = reinterpret_cast<uint32_t*>(bins + n_images);
  if (hipMemsetAsync(work, 0, wg_alpha_estimate_work_bytes(n_images), s) != hipSuccess)
    return wg::check_launch("hipMemsetAsync(alpha estimate)");
  const int rows = (height - 2) / 2;
  const int fast = (width & 15) == 0 && (pitch & 15) == 0 && (reinterpret_cast<uintptr_t>(data) & 15) == 0;
  if (rows > 0) {
    hipLaunchKernelGGL(k_alpha_meanwalk, dim3(grid_of(rows, 64), n_images), dim3(64), 0, s, data, (int)width,
                       (int)height, pitch, rows, fast, bins);
    const int rc = wg::check_launch("k_alpha_meanwalk");
    if (rc != WG_OK) return rc;
  }
  const int groups = (width + 15) / 16;
  hipLaunchKernelGGL(k_alpha_stats, dim3(grid_of((int64_t)groups * height, 256), n_images), dim3(256), 0, s, data,
                     (int)width, (int)height, pitch, groups, fast, bins, sets);
  int rc = wg::check_launch("k_alpha_stats");
  if (rc != WG_OK) return rc;
  hipLaunchKernelGGL(k_alpha_finalize, dim3(grid_of(n_images, 64)), dim3(64), 0, s, bins, sets, (int)n_images,
                     best_filter, num_colors);
  return wg::check_launch("k_alpha_finalize");
}

extern "C" int wg_apply_alpha_multiply(uint8_t* rgba, int32_t alpha_first, int32_t width, int32_t height,
                                       int32_t stride, int64_t pitch, int32_t n_images, int32_t inverse, void* stream) {
  WG_REQUIRE(rgba && width > 0 && height > 0 && n_images > 0 && stride >= 4 * width);
  WG_REQUIRE((stride & 3) == 0 && (pitch & 3) == 0 && (reinterpret_cast<uintptr_t>(rgba) & 3) == 0);
  WG_REQUIRE(pitch >= (int64_t)stride * (height - 1) + 4 * width);
  const int64_t total = (int64_t)width * height * n_images;
  hipLaunchKernelGGL(k_alpha_multiply, dim3(grid_of(total, 256)), dim3(256), 0, wg::as_stream(stream), rgba,
                     (int)(alpha_first != 0), (int)width, (int)height, (int)stride, pitch, (int)(inverse != 0), total);
  return wg::check_launch("k_alpha_multiply");
}

extern "C" int wg_mult_argb(uint32_t* argb, int64_t n, int32_t inverse, void* stream) {
  WG_REQUIRE(argb && n >= 0);
  if (n == 0) return WG_OK;
  hipLaunchKernelGGL(k_mult_argb, dim3(grid_of(n, 256)), dim3(256), 0, wg::as_stream(stream), argb, n, (int)(inverse != 0));
  return wg::check_launch("k_mult_argb");
}

extern "C" int wg_apply_alpha_multiply_4444(uint8_t* data, int32_t width, int32_t height, int32_t stride,
                                            int64_t pitch, int32_t n_images, void* stream) {
  WG_REQUIRE(data && width > 0 && height > 0 && n_images > 0 && stride >= 2 * width);
  WG_REQUIRE(pitch >= (int64_t)stride * (height - 1) + 2 * width);
  const int64_t total = (int64_t)width * height * n_images;
  hipLaunchKernelGGL(k_alpha_4444, dim3(grid_of(total, 256)), dim3(256), 0, wg::as_stream(stream), data, (int)width,
                     (int)height, (int)stride, pitch, total);
  return wg::check_launch("k_alpha_4444");
}

extern "C" int wg_dispatch_alpha(const uint8_t* alpha, int32_t alpha_stride, int32_t width, int32_t height, uint8_t* dst,
                                 int32_t dst_stride, int32_t alpha_off, int32_t* has_transparency, void* stream) {
  WG_REQUIRE(alpha && dst && has_transparency && width > 0 && height > 0 && alpha_off >= 0 && alpha_off <= 3);
  WG_REQUIRE(alpha_stride >= width && dst_stride >= 4 * width);
  hipStream_t s = wg::as_stream(stream);
  if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(has_transparency), 0, 1, s) != hipSuccess)
    return wg::check_launch("hipMemsetD32Async(dispatch flag)");
  hipLaunchKernelGGL(k_dispatch_alpha, dim3(grid_of((int64_t)width * height, 256)), dim3(256), 0, s, alpha,
                     (int)alpha_stride, (int)width, (int)height, dst, (int)dst_stride, (int)alpha_off,
                     reinterpret_cast<int*>(has_transparency));
  return wg::check_launch("k_dispatch_alpha");
}

extern "C" int wg_extract_alpha(const uint8_t* src, int32_t src_stride, int32_t width, int32_t height, uint8_t* alpha,
                                int32_t alpha_stride, int32_t alpha_off, int32_t* all_opaque, void* stream) {
  WG_REQUIRE(src && alpha && all_opaque && width > 0 && height > 0 && alpha_off >= 0 && alpha_off <= 3);
  WG_REQUIRE(alpha_stride >= width && src_stride >= 4 * width);
  hipStream_t s = wg::as_stream(stream);
  if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(all_opaque), 1, 1, s) != hipSuccess)
    return wg::check_launch("hipMemsetD32Async(extract flag)");
  hipLaunchKernelGGL(k_extract_alpha, dim3(grid_of((int64_t)width * height, 256)), dim3(256), 0, s, src,
                     (int)src_stride, (int)width, (int)height, alpha, (int)alpha_stride, (int)alpha_off,
                     reinterpret_cast<int*>(all_opaque));
  return wg::check_launch("k_extract_alpha");
}

extern "C" int wg_has_alpha(const uint8_t* src, int64_t length, int32_t step, int32_t* any_transparent, void* stream) {
  WG_REQUIRE(src && any_transparent && length >= 0 && (step == 1 || step == 4));
  hipStream_t s = wg::as_stream(stream);
  if (hipMemsetAsync(any_transparent, 0, sizeof(int32_t), s) != hipSuccess)
    return wg::check_launch("hipMemsetAsync(has_alpha flag)");
  if (length == 0) return WG_OK;
  hipLaunchKernelGGL(k_has_alpha, dim3(grid_of(length, 256)), dim3(256), 0, s, src, length, (int)step, any_transparent);
  return wg::check_launch("k_has_alpha");
}

extern "C" int wg_alpha_replace(uint32_t* argb, int64_t length, uint32_t color, void* stream) {
  WG_REQUIRE(argb && length >= 0);
  if (length == 0) return WG_OK;
  hipLaunchKernelGGL(k_alpha_replace, dim3(grid_of(length, 256)), dim3(256), 0, wg::as_stream(stream), argb, length,
                     color);
  return wg::check_launch("k_alpha_replace");
}

extern "C" int wg_dispatch_alpha_to_green(const uint8_t* alpha, int32_t alpha_stride, int32_t width, int32_t height,
                                          uint32_t* dst, int32_t dst_stride, void* stream) {
  WG_REQUIRE(alpha && dst && width > 0 && height > 0 && alpha_stride >= width && dst_stride >= width);
  hipLaunchKernelGGL(k_alpha_to_green, dim3(grid_of((int64_t)width * height, 256)), dim3(256), 0,
                     wg::as_stream(stream), alpha, (int)alpha_stride, (int)width, (int)height, dst, (int)dst_stride);
  return wg::check_launch("k_alpha_to_green");
}

extern "C" int wg_extract_green(const uint32_t* argb, uint8_t* alpha, int64_t size, void* stream) {
  WG_REQUIRE(argb && alpha && size >= 0);
  if (size == 0) return WG_OK;
  hipLaunchKernelGGL(k_extract_green, dim3(grid_of(size, 256)), dim3(256), 0, wg::as_stream(stream), argb, alpha, size);
  return wg::check_launch("k_extract_green");
}

extern "C" int wg_pack_rgb(const uint8_t* r, const uint8_t* g, const uint8_t* b, int64_t length, int32_t step,
                           uint32_t* out, void* stream) {
  WG_REQUIRE(r && g && b && out && length >= 0 && step > 0);
  if (length == 0) return WG_OK;
  hipLaunchKernelGGL(k_pack_rgb, dim3(grid_of(length, 256)), dim3(256), 0, wg::as_stream(stream), r, g, b, length,
                     (int)step, out);
  return wg::check_launch("k_pack_rgb");
}
