// sharpyuv.hip -- SharpYUV RGB -> YUV420 on gfx950,
// any transfer function and conversion matrix (sharpyuv/sharpyuv.go:39-432),
// and convertStandard (:68-115) when sharpening is off (k_sharp_standard).
//
//   k_sharp_init   import + gray Y, target W, target / initial chroma
//                  residuals (convertSharp phase 1, :196-222): one thread per
//                  2x2 block, fully parallel
//   k_sharp_wave   the iterative refinement (:224-264).  Each iteration sweeps
//                  the row pairs in order and updates the chroma residuals in
//                  place, so row pair j reads row pair j-1's values from the
//                  SAME iteration (Gauss-Seidel): a sweep is sequential by
//                  construction.  But iteration k+1 at row pair j needs only
//                  iteration k's rows up to j+1, so the four iterations run
//                  as a pipeline, each reading state k and writing state k+1
//                  (five states per image, out of place), iteration k+1
//                  trailing k by three row pairs behind progress counters
//                  (published every WB_PUB row pairs, once the wave's stores
//                  have drained); and an iteration's columns split into
//                  one-wave bands of WB_OWN columns that recompute a WB_HALO
//                  halo on each side and meet their neighbours once every
//                  WB_HALO row pairs (see the kernel).
//                  The early exit (:254-263) needs each iteration's global
//                  |dY| sum; all four iterations run speculatively and
//                  k_sharp_final picks the state the reference would stop at.
//   k_sharp_final  W/RGB -> YUV with the matrix (:390-432), per pixel
//
// All arithmetic is integer (the reference's int / int64 / int16 with wrap);
// the gamma tables are built on the host (sharpyuv_host.cpp) like
// initGammaTables (gamma.go:48-88) and staged in LDS.  For the transfer
// functions other than sRGB (LUT = true) GammaToLinear is the same 1024-entry
// LDS table and LinearToGamma a direct uint16 table in global memory (up to
// 72k entries, L2-resident), gamma.go:360-446.
#include <algorithm>

#include "wg_common.h"
#include "wg_instr.h"

namespace {

constexpr int G2L_N = 1026, L2G_N = 514;
constexpr int SFIX = 2, BD = 10, MAXY = (1 << BD) - 1;

struct SharpTabs {
  uint32_t g2l[G2L_N];
  uint32_t l2g[L2G_N];
};

__device__ __forceinline__ uint32_t to_linear(const uint32_t* g2l, int v) { return g2l[v]; }  // bitDepth 10: exact table
// fromLinearSrgb at bitDepth 10: fixedPointInterpolation(v, l2g, 7, -6) (gamma.go:97-123)
__device__ __forceinline__ int from_linear(const uint32_t* l2g, uint32_t v) {
  const uint32_t pos = v >> 7, x = v & 127u;
  const uint32_t v0 = l2g[pos] >> 6, v1 = l2g[pos + 1] >> 6;
  return (int)(v0 + (((v1 - v0) * x + 64u) >> 7));
}
// LinearToGamma: the sRGB interpolation, or the direct table of another transfer
template <bool LUT>
__device__ __forceinline__ int from_lin(const uint32_t* l2g, const uint16_t* lut, int n, uint32_t v) {
  if (LUT) return lut[min(v, (uint32_t)(n - 1))];
  return from_linear(l2g, v);
}
__device__ __forceinline__ int gray(int64_t r, int64_t g, int64_t b) {
  return (int)((13933 * r + 46871 * g + 4732 * b + 32768) >> 16);
}
__device__ __forceinline__ int clip_bd(int v) { return min(max(v, 0), MAXY); }

// Per image working set: NSTATE states of (best_y: w*h uint16, best_uv: uvh
// rows of uv_rs int16 = the 3 planes of uvw residuals R-W, G-W, B-W, padded
// to 16 bytes), the targets in the same layouts, and per image the four
// iterations' |dY| sums, progress counters and the iteration count.
constexpr int NSTATE = 5;  // state 0 = phase 1's result, state k+1 = after iteration k

struct SharpArgs {
  const uint8_t* rgb;
  int64_t rgb_pitch;
  int rgb_stride, width, height, w, h, uvw, uvh, uv_rs;
  uint16_t* best_y;     // state 0 of image 0; state s of image i at + i * img_elems_y + s * state_y
  uint16_t* target_y;   // image i at + i * img_elems_y
  int16_t* best_uv;
  int16_t* target_uv;
  int64_t img_y, state_y, img_uv, state_uv;  // elements
  const SharpTabs* tabs;
  const uint16_t* lut;  // LinearToGamma of a non-sRGB transfer (LUT kernels)
  int lut_n;
  uint64_t* sums;  // [n_img][4]
  int* prog;       // [n_img][4] row pairs finished per iteration
  int* iters;      // [n_img] iterations the reference runs (-1: a dependency wait timed out)
  uint64_t* hand;  // [n_img][4][bands][2][WB_OWN] edge granules {3 x int16 updated chroma, row tag} (halo reloads)
  int n_img;
  const uint8_t* work0;  // (WG_BOUNDS) the whole work buffer and its size
  int64_t work_n;
  uint64_t* stamps;  // (WG_TIMELINES builds) per k_sharp_wave block and role [4]: start, end,
                     // global-wait ticks | waits << 32, LDS-wait ticks | waits << 32
};

__device__ __forceinline__ void load_tabs(SharpTabs& dst, const SharpTabs* src) {
  for (int i = threadIdx.x; i < G2L_N; i += blockDim.x) dst.g2l[i] = src->g2l[i];
  for (int i = threadIdx.x; i < L2G_N; i += blockDim.x) dst.l2g[i] = src->l2g[i];
  __syncthreads();
}

// phase 1: thread = one UV position (i, jUV) of one image
template <bool LUT>
__global__ __launch_bounds__(256) void k_sharp_init(SharpArgs a, int n_img) {
  __shared__ SharpTabs t;
  load_tabs(t, a.tabs);
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)a.uvw * a.uvh;
  if (gid >= per * n_img) return;
  const int img = (int)(gid / per);
  const int64_t p = gid - img * per;
  const int ju = (int)(p / a.uvw), i = (int)(p - (int64_t)ju * a.uvw);
  const int j = 2 * ju;
  if (j >= a.height) return;  // cannot happen: uvh = ceil(height / 2)
  const uint8_t* rgb = a.rgb + img * a.rgb_pitch;
  int c[2][2][3];  // [row][col][channel] at 10-bit precision (importOneRow, :271-285)
  for (int r = 0; r < 2; r++) {
    const int row = (j + r < a.height) ? j + r : j;  // odd height: last row pair repeats the row
    for (int k = 0; k < 2; k++) {
      const int x = min(2 * i + k, a.width - 1);  // odd width: replicate the last pixel
      const uint8_t* px = rgb + (int64_t)row * a.rgb_stride + 3 * x;
      const bool in = WG_CHK(px, 3, a.rgb, (int64_t)n_img * a.rgb_pitch, "k_sharp_init rgb");
      c[r][k][0] = in ? px[0] << SFIX : 0;
      c[r][k][1] = in ? px[1] << SFIX : 0;
      c[r][k][2] = in ? px[2] << SFIX : 0;
    }
  }
  uint16_t* by = a.best_y + img * a.img_y;
  uint16_t* ty = a.target_y + img * a.img_y;
  uint32_t lin[2][2][3];
  for (int r = 0; r < 2; r++)
    for (int k = 0; k < 2; k++) {
      const int64_t o = (int64_t)(j + r) * a.w + 2 * i + k;
      if (!WG_CHK(by + o, 2, a.work0, a.work_n, "k_sharp_init best_y") ||
          !WG_CHK(ty + o, 2, a.work0, a.work_n, "k_sharp_init target_y"))
        continue;
      by[o] = (uint16_t)gray(c[r][k][0], c[r][k][1], c[r][k][2]);  // storeGray
      for (int ch = 0; ch < 3; ch++) lin[r][k][ch] = to_linear(t.g2l, c[r][k][ch]);
      ty[o] = (uint16_t)from_lin<LUT>(t.l2g, a.lut, a.lut_n, (uint32_t)gray(lin[r][k][0], lin[r][k][1], lin[r][k][2]));  // updateW
    }
  int rgbv[3];  // updateChroma (:303-315): scaleDown in linear light
  for (int ch = 0; ch < 3; ch++)
    rgbv[ch] = from_lin<LUT>(t.l2g, a.lut, a.lut_n, (lin[0][0][ch] + lin[0][1][ch] + lin[1][0][ch] + lin[1][1][ch] + 2) >> 2);
  const int gv = gray(rgbv[0], rgbv[1], rgbv[2]);
  int16_t* tuv = a.target_uv + img * a.img_uv + (int64_t)ju * a.uv_rs;
  int16_t* buv = a.best_uv + img * a.img_uv + (int64_t)ju * a.uv_rs;
  for (int ch = 0; ch < 3; ch++) {
    const int16_t d = (int16_t)(rgbv[ch] - gv);
    if (WG_CHK(tuv + ch * a.uvw + i, 2, a.work0, a.work_n, "k_sharp_init target_uv")) tuv[ch * a.uvw + i] = d;
    if (WG_CHK(buv + ch * a.uvw + i, 2, a.work0, a.work_n, "k_sharp_init best_uv")) buv[ch * a.uvw + i] = d;
  }
}

constexpr uint64_t SPIN_TICKS = 200000000ull;  // 2 s of s_memrealtime (100 MHz)

// Hand-off loads / stores between the iteration workgroups: agent-scope
// relaxed atomics, i.e. sc1 (write-through stores, L1-bypassing loads); every
// load of handed-off bytes is one, every store of them too, and the progress
// counter is stored after the wave's vmcnt(0)
// (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ uint32_t ld_sc1(const void* p) {
  return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(void* p, uint32_t v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1_64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_16(void* p, uint16_t v) {
  __hip_atomic_store(reinterpret_cast<uint16_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// phase 2: workgroup = ONE WAVE = (image, iteration, column band).  A
// refinement iteration is a Gauss-Seidel sweep over the row pairs: row pair j
// reads the chroma row j-1 updated by the SAME iteration (prev), so a sweep is
// sequential in j; but the update of UV column i reads prev only at columns
// i-1..i+1, so a band of columns can run ahead of its neighbours by
// recomputing a halo.  Iteration k+1 trails iteration k (its input state) by
// three row pairs behind per-band progress counters.  Blocks are ordered
// (image, iteration, band), so every wait is on a block dispatched earlier or
// on a neighbour of the same iteration, and a launch holds only as many
// images as are resident at once.
//
// Lane = UV column (WB_OWN own columns and WB_HALO halo columns each side), the prev / cur /
// next chroma rows in registers and the neighbour columns by whole-wave DPP
// shifts (wave_shr / wave_shl), so a step has no workgroup barrier and no
// LDS row traffic -- only the gamma tables stay in LDS.  The band's edge
// lanes read garbage neighbours, which eats one halo column per step (through
// prev, the only row this iteration produces itself; cur / next / luma come
// from the previous state in memory every step), so every WB_HALO row pairs
// the halo lanes reload prev from the neighbour bands' updated row above:
// since round 6 from 8-B {values, row tag} granules of the neighbours' own
// columns, written as each WB_HALO-th row is made and polled by tag (before:
// the neighbours' progress words after their store drains, then the row --
// a drain and two dependent round trips a reload; iteration 0's walk 1,614
// -> 1,528 µs at 4096^2).
// WB_PUB: row pairs between progress publications (each a store drain),
// for the next iteration's input waits only since round 6 (the halo reloads
// take the neighbours' edge granules): 16 / 32 / 64 -> C5 SharpYUV
// 1.92-1.94 / 1.89-1.92 / 1.95 ms
constexpr int WB_OWN = 32, WB_HALO = (64 - WB_OWN) / 2, WB_PUB = 32;
static_assert(WB_OWN + 2 * WB_HALO == 64, "wave band layout");

// (bound_ctrl: the wave's end lanes, always halo lanes, read 0 -- no register to initialise)
__device__ __forceinline__ int dpp_from_left(int v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true); }   // wave_shr:1: lane i <- i - 1
__device__ __forceinline__ int dpp_from_right(int v) { return __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true); }  // wave_shl:1: lane i <- i + 1

// the gray value of linear RGB (gray() for inputs in [0, 65535] -- sRGB's
// linear values and every gamma value: the weights sum to 65536, so the sum
// fits 32 bits unsigned)
// a * b + c on the 24-bit multiplier (full rate, where v_mul_lo_u32 is
// quarter rate): a, b < 2^24 and the result < 2^32 at every call
__device__ __forceinline__ uint32_t mad_u24(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t gray_u32(uint32_t r, uint32_t g, uint32_t b) {
  return mad_u24(r, 13933u, mad_u24(g, 46871u, mad_u24(b, 4732u, 32768u))) >> 16;
}
// from_lin for the walk: fromLinearSrgb's interpolation on the 24-bit
// multiplier (the table is non-decreasing, so v1 - v0 >= 0, and
// (v1 - v0) * x + 64 < 2^17)
template <bool LUT>
__device__ __forceinline__ int from_lin_w(const uint32_t* l2g, const uint16_t* lut, int n, uint32_t v) {
  if (LUT) return lut[min(v, (uint32_t)(n - 1))];
  const uint32_t pos = v >> 7, x = v & 127u;
  const uint32_t v0 = l2g[pos] >> 6, v1 = l2g[pos + 1] >> 6;
  return (int)(v0 + (mad_u24(v1 - v0, x, 64u) >> 7));
}
// a 32-bit word at a wave-uniform base + uniform byte offset + this lane's
// byte offset: the uniform part stays in SGPRs (global_load saddr + a 32-bit
// VGPR offset) instead of a 64-bit address per lane and load
template <typename T>
__device__ __forceinline__ const uint32_t* at(const T* base, uint32_t ubytes, uint32_t lbytes) {
  return reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(base) + ubytes + lbytes);
}
// (the lane offsets are laundered once a step: hoisted out of the walk, base
// + lane offset would become a 64-bit per-lane pointer and every load a 64-bit add)
__device__ __forceinline__ void launder_v(uint32_t& v) { asm volatile("" : "+v"(v)); }

// The band walk is split between the workgroup's two waves (round 4): wave A
// (ROLE 0) makes row j of each row pair -- the Gauss-Seidel chain: it reads
// prev, the row pair above's updated chroma -- and the chroma update; wave B
// (ROLE 1) makes row j + 1, which reads only the input state (cur and next),
// so it runs ahead of A and hands A, per row pair and column, its two
// pixels' linear RGB sums through an LDS ring (XD row pairs deep).  A's
// step is then half the interpolation, half the gamma lookups and half the
// luma update of the one-wave walk: the walk was issue-bound (one wave alone
// on its SIMD, ~650 instructions a row pair).
constexpr int XD = WB_PUB <= 16 ? 16 : 32;  // exchange ring depth, in row pairs (>= WB_PUB: see the drain hand-shake)
struct SharpX {
  uint4 sum[XD][64];  // B's row j + 1: the sums of its two pixels' linear R, G, B per column lane
  int prog_b;         // row pairs B has put into sum[]
  int prog_a;         // row pairs A has taken out of sum[]
  int drained_b;      // row pairs whose luma stores B has drained (for A's progress publication)
};
__device__ __forceinline__ int lds_acquire(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// One band of one iteration, one row of each row pair (ROLE).  EDGE: the
// band's lanes include column 0 or column uvw - 1 (the reference's filter2
// at the plane's edges); the other bands run without those selects.
template <bool LUT, bool EDGE, int ROLE>
__device__ __forceinline__ void sharp_wave_band(const SharpArgs& a, const SharpTabs& t, SharpX& x, int nb, int band,
                                                int it, int img) {
  const int lane = threadIdx.x & 63;
  const int uvw = a.uvw, uvh = a.uvh, w = a.w, rs = a.uv_rs;
  const int c = band * WB_OWN - WB_HALO + lane;  // this lane's UV column
  const bool act = c >= 0 && c < uvw;
  const bool own = act && lane >= WB_HALO && lane < WB_HALO + WB_OWN;
  const int cl = act ? c : 0;  // a valid column for address arithmetic
  const uint16_t* in_y = a.best_y + img * a.img_y + it * a.state_y;
  uint16_t* out_y = const_cast<uint16_t*>(in_y) + a.state_y;
  const int16_t* in_uv = a.best_uv + img * a.img_uv + it * a.state_uv;
  int16_t* out_uv = const_cast<int16_t*>(in_uv) + a.state_uv;
  const uint16_t* ty = a.target_y + img * a.img_y;
  const int16_t* tuv = a.target_uv + img * a.img_uv;
  int* prog_img = a.prog + (int64_t)img * 4 * nb;  // [iteration][band]: row pairs finished
  int* prog_out = prog_img + it * nb + band;
  uint64_t* hand_it = a.hand + ((int64_t)img * 4 + it) * nb * 2 * WB_OWN;  // this iteration's bands' edge granules
  bool timed_out = false;  // wave-uniform
  // (WG_TIMELINES builds) s_memrealtime (100 MHz) at the walk's start and
  // end, and the ticks spent in the two kinds of dependency wait
  WG_IF_TIMELINES(const uint64_t t_walk = __builtin_amdgcn_s_memrealtime(); uint64_t gw_ticks = 0, gw_n = 0, lw_ticks = 0, lw_n = 0;)
  // byte offsets inside one state plane fit 32 bits (a 16383^2 image's Y
  // state is 537 MB): 32-bit scalar row offsets, not 64-bit products
  const uint32_t uv_row_bytes = 2u * (uint32_t)rs, y_row_bytes = 2u * (uint32_t)w;

  // wait (the whole wave, on one wave-uniform address) until band bb of
  // iteration ii has finished `need` row pairs; the progress seen (uvh for a band that does not exist)
  // (WG_BOUNDS) every work-buffer access of the walk checked against the buffer
  auto ld_w = [&](const uint32_t* p, const char* site) -> uint32_t {
    return WG_CHK(p, 4, a.work0, a.work_n, site) ? ld_sc1(p) : 0u;
  };
  auto ld_t = [&](const uint32_t* p, const char* site) -> uint32_t {
    return WG_CHK(p, 4, a.work0, a.work_n, site) ? *p : 0u;
  };
  auto wait_for = [&](int ii, int bb, int need) -> int {
    if (bb < 0 || bb >= nb || timed_out) return uvh;
    const int* p = prog_img + ii * nb + bb;
    if (!WG_CHK(p, 4, a.work0, a.work_n, "k_sharp_wave prog load")) return uvh;
    const uint64_t t0 = wg::wait_clock();
    for (uint32_t k = 0;; k++) {
      const int v = __builtin_amdgcn_readfirstlane((int)ld_sc1(p));
      if (v >= need) {
        WG_IF_TIMELINES(if (k > 0) { gw_ticks += wg::wait_clock() - t0; gw_n++; })
        return v;
      }
      if ((k & 63) == 63 && wg::wait_clock() - t0 > SPIN_TICKS) {
        timed_out = true;
        return uvh;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  };
  // the same for the other wave's LDS progress word
  auto wait_lds = [&](const int* p, int need) {
    if (timed_out || __builtin_amdgcn_readfirstlane(lds_acquire(p)) >= need) return;
    const uint64_t t0 = wg::wait_clock();
    for (uint32_t k = 0;; k++) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_readfirstlane(lds_acquire(p)) >= need) {
        WG_IF_TIMELINES(lw_ticks += wg::wait_clock() - t0; lw_n++;)
        return;
      }
      if ((k & 63) == 63 && wg::wait_clock() - t0 > SPIN_TICKS) {
        timed_out = true;
        return;
      }
    }
  };
  int seen_in = it == 0 ? uvh : 0;  // input state rows known ready (iteration it-1, bands band-1..band+1)
  auto wait_input = [&](int need) {
    if (seen_in < need) {
      int m = uvh;
      for (int d = -1; d <= 1; d++) m = min(m, wait_for(it - 1, band + d, need));
      seen_in = m;
    }
  };
  // A chroma row of 3 int16 channels at this lane's column, from a state row.
  // The loads are unconditional (clamped columns / rows) and keep the raw
  // zero-extended halves: a load inside a branch, or one whose value is
  // sign-extended right away, makes the compiler wait for it there, which
  // would serialise the prefetch two row pairs ahead.
  // 16-bit values travel as the aligned 32-bit word holding them (a 16-bit
  // load's result gets masked right away, which again forces the wait):
  // element e of a 4-byte-aligned state base is in word e >> 1, half e & 1.
  // Rows are 16-byte aligned, so a channel's word and half depend only on
  // the column and the channel: the lane's byte offsets lo_uv / half shifts
  // hs, fixed for the walk.  The other half may be a neighbour's value being
  // stored concurrently: it is never used.
  int hs[3];
  uint32_t lo_uv[3], st_uv[3];
#pragma unroll
  for (int ch = 0; ch < 3; ch++) {
    hs[ch] = 16 * ((ch * uvw + cl) & 1);
    lo_uv[ch] = 4u * (uint32_t)((ch * uvw + cl) >> 1);
    st_uv[ch] = 2u * (uint32_t)(ch * uvw + cl);
  }
  uint32_t lo_y = 4u * (uint32_t)cl;  // the luma pair at x = 2cl, 2cl + 1 of a row
  struct Row {
    uint32_t v[3];
  };
  auto load_row = [&](int row) {
    Row r;
    const uint32_t ub = (uint32_t)min(row, uvh - 1) * uv_row_bytes;  // clamped: the last row pair's next is its cur
#pragma unroll
    for (int ch = 0; ch < 3; ch++) r.v[ch] = ld_w(at(in_uv, ub, lo_uv[ch]), "k_sharp_wave in_uv");
    return r;
  };
  // this role's luma row of a row pair: the input state's and the target's
  // pixel pair, and (A) the chroma targets
  struct In {
    uint32_t y, ty, tuv[ROLE == 0 ? 3 : 1];
  };
  auto load_in = [&](int jp) {
    In r;
    const int jc = min(jp, uvh - 1);
    const uint32_t yb = (uint32_t)(2 * jc + ROLE) * y_row_bytes;
    r.y = ld_w(at(in_y, yb, lo_y), "k_sharp_wave in_y");
    r.ty = ld_t(at(ty, yb, lo_y), "k_sharp_wave target_y");
    if constexpr (ROLE == 0) {
      const uint32_t ub = (uint32_t)jc * uv_row_bytes;
#pragma unroll
      for (int ch = 0; ch < 3; ch++) r.tuv[ch] = ld_t(at(tuv, ub, lo_uv[ch]), "k_sharp_wave target_uv");
    }
    return r;
  };
  // the signed 16-bit value of this column's channel ch in a loaded word
  auto sx16 = [&](uint32_t v, int ch) { return __builtin_amdgcn_sbfe((int)v, hs[ch], 16); };

  uint32_t my_sum = 0;  // |dY| over this lane's pixels: < 2 * 1023 per row pair, uvh <= 2^13
  // rings of four row pairs, indexed by ju % 4 (compile-time after the
  // unrolled loop below, so no register moves): the input state's chroma row
  // and this role's luma / target row of row pairs ju .. ju + 3, prefetched
  // three ahead
  Row R[4];
  In I[4];
  wait_input(min(4, uvh));
  R[0] = load_row(0);
  R[1] = load_row(1);
  R[2] = load_row(2);
  I[0] = load_in(0);
  I[1] = load_in(1);
  I[2] = load_in(2);
  Row P = R[0];  // (A) prev(row 0) = cur(row 0)
  auto step = [&](int ju, const Row& C, const Row& N, Row& pf_row, const In& in_cur, In& pf_in) {
    wait_input(min(ju + 4, uvh));  // UV row ju + 3 and luma pair ju + 3 of the input state
    if constexpr (ROLE == 0) {
      if (ju > 0 && ju % WB_HALO == 0) {
        // the halo lanes' prev: the neighbours' updated row ju - 1, polled
        // straight from their edge granules (tag ju: no progress word, no
        // store drain between the bands)
        const bool need = act && !own;
        const uint64_t* g = hand_it + (int64_t)((lane < WB_HALO ? band - 1 : band + 1) * 2 + ((ju / WB_HALO) & 1)) * WB_OWN +
                            (lane < WB_HALO ? lane + WB_HALO : lane - WB_HALO - WB_OWN);
        uint64_t v = 0;
        if (need && WG_CHK(g, 8, a.work0, a.work_n, "k_sharp_wave halo")) v = ld_sc1_64(g);
        if (__builtin_amdgcn_ballot_w64(need && (int)(v >> 48) != ju)) {
          const uint64_t t0 = wg::wait_clock();
          for (uint32_t k = 0;; k++) {
            __builtin_amdgcn_s_sleep(1);
            if (need && (int)(v >> 48) != ju && WG_CHK(g, 8, a.work0, a.work_n, "k_sharp_wave halo")) v = ld_sc1_64(g);
            if (!__builtin_amdgcn_ballot_w64(need && (int)(v >> 48) != ju)) break;
            if ((k & 63) == 63 && wg::wait_clock() - t0 > SPIN_TICKS) {
              timed_out = true;
              break;
            }
          }
          WG_IF_TIMELINES(gw_ticks += wg::wait_clock() - t0; gw_n++;)
        }
        if (need) {
#pragma unroll
          for (int ch = 0; ch < 3; ch++) P.v[ch] = (uint32_t)(uint16_t)(v >> (16 * ch)) << hs[ch];
        }
      }
    } else {
      wait_lds(&x.prog_a, ju - XD + 1);  // A has taken ring slot ju % XD's previous row pair
    }
    const int j = 2 * ju;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
      launder_v(lo_uv[ch]);
      launder_v(st_uv[ch]);
    }
    launder_v(lo_y);
    pf_row = load_row(ju + 3);
    pf_in = load_in(ju + 3);
    // (A) B's sums of this row pair, read now and used after A's own half:
    // B's progress word first (acquire, pairing with B's release of it),
    // then the slot, with no wait between, so a B that is ahead -- the usual
    // case -- costs no round trip on A's chain.  A workgroup-scope acquire of
    // an LDS word adds no instruction on gfx950 (LDS accesses of a wave
    // retire in order); it keeps the compiler from hoisting the slot read.
    uint4 sb = make_uint4(0, 0, 0, 0);
    int pb = 0;
    if constexpr (ROLE == 0) {
      pb = __hip_atomic_load(&x.prog_b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
      asm volatile("" ::: "memory");
      sb = x.sum[ju % XD][lane];
    }
    // interpolateTwoRows (:322-359) for pixels x = 2c, 2c + 1 of row j (A:
    // from cur and prev) or j + 1 (B: from cur and next)
    const Row& O = ROLE == 0 ? P : N;
    int iv[2][3];
    const int by0 = in_cur.y & 0xffff, by1 = in_cur.y >> 16;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
      const int a1 = sx16(C.v[ch], ch), b1 = sx16(O.v[ch], ch);
      const int a0 = dpp_from_left(a1), b0 = dpp_from_left(b1);
      const int a2 = dpp_from_right(a1), b2 = dpp_from_right(b1);
      int e0, e1;
      if (EDGE && c == 0) e0 = (a1 * 3 + b1 + 2) >> 2;  // filter2(cur[0], prev / next[0])
      else e0 = (a1 * 9 + a0 * 3 + b1 * 3 + b0 + 8) >> 4;
      if (EDGE && c == uvw - 1) e1 = (a1 * 3 + b1 + 2) >> 2;  // x = w-1: filter2(cur[uvw-1], prev / next[uvw-1])
      else e1 = (a1 * 9 + a2 * 3 + b1 * 3 + b2 + 8) >> 4;
      iv[0][ch] = clip_bd(by0 + e0);
      iv[1][ch] = clip_bd(by1 + e1);
    }
    // updateW -> bestRGBY, sharpYUVUpdateY (:361-381)
    uint32_t lin[2][3];
    int ny[2];
#pragma unroll
    for (int cc = 0; cc < 2; cc++) {
#pragma unroll
      for (int ch = 0; ch < 3; ch++) lin[cc][ch] = to_linear(t.g2l, iv[cc][ch]);
      // (the other transfer functions' linear values reach ~72k: 64-bit gray)
      const uint32_t g = LUT ? (uint32_t)gray(lin[cc][0], lin[cc][1], lin[cc][2]) : gray_u32(lin[cc][0], lin[cc][1], lin[cc][2]);
      const int yv = from_lin_w<LUT>(t.l2g, a.lut, a.lut_n, g);
      const int d = (int)((in_cur.ty >> (16 * cc)) & 0xffff) - yv;
      ny[cc] = clip_bd((cc ? by1 : by0) + d);
      my_sum += (uint32_t)abs(d);
    }
    const uint32_t ynew = (uint32_t)ny[0] | (uint32_t)ny[1] << 16;
    uint8_t* oy = reinterpret_cast<uint8_t*>(out_y) + (uint32_t)(j + ROLE) * y_row_bytes;
    if constexpr (ROLE == 1) {
      // hand A this row pair's linear sums, then store the luma row
      x.sum[ju % XD][lane] = make_uint4(lin[0][0] + lin[1][0], lin[0][1] + lin[1][1], lin[0][2] + lin[1][2], 0u);
      if (lane == 0) lds_release(&x.prog_b, ju + 1);
      if (own && WG_CHK(oy + lo_y, 4, a.work0, a.work_n, "k_sharp_wave out_y")) st_sc1(oy + lo_y, ynew);
      if ((ju + 1) % WB_PUB == 0 || ju + 1 == uvh) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) lds_release(&x.drained_b, ju + 1);
      }
    } else {
      // updateChroma -> bestRGBUV, sharpYUVUpdateRGB (:383-388), with B's
      // sums of row j + 1
      if (__builtin_amdgcn_readfirstlane(pb) < ju + 1) {  // B was not ahead: wait, then read the slot again
        wait_lds(&x.prog_b, ju + 1);
        sb = x.sum[ju % XD][lane];
      }
      if (lane == 0) lds_release(&x.prog_a, ju + 1);  // (the sums are in registers: the slot is free)
      const uint32_t bs[3] = {sb.x, sb.y, sb.z};
      int rgbv[3];
#pragma unroll
      for (int ch = 0; ch < 3; ch++)
        rgbv[ch] = from_lin_w<LUT>(t.l2g, a.lut, a.lut_n, (lin[0][ch] + lin[1][ch] + bs[ch] + 2) >> 2);
      const int gv = (int)gray_u32(rgbv[0], rgbv[1], rgbv[2]);
      int upd[3];
#pragma unroll
      for (int ch = 0; ch < 3; ch++) {
        const int16_t srcv = (int16_t)(rgbv[ch] - gv);
        const int16_t d = (int16_t)(sx16(in_cur.tuv[ch], ch) - srcv);
        upd[ch] = (int16_t)(sx16(C.v[ch], ch) + d);
      }
      // publish this band's own columns of the updated UV row ju and luma row j (write-through)
      if (own) {
        uint8_t* ob = reinterpret_cast<uint8_t*>(out_uv) + (uint32_t)ju * uv_row_bytes;
#pragma unroll
        for (int ch = 0; ch < 3; ch++)
          if (WG_CHK(ob + st_uv[ch], 2, a.work0, a.work_n, "k_sharp_wave out_uv")) st_sc1_16(ob + st_uv[ch], (uint16_t)upd[ch]);
        if (WG_CHK(oy + lo_y, 4, a.work0, a.work_n, "k_sharp_wave out_y")) st_sc1(oy + lo_y, ynew);
      }
#pragma unroll
      for (int ch = 0; ch < 3; ch++) P.v[ch] = (uint32_t)(uint16_t)upd[ch] << hs[ch];  // prev <- the updated cur (in its half)
      if ((ju + 1) % WB_HALO == 0 && ju + 1 < uvh && own) {
        // the neighbours' next halo reload: this row's own columns as 8-B
        // granules, one write-through store each (untorn: the tag ju + 1
        // comes with the values); two slots, so a slot is rewritten only
        // after both neighbours have passed the reload that read it
        uint64_t* gm = hand_it + (int64_t)(band * 2 + (((ju + 1) / WB_HALO) & 1)) * WB_OWN + (lane - WB_HALO);
        const uint64_t gv = (uint64_t)(uint16_t)upd[0] | (uint64_t)(uint16_t)upd[1] << 16 | (uint64_t)(uint16_t)upd[2] << 32 |
                            (uint64_t)(ju + 1) << 48;
        if (WG_CHK(gm, 8, a.work0, a.work_n, "k_sharp_wave hand store"))
          __hip_atomic_store(gm, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if ((ju + 1) % WB_PUB == 0 || ju + 1 == uvh) {
        // publish row pairs <= ju once this wave's stores of them are done,
        // and B's (a drain also waits for the loads in flight, so only every
        // WB_PUB steps)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wait_lds(&x.drained_b, ju + 1);
        if (lane == 0 && WG_CHK(prog_out, 4, a.work0, a.work_n, "k_sharp_wave prog store")) st_sc1(prog_out, (uint32_t)(ju + 1));
      }
    }
  };
  for (int j0 = 0; j0 < uvh; j0 += 4) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (j0 + k >= uvh) break;  // wave-uniform
      step(j0 + k, R[k], R[(k + 1) & 3], R[(k + 3) & 3], I[k], I[(k + 3) & 3]);
    }
  }
  // the band's share of the iteration's |dY| sum over its own columns
  // (:254-263); k_sharp_final applies the exit rule
  unsigned long long sm = own ? my_sum : 0u;
  for (int off = 32; off > 0; off >>= 1) sm += __shfl_down(sm, off, 64);
  if (lane == 0 && WG_CHK(a.sums + img * 4 + it, 8, a.work0, a.work_n, "k_sharp_wave sums") &&
      WG_CHK(a.iters + img, 4, a.work0, a.work_n, "k_sharp_wave iters")) {
    atomicAdd(reinterpret_cast<unsigned long long*>(a.sums + img * 4 + it), sm);
    if (timed_out) a.iters[img] = -1;
  }
  WG_IF_TIMELINES(if (lane == 0) {
    uint64_t* st = a.stamps + 4 * (2 * (((int64_t)img * 4 + it) * nb + band) + ROLE);
    st[0] = t_walk;
    st[1] = __builtin_amdgcn_s_memrealtime();
    st[2] = gw_ticks | gw_n << 32;
    st[3] = lw_ticks | lw_n << 32;
  })
}

template <bool LUT>
__global__ __launch_bounds__(128) void k_sharp_wave(SharpArgs a, int nb) {
  __shared__ SharpTabs t;
  __shared__ SharpX x;
  const int blk = blockIdx.x, band = blk % nb, it = (blk / nb) & 3, img = blk / (4 * nb);
  if (img >= a.n_img) return;  // uniform over the block
  if (threadIdx.x == 0) x.prog_b = x.prog_a = x.drained_b = 0;
  load_tabs(t, a.tabs);  // (its barrier also orders the counters' initialisation)
  const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the band's lanes cover columns band * WB_OWN - WB_HALO .. + 63
  const int c0 = band * WB_OWN - WB_HALO;
  const bool edge = c0 <= 0 || c0 + 63 >= a.uvw - 1;
  if (role == 0) {
    if (edge) sharp_wave_band<LUT, true, 0>(a, t, x, nb, band, it, img);
    else sharp_wave_band<LUT, false, 0>(a, t, x, nb, band, it, img);
  } else {
    if (edge) sharp_wave_band<LUT, true, 1>(a, t, x, nb, band, it, img);
    else sharp_wave_band<LUT, false, 1>(a, t, x, nb, band, it, img);
  }
}

// The iterations the reference runs (:224-264): 0 and 1 always; after
// iteration k >= 1 it stops when sum_k < 3wh or sum_k > sum_{k-1}.
__device__ __forceinline__ int sharp_iters(const uint64_t* sums, uint64_t threshold) {
  for (int k = 1; k < 4; k++)
    if (sums[k] < threshold || sums[k] > sums[k - 1]) return k + 1;
  return 4;
}

struct FinalArgs {
  const uint16_t* best_y;
  const int16_t* best_uv;
  const uint64_t* sums;
  int* iters;
  uint8_t* y;
  uint8_t* u;
  uint8_t* v;
  int64_t img_y, state_y, img_uv, state_uv, out_y_pitch, out_uv_pitch;
  int y_stride, uv_stride, width, height, w, uvw, uvh, uv_rs;
  int m[12];
  const uint8_t* work0;  // (WG_BOUNDS) the work buffer and its size
  int64_t work_n;
};

// convertWRGBToYUV (:390-432) of the state the reference stops at: thread
// per Y pixel; threads of even (x, y) also produce the U / V sample.
__global__ __launch_bounds__(256) void k_sharp_final(FinalArgs a, int n_img) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)a.width * a.height;
  if (gid >= per * n_img) return;
  const int img = (int)(gid / per);
  const int64_t p = gid - img * per;
  const int j = (int)(p / a.width), i = (int)(p - (int64_t)j * a.width);
  const int n_it = sharp_iters(a.sums + img * 4, (uint64_t)3 * a.w * ((a.height + 1) & ~1));
  if (p == 0 && a.iters[img] >= 0) a.iters[img] = n_it;
  const uint16_t* by = a.best_y + img * a.img_y + n_it * a.state_y;  // state n_it = after iteration n_it - 1
  const int16_t* buv = a.best_uv + img * a.img_uv + n_it * a.state_uv;
  constexpr int SHIFT = 16 + SFIX;
  const int64_t rounder = (int64_t)1 << (SHIFT - 1);
  const int uvi = (j / 2) * a.uv_rs + (i >> 1);
  if (!WG_CHK(by + (int64_t)j * a.w + i, 2, a.work0, a.work_n, "k_sharp_final best_y") ||
      !WG_CHK(buv + uvi, 2, a.work0, a.work_n, "k_sharp_final best_uv") ||
      !WG_CHK(buv + uvi + 2 * a.uvw, 2, a.work0, a.work_n, "k_sharp_final best_uv") ||
      !WG_CHK(a.y + img * a.out_y_pitch + (int64_t)j * a.y_stride + i, 1, a.y, (int64_t)n_img * a.out_y_pitch,
              "k_sharp_final y") ||
      !WG_CHK(a.u + img * a.out_uv_pitch + (int64_t)(j >> 1) * a.uv_stride + (i >> 1), 1, a.u,
              (int64_t)n_img * a.out_uv_pitch, "k_sharp_final uv"))
    return;
  const int64_t wv = by[(int64_t)j * a.w + i];
  const int64_t r = buv[uvi] + wv, g = buv[uvi + a.uvw] + wv, b = buv[uvi + 2 * a.uvw] + wv;
  const int64_t yv = (int64_t)a.m[0] * r + (int64_t)a.m[1] * g + (int64_t)a.m[2] * b + ((int64_t)a.m[3] << SFIX) + rounder;
  a.y[img * a.out_y_pitch + (int64_t)j * a.y_stride + i] = (uint8_t)min(max((int)(int32_t)(yv >> SHIFT), 0), 255);
  if (((i | j) & 1) == 0) {
    const int64_t ur = buv[uvi], ug = buv[uvi + a.uvw], ub = buv[uvi + 2 * a.uvw];
    const int64_t uu = (int64_t)a.m[4] * ur + (int64_t)a.m[5] * ug + (int64_t)a.m[6] * ub + ((int64_t)a.m[7] << SFIX) + rounder;
    const int64_t vv = (int64_t)a.m[8] * ur + (int64_t)a.m[9] * ug + (int64_t)a.m[10] * ub + ((int64_t)a.m[11] << SFIX) + rounder;
    const int64_t o = img * a.out_uv_pitch + (int64_t)(j >> 1) * a.uv_stride + (i >> 1);
    a.u[o] = (uint8_t)min(max((int)(int32_t)(uu >> SHIFT), 0), 255);
    a.v[o] = (uint8_t)min(max((int)(int32_t)(vv >> SHIFT), 0), 255);
  }
}

// convertStandard (:68-115): thread = one U/V sample; it also writes the up
// to four Y pixels of its 2x2 block (rgbToYUVComponent, clipU8)
struct StdArgs {
  const uint8_t* rgb;
  uint8_t *y, *u, *v;
  int64_t rgb_pitch, y_pitch, uv_pitch;
  int rgb_stride, y_stride, uv_stride, width, height, uvw, uvh;
  int m[12];
};
__device__ __forceinline__ int yuv_comp(int r, int g, int b, const int* c) {
  const int64_t l = (int64_t)c[0] * r + (int64_t)c[1] * g + (int64_t)c[2] * b + (int64_t)c[3] + (1 << 15);
  return min(max((int)(int32_t)(l >> 16), 0), 255);
}
__global__ __launch_bounds__(256) void k_sharp_standard(StdArgs a, int n_img) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)a.uvw * a.uvh;
  if (gid >= per * n_img) return;
  const int img = (int)(gid / per);
  const int64_t p = gid - img * per;
  const int j = (int)(p / a.uvw), i = (int)(p - (int64_t)j * a.uvw);
  const uint8_t* rgb = a.rgb + img * a.rgb_pitch;
  int sr = 0, sg = 0, sb = 0, n = 0;
  for (int dy = 0; dy < 2; dy++) {
    const int yy = 2 * j + dy;
    if (yy >= a.height) continue;
    for (int dx = 0; dx < 2; dx++) {
      const int xx = 2 * i + dx;
      if (xx >= a.width) continue;
      const uint8_t* px = rgb + (int64_t)yy * a.rgb_stride + 3 * xx;
      sr += px[0];
      sg += px[1];
      sb += px[2];
      n++;
      a.y[img * a.y_pitch + (int64_t)yy * a.y_stride + xx] = (uint8_t)yuv_comp(px[0], px[1], px[2], a.m);
    }
  }
  const int ar = (sr + n / 2) / n, ag = (sg + n / 2) / n, ab = (sb + n / 2) / n;
  const int64_t o = img * a.uv_pitch + (int64_t)j * a.uv_stride + i;
  a.u[o] = (uint8_t)yuv_comp(ar, ag, ab, a.m + 4);
  a.v[o] = (uint8_t)yuv_comp(ar, ag, ab, a.m + 8);
}

}  // namespace

namespace wg {
// sharpyuv_host.cpp: g2l[1026] then l2g[514] (uint32), then for tf != sRGB
// the direct LinearToGamma table (uint16, *lut_n entries)
const void* sharpyuv_tables_device(int tf, int* lut_n);
}

namespace {
struct SharpLayout {
  size_t y_elems, uv_elems, img_y, img_uv, bytes_img;
  int uv_rs;
};
SharpLayout sharp_layout(int width, int height) {
  SharpLayout L;
  const size_t w = (size_t)((width + 1) & ~1), h = (size_t)((height + 1) & ~1);
  L.uv_rs = (int)((3 * (w / 2) + 7) & ~(size_t)7);  // UV row: 3 planes, padded to 16 bytes
  L.y_elems = (w * h + 7) & ~(size_t)7;
  L.uv_elems = (size_t)L.uv_rs * (h / 2);
  L.img_y = (NSTATE + 1) * L.y_elems;  // NSTATE states + the target
  L.img_uv = (NSTATE + 1) * L.uv_elems;
  L.bytes_img = 2 * (L.img_y + L.img_uv);
  return L;
}
// the tail after the images: sums [n][4] u64 | iters [n] | prog [n][4][bands]
// | (8-B aligned) hand [n][4][bands][2][WB_OWN] | (WG_TIMELINES) stamps
size_t sharp_hand_offset(int n, int nb) { return ((size_t)n * (32 + 4 + 16 * nb) + 7) & ~(size_t)7; }
// one-wave column bands of one refinement iteration (k_sharp_wave)
int sharp_bands(int width) {
  const int uvw = ((width + 1) & ~1) / 2;
  return (uvw + WB_OWN - 1) / WB_OWN;
}
}  // namespace

extern "C" size_t wg_sharpyuv_work_bytes(int32_t width, int32_t height, int32_t n_images) {
  if (width <= 0 || height <= 0 || n_images <= 0) return 0;
  const SharpLayout L = sharp_layout(width, height);
  const int nb = sharp_bands(width);
  // (+ the timeline records: 32 B a wave, two waves a block, 4 * nb blocks an image)
  // (+ the edge granules: 2 slots of WB_OWN 8-B granules per band and iteration)
  return n_images * L.bytes_img + sharp_hand_offset(n_images, nb) + (size_t)n_images * 4 * nb * 2 * WB_OWN * 8 + 16
         WG_IF_TIMELINES(+(size_t)n_images * 4 * nb * 64);
}

extern "C" int wg_sharpyuv_convert_ex(const uint8_t* rgb, int32_t width, int32_t height, int32_t rgb_stride,
                                      int64_t rgb_pitch, const int32_t* matrix_host, int32_t transfer,
                                      int32_t sharp_enabled, int32_t n_images, uint8_t* y, int32_t y_stride,
                                      int64_t y_pitch, uint8_t* u, uint8_t* v, int32_t uv_stride, int64_t uv_pitch,
                                      void* work, void* stream) {
  WG_REQUIRE(rgb && matrix_host && y && u && v && width > 0 && height > 0 && n_images > 0);
  // (the walk's in-plane byte offsets are 32-bit: 2 B a pixel, < 2^31)
  WG_REQUIRE((int64_t)((width + 1) & ~1) * ((height + 1) & ~1) < (1ll << 30));
  WG_REQUIRE(rgb_stride >= 3 * width && y_stride >= width && uv_stride >= (width + 1) / 2);
  hipStream_t s = wg::as_stream(stream);
  if (!sharp_enabled) {  // convertStandard (sharpyuv.go:68-115)
    StdArgs sa;
    sa.rgb = rgb;
    sa.y = y;
    sa.u = u;
    sa.v = v;
    sa.rgb_pitch = rgb_pitch;
    sa.y_pitch = y_pitch;
    sa.uv_pitch = uv_pitch;
    sa.rgb_stride = rgb_stride;
    sa.y_stride = y_stride;
    sa.uv_stride = uv_stride;
    sa.width = width;
    sa.height = height;
    sa.uvw = (width + 1) >> 1;
    sa.uvh = (height + 1) >> 1;
    for (int k = 0; k < 12; k++) sa.m[k] = matrix_host[k];
    const int64_t cells = (int64_t)sa.uvw * sa.uvh * n_images;
    hipLaunchKernelGGL(k_sharp_standard, dim3(wg::blocks_for(cells, 256)), dim3(256), 0, s, sa, n_images);
    return wg::check_launch("k_sharp_standard");
  }
  WG_REQUIRE(work && (reinterpret_cast<uintptr_t>(work) & 15) == 0);
  // H.273 codes the reference implements (gamma.go:11-28); others give 0 there too
  WG_REQUIRE(transfer >= 0 && transfer <= 18);
  const int w = (width + 1) & ~1, h = (height + 1) & ~1;
  const int uvw = w / 2, uvh = h / 2;
  const int nb = sharp_bands(width);
  int lut_n = 0;
  const void* tabs = wg::sharpyuv_tables_device(transfer, &lut_n);
  if (!tabs) return WG_EHIP;
  const bool lut = transfer != 13;
  const SharpLayout L = sharp_layout(width, height);
  uint8_t* base = static_cast<uint8_t*>(work);
  SharpArgs a;
  a.rgb = rgb;
  a.rgb_pitch = rgb_pitch;
  a.rgb_stride = rgb_stride;
  a.width = width;
  a.height = height;
  a.w = w;
  a.h = h;
  a.uvw = uvw;
  a.uvh = uvh;
  a.uv_rs = L.uv_rs;
  // per image: Y states 0..4 | target Y | UV states 0..4 | target UV; then
  // sums [n][4] u64 | prog [n][4] | iters [n]
  a.best_y = reinterpret_cast<uint16_t*>(base);
  a.target_y = a.best_y + NSTATE * L.y_elems;
  a.best_uv = reinterpret_cast<int16_t*>(base + 2 * L.img_y);
  a.target_uv = a.best_uv + NSTATE * L.uv_elems;
  a.img_y = (int64_t)(L.bytes_img / 2);
  a.img_uv = (int64_t)(L.bytes_img / 2);
  a.state_y = (int64_t)L.y_elems;
  a.state_uv = (int64_t)L.uv_elems;
  a.tabs = static_cast<const SharpTabs*>(tabs);
  a.lut = reinterpret_cast<const uint16_t*>(static_cast<const uint8_t*>(tabs) + sizeof(SharpTabs));
  a.lut_n = lut_n;
  // tail: sums [n][4] u64 | iters [n] | prog [n][4][bands] | hand (sharp_hand_offset)
  uint8_t* tail = base + n_images * L.bytes_img;
  a.sums = reinterpret_cast<uint64_t*>(tail);
  a.iters = reinterpret_cast<int*>(tail + (size_t)n_images * 32);
  a.prog = a.iters + n_images;
  a.hand = reinterpret_cast<uint64_t*>(tail + sharp_hand_offset(n_images, nb));
  a.n_img = n_images;
  a.work0 = base;
  a.work_n = (int64_t)wg_sharpyuv_work_bytes(width, height, n_images);
  // (WG_TIMELINES builds: the records follow the counters, 8-B aligned)
  const size_t tail_n = sharp_hand_offset(n_images, nb) + (size_t)n_images * 4 * nb * 2 * WB_OWN * 8;
  a.stamps = reinterpret_cast<uint64_t*>(tail + tail_n);
  if (hipMemsetAsync(tail, 0, tail_n, s) != hipSuccess)
    return wg::check_launch("hipMemsetAsync(sharpyuv)");
  const int64_t cells = (int64_t)uvw * uvh * n_images;
  if (lut)
    hipLaunchKernelGGL(k_sharp_init<true>, dim3(wg::blocks_for(cells, 256)), dim3(256), 0, s, a, n_images);
  else
    hipLaunchKernelGGL(k_sharp_init<false>, dim3(wg::blocks_for(cells, 256)), dim3(256), 0, s, a, n_images);
  int rc = wg::check_launch("k_sharp_init");
  if (rc != WG_OK) return rc;
  // every wait is on a block of the same launch: launch at most as many
  // images as the device holds at once (4 iterations x nb bands each)
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sharp_wave<false>, 128, 0) != hipSuccess ||
      per_cu <= 0)
    return wg::check_launch("sharpyuv occupancy");
  const int chunk = std::max(1, per_cu * cus / (4 * nb));  // images per launch
  if (4 * nb > per_cu * cus) return wg::invalid("sharpyuv: image too wide for one device's resident workgroups");
  for (int i0 = 0; i0 < n_images; i0 += chunk) {
    SharpArgs c = a;
    c.n_img = std::min(chunk, n_images - i0);
    c.best_y += i0 * a.img_y;
    c.target_y += i0 * a.img_y;
    c.best_uv += i0 * a.img_uv;
    c.target_uv += i0 * a.img_uv;
    c.sums += 4 * i0;
    c.prog += 4 * nb * i0;
    c.hand += (int64_t)4 * nb * 2 * WB_OWN * i0;
    c.iters += i0;
    const unsigned grid = (unsigned)(c.n_img * 4 * nb);
    if (lut)
      hipLaunchKernelGGL(k_sharp_wave<true>, dim3(grid), dim3(128), 0, s, c, nb);
    else
      hipLaunchKernelGGL(k_sharp_wave<false>, dim3(grid), dim3(128), 0, s, c, nb);
    rc = wg::check_launch("k_sharp_wave");
    if (rc != WG_OK) return rc;
  }
  FinalArgs f;
  f.best_y = a.best_y;
  f.best_uv = a.best_uv;
  f.sums = a.sums;
  f.iters = a.iters;
  f.y = y;
  f.u = u;
  f.v = v;
  f.img_y = a.img_y;
  f.state_y = a.state_y;
  f.img_uv = a.img_uv;
  f.state_uv = a.state_uv;
  f.out_y_pitch = y_pitch;
  f.out_uv_pitch = uv_pitch;
  f.y_stride = y_stride;
  f.uv_stride = uv_stride;
  f.width = width;
  f.height = height;
  f.w = w;
  f.uvw = uvw;
  f.uvh = uvh;
  f.uv_rs = L.uv_rs;
  for (int k = 0; k < 12; k++) f.m[k] = matrix_host[k];
  f.work0 = a.work0;
  f.work_n = a.work_n;
  const int64_t px = (int64_t)width * height * n_images;
  hipLaunchKernelGGL(k_sharp_final, dim3(wg::blocks_for(px, 256)), dim3(256), 0, s, f, n_images);
  return wg::check_launch("k_sharp_final");
}

extern "C" int wg_sharpyuv_convert(const uint8_t* rgb, int32_t width, int32_t height, int32_t rgb_stride,
                                   int64_t rgb_pitch, const int32_t* matrix_host, int32_t n_images, uint8_t* y,
                                   int32_t y_stride, int64_t y_pitch, uint8_t* u, uint8_t* v, int32_t uv_stride,
                                   int64_t uv_pitch, void* work, void* stream) {
  return wg_sharpyuv_convert_ex(rgb, width, height, rgb_stride, rgb_pitch, matrix_host, 13, 1, n_images, y, y_stride,
                                y_pitch, u, v, uv_stride, uv_pitch, work, stream);
}

// Iterations each image ran (the reference's count, 2..4), or -1 where a
// pipeline dependency wait timed out (output invalid).  Host-synchronous.
extern "C" int wg_sharpyuv_iterations(const void* work, int32_t width, int32_t height, int32_t n_images, int32_t* out,
                                      void* stream) {
  WG_REQUIRE(work && out && width > 0 && height > 0 && n_images > 0);
  const SharpLayout L = sharp_layout(width, height);
  const uint8_t* tail = static_cast<const uint8_t*>(work) + n_images * L.bytes_img;
  hipStream_t s = wg::as_stream(stream);
  if (hipMemcpyAsync(out, tail + (size_t)n_images * 32, sizeof(int32_t) * n_images, hipMemcpyDeviceToHost, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return wg::check_launch("wg_sharpyuv_iterations");
  for (int i = 0; i < n_images; i++)
    if (out[i] < 0) {
      wg::set_error("sharpyuv: a pipeline dependency wait timed out (output invalid)");
      return WG_EHIP;
    }
  return WG_OK;
}
