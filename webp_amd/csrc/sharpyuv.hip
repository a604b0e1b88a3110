// sharpyuv.hip -- SharpYUV RGB -> YUV420 on gfx950,
// any transfer function and conversion matrix (sharpyuv/sharpyuv.go:39-432),
// and convertStandard (:68-115) when sharpening is off (k_sharp_standard).
//
//   k_sharp_init   import + gray Y, target W, target / initial chroma
//                  residuals (convertSharp phase 1, :196-222): one thread per
//                  2x2 block, fully parallel
//   k_sharp_pipe   the iterative refinement (:224-264).  Each iteration sweeps
//                  the row pairs in order and updates the chroma residuals in
//                  place, so row pair j reads row pair j-1's values from the
//                  SAME iteration (Gauss-Seidel): a sweep is sequential by
//                  construction.  But iteration k+1 at row pair j needs only
//                  iteration k's rows up to j+1, so the four iterations run
//                  as a pipeline: one workgroup per (image, iteration), each
//                  reading state k and writing state k+1 (five states per
//                  image, out of place), iteration k+1 trailing k by three
//                  row pairs behind a progress counter (published one step
//                  late, when every wave has drained its stores).  The early exit
//                  (:254-263) needs each iteration's global |dY| sum; all
//                  four iterations run speculatively and k_sharp_final picks
//                  the state the reference would stop at.  Inside a
//                  workgroup the whole width runs in parallel, the updated
//                  row kept in LDS as the next row's "prev".
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
  int n_img;
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
      c[r][k][0] = px[0] << SFIX;
      c[r][k][1] = px[1] << SFIX;
      c[r][k][2] = px[2] << SFIX;
    }
  }
  uint16_t* by = a.best_y + img * a.img_y;
  uint16_t* ty = a.target_y + img * a.img_y;
  uint32_t lin[2][2][3];
  for (int r = 0; r < 2; r++)
    for (int k = 0; k < 2; k++) {
      const int64_t o = (int64_t)(j + r) * a.w + 2 * i + k;
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
    tuv[ch * a.uvw + i] = d;
    buv[ch * a.uvw + i] = d;
  }
}

constexpr int ITER_THREADS = 1024;
constexpr uint64_t SPIN_TICKS = 200000000ull;  // 2 s of s_memrealtime (100 MHz)

// Hand-off loads / stores between the iteration workgroups: agent-scope
// relaxed atomics, i.e. sc1 (write-through stores, L1-bypassing loads); every
// load of handed-off bytes is one, every store of them too, and the progress
// counter is stored after every wave's vmcnt(0) and a workgroup barrier
// (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ uint32_t ld_sc1(const void* p) {
  return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(void* p, uint32_t v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// phase 2: workgroup = (image, iteration).  Blocks are grouped 32 to eight
// images so that an image's four iterations have equal blockIdx % 8 (one XCD
// under the round-robin placement: a speed matter only) and iteration k's
// block precedes iteration k+1's.  Thread t owns UV columns t + k*1024,
// k < MAX_COLS: 2 covers widths up to 4096, 8 up to 16384.
template <int MAX_COLS, bool LUT>
__global__ __launch_bounds__(ITER_THREADS) void k_sharp_pipe(SharpArgs a) {
  __shared__ SharpTabs t;
  extern __shared__ int16_t rows[];  // prev / cur / next UV rows: 3 rows of uv_rs
  __shared__ unsigned long long part[ITER_THREADS / 64];
  __shared__ int timed_out;
  const int b = blockIdx.x, it = (b & 31) >> 3, img = (b >> 5) * 8 + (b & 7);
  if (img >= a.n_img) return;  // uniform over the block
  load_tabs(t, a.tabs);
  const int tid = threadIdx.x;
  const int uvw = a.uvw, uvh = a.uvh, w = a.w, rs = a.uv_rs;
  const uint16_t* in_y = a.best_y + img * a.img_y + it * a.state_y;
  uint16_t* out_y = const_cast<uint16_t*>(in_y) + a.state_y;
  const int16_t* in_uv = a.best_uv + img * a.img_uv + it * a.state_uv;
  int16_t* out_uv = const_cast<int16_t*>(in_uv) + a.state_uv;
  const uint16_t* ty = a.target_y + img * a.img_y;
  const int16_t* tuv = a.target_uv + img * a.img_uv;
  int* prog_in = a.prog + img * 4 + it - 1;  // iteration it-1 (it > 0)
  int* prog_out = a.prog + img * 4 + it;
  int16_t* lds_row[3] = {rows, rows + rs, rows + 2 * rs};  // rotating prev / cur / next
  const int words = (3 * uvw + 1) >> 1;  // u32 words of a UV row (the padding absorbs the odd one)
  int seen = it == 0 ? uvh : 0;
  if (tid == 0) timed_out = 0;

  // thread 0: wait until iteration it-1 has finished `need` row pairs
  auto wait_rows = [&](int need) {
    if (tid == 0 && seen < need) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (uint32_t k = 0;; k++) {
        seen = (int)ld_sc1(prog_in);
        if (seen >= need) break;
        if ((k & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS) {
          timed_out = 1;
          seen = uvh;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  };

  uint64_t my_sum = 0;
  int pi = 0, ci = 1, ni = 2;
  // rows 0 and 1 of the input state: prev(row 0) = cur(row 0) = row 0
  wait_rows(min(2, uvh));
  __syncthreads();
  for (int i = tid; i < words; i += ITER_THREADS) {
    const uint32_t v0 = ld_sc1(in_uv + 2 * i);
    reinterpret_cast<uint32_t*>(lds_row[ci])[i] = v0;
    reinterpret_cast<uint32_t*>(lds_row[pi])[i] = v0;
    reinterpret_cast<uint32_t*>(lds_row[ni])[i] = uvh > 1 ? ld_sc1(in_uv + rs + 2 * i) : v0;
  }
  // luma pair 0 of the input state; later pairs are loaded one step ahead
  // (and the targets: target luma pair, target chroma of the row)
  uint32_t ycur[MAX_COLS][2], tycur[MAX_COLS][2];
  int16_t tuvcur[MAX_COLS][3];
#pragma unroll
  for (int k = 0; k < MAX_COLS; k++) {
    const int i = tid + k * ITER_THREADS;
    ycur[k][0] = i < uvw ? ld_sc1(in_y + 2 * i) : 0u;
    ycur[k][1] = i < uvw ? ld_sc1(in_y + w + 2 * i) : 0u;
    tycur[k][0] = i < uvw ? *reinterpret_cast<const uint32_t*>(ty + 2 * i) : 0u;
    tycur[k][1] = i < uvw ? *reinterpret_cast<const uint32_t*>(ty + w + 2 * i) : 0u;
    for (int ch = 0; ch < 3; ch++) tuvcur[k][ch] = i < uvw ? tuv[ch * uvw + i] : 0;
  }
  for (int ju = 0; ju < uvh; ju++) {
    wait_rows(min(ju + 3, uvh));  // Y pair ju + 1 and UV row ju + 2 of the input state
    __syncthreads();
    const int16_t* P = lds_row[pi];
    const int16_t* C = lds_row[ci];
    const int16_t* N = lds_row[ni];
    const int j = 2 * ju;
    // prefetch the row after next (the next step's "next") into registers
    const bool have_nn = ju + 2 < uvh;
    uint32_t pf[(MAX_COLS * ITER_THREADS * 3 / 2 + ITER_THREADS - 1) / ITER_THREADS];
    constexpr int PFN = sizeof(pf) / sizeof(pf[0]);
#pragma unroll
    for (int k = 0; k < PFN; k++) {
      const int i = tid + k * ITER_THREADS;
      pf[k] = (have_nn && i < words) ? ld_sc1(in_uv + (int64_t)(ju + 2) * rs + 2 * i) : 0u;
    }
    uint32_t ynext[MAX_COLS][2], tynext[MAX_COLS][2];  // luma pair ju + 1, its targets
    int16_t tuvnext[MAX_COLS][3];
    const bool have_ny = ju + 1 < uvh;
#pragma unroll
    for (int k = 0; k < MAX_COLS; k++) {
      const int i = tid + k * ITER_THREADS;
      const bool ok = have_ny && i < uvw;
      const int64_t yn = (int64_t)(j + 2) * w + 2 * i;
      ynext[k][0] = ok ? ld_sc1(in_y + yn) : 0u;
      ynext[k][1] = ok ? ld_sc1(in_y + yn + w) : 0u;
      tynext[k][0] = ok ? *reinterpret_cast<const uint32_t*>(ty + yn) : 0u;
      tynext[k][1] = ok ? *reinterpret_cast<const uint32_t*>(ty + yn + w) : 0u;
      for (int ch = 0; ch < 3; ch++) tuvnext[k][ch] = ok ? tuv[(int64_t)(ju + 1) * rs + ch * uvw + i] : 0;
    }
    int16_t upd[MAX_COLS][3];  // the updated row: written to LDS only after every thread read P/C/N
    uint32_t ynew[MAX_COLS][2];  // the updated luma pair: stored after the barriers, off the wait below
#pragma unroll
    for (int k = 0; k < MAX_COLS; k++) {
      const int i = tid + k * ITER_THREADS;
      if (i >= uvw) continue;
      // interpolateTwoRows (:322-359) for pixels x = 2i, 2i+1 of rows j, j+1
      int iv[2][2][3];
      const uint32_t r0 = ycur[k][0], r1 = ycur[k][1];
      const int by00 = r0 & 0xffff, by01 = r0 >> 16, by10 = r1 & 0xffff, by11 = r1 >> 16;
      for (int ch = 0; ch < 3; ch++) {
        const int o = ch * uvw;
        const int a1 = C[o + i], b1 = P[o + i], n1 = N[o + i];
        int e0, e1, f0, f1;  // x = 2i: row j / j+1
        if (i == 0) {
          e0 = ((a1 * 3 + b1 + 2) >> 2);  // filter2(cur[0], prev[0])
          f0 = ((a1 * 3 + n1 + 2) >> 2);
        } else {  // v1 of i-1: (a1*9 + a0*3 + b1*3 + b0 + 8) >> 4
          const int a0 = C[o + i - 1], b0 = P[o + i - 1], n0 = N[o + i - 1];
          e0 = (a1 * 9 + a0 * 3 + b1 * 3 + b0 + 8) >> 4;
          f0 = (a1 * 9 + a0 * 3 + n1 * 3 + n0 + 8) >> 4;
        }
        if (i == uvw - 1) {  // x = w-1: filter2(cur[uvw-1], prev[uvw-1])
          e1 = ((a1 * 3 + b1 + 2) >> 2);
          f1 = ((a1 * 3 + n1 + 2) >> 2);
        } else {  // v0 of i: (a0*9 + a1*3 + b0*3 + b1 + 8) >> 4 with a0 = cur[i]
          const int a2 = C[o + i + 1], b2 = P[o + i + 1], n2 = N[o + i + 1];
          e1 = (a1 * 9 + a2 * 3 + b1 * 3 + b2 + 8) >> 4;
          f1 = (a1 * 9 + a2 * 3 + n1 * 3 + n2 + 8) >> 4;
        }
        iv[0][0][ch] = clip_bd(by00 + e0);
        iv[0][1][ch] = clip_bd(by01 + e1);
        iv[1][0][ch] = clip_bd(by10 + f0);
        iv[1][1][ch] = clip_bd(by11 + f1);
      }
      // updateW -> bestRGBY, sharpYUVUpdateY (:361-381)
      uint32_t lin[2][2][3];
      int yv[2][2];
      for (int r = 0; r < 2; r++)
        for (int c = 0; c < 2; c++) {
          for (int ch = 0; ch < 3; ch++) lin[r][c][ch] = to_linear(t.g2l, iv[r][c][ch]);
          yv[r][c] = from_lin<LUT>(t.l2g, a.lut, a.lut_n, (uint32_t)gray(lin[r][c][0], lin[r][c][1], lin[r][c][2]));
        }
      const int byv[2][2] = {{by00, by01}, {by10, by11}};
      int ny[2][2];
      for (int r = 0; r < 2; r++)
        for (int c = 0; c < 2; c++) {
          const int d = (int)((tycur[k][r] >> (16 * c)) & 0xffff) - yv[r][c];
          ny[r][c] = clip_bd(byv[r][c] + d);
          my_sum += (uint64_t)(d < 0 ? -d : d);
        }
      ynew[k][0] = (uint32_t)ny[0][0] | (uint32_t)ny[0][1] << 16;
      ynew[k][1] = (uint32_t)ny[1][0] | (uint32_t)ny[1][1] << 16;
      // updateChroma -> bestRGBUV, sharpYUVUpdateRGB (:383-388)
      int rgbv[3];
      for (int ch = 0; ch < 3; ch++)
        rgbv[ch] = from_lin<LUT>(t.l2g, a.lut, a.lut_n, (lin[0][0][ch] + lin[0][1][ch] + lin[1][0][ch] + lin[1][1][ch] + 2) >> 2);
      const int gv = gray(rgbv[0], rgbv[1], rgbv[2]);
      for (int ch = 0; ch < 3; ch++) {
        const int16_t src = (int16_t)(rgbv[ch] - gv);
        const int16_t d = (int16_t)(tuvcur[k][ch] - src);
        upd[k][ch] = (int16_t)(C[ch * uvw + i] + d);
      }
    }
    // drain this wave's stores of row pair ju-1 (issued at the end of the
    // last step) and the prefetches (issued before the compute): the wait
    // overlaps the compute
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every read of P/C/N for this step is done
    // row pairs < ju are out: every wave drained its stores of them
    if (tid == 0 && ju > 0) st_sc1(prog_out, (uint32_t)ju);
#pragma unroll
    for (int k = 0; k < MAX_COLS; k++) {
      ycur[k][0] = ynext[k][0];
      ycur[k][1] = ynext[k][1];
      tycur[k][0] = tynext[k][0];
      tycur[k][1] = tynext[k][1];
      for (int ch = 0; ch < 3; ch++) tuvcur[k][ch] = tuvnext[k][ch];
    }
    // rotate: prev <- updated cur (into the old prev slot), cur <- next,
    // next <- prefetched row (or, on the last row pair, a copy of cur)
    const int npi = pi, nci = ni, nni = ci;
#pragma unroll
    for (int k = 0; k < MAX_COLS; k++) {
      const int i = tid + k * ITER_THREADS;
      if (i < uvw)
        for (int ch = 0; ch < 3; ch++) lds_row[npi][ch * uvw + i] = upd[k][ch];
    }
#pragma unroll
    for (int k = 0; k < PFN; k++) {
      const int i = tid + k * ITER_THREADS;
      if (i < words)
        reinterpret_cast<uint32_t*>(lds_row[nni])[i] = have_nn ? pf[k] : reinterpret_cast<const uint32_t*>(lds_row[nci])[i];
    }
    pi = npi;
    ci = nci;
    ni = nni;
    __syncthreads();
    // publish the updated UV row ju (write-through) and drain this wave's stores
    for (int i = tid; i < words; i += ITER_THREADS)
      st_sc1(out_uv + (int64_t)ju * rs + 2 * i, reinterpret_cast<const uint32_t*>(lds_row[pi])[i]);
#pragma unroll
    for (int k = 0; k < MAX_COLS; k++) {
      const int i = tid + k * ITER_THREADS;
      if (i < uvw) {
        st_sc1(out_y + (int64_t)j * w + 2 * i, ynew[k][0]);
        st_sc1(out_y + (int64_t)(j + 1) * w + 2 * i, ynew[k][1]);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) st_sc1(prog_out, (uint32_t)uvh);
  // the iteration's |dY| sum (:254-263); k_sharp_final applies the exit rule
  unsigned long long sm = my_sum;
  for (int off = 32; off > 0; off >>= 1) sm += __shfl_down(sm, off, 64);
  if ((tid & 63) == 0) part[tid >> 6] = sm;
  __syncthreads();
  if (tid == 0) {
    uint64_t sum = 0;
    for (int k = 0; k < ITER_THREADS / 64; k++) sum += part[k];
    a.sums[img * 4 + it] = sum;
    if (timed_out) a.iters[img] = -1;
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
}  // namespace

extern "C" size_t wg_sharpyuv_work_bytes(int32_t width, int32_t height, int32_t n_images) {
  if (width <= 0 || height <= 0 || n_images <= 0) return 0;
  const SharpLayout L = sharp_layout(width, height);
  return n_images * L.bytes_img + (size_t)n_images * (4 * 8 + 4 * 4 + 4) + 16;
}

extern "C" int wg_sharpyuv_convert_ex(const uint8_t* rgb, int32_t width, int32_t height, int32_t rgb_stride,
                                      int64_t rgb_pitch, const int32_t* matrix_host, int32_t transfer,
                                      int32_t sharp_enabled, int32_t n_images, uint8_t* y, int32_t y_stride,
                                      int64_t y_pitch, uint8_t* u, uint8_t* v, int32_t uv_stride, int64_t uv_pitch,
                                      void* work, void* stream) {
  WG_REQUIRE(rgb && matrix_host && y && u && v && width > 0 && height > 0 && n_images > 0);
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
  WG_REQUIRE(uvw <= 8 * ITER_THREADS);
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
  uint8_t* tail = base + n_images * L.bytes_img;
  a.sums = reinterpret_cast<uint64_t*>(tail);
  a.prog = reinterpret_cast<int*>(tail + (size_t)n_images * 32);
  a.iters = a.prog + 4 * n_images;
  a.n_img = n_images;
  if (hipMemsetAsync(tail, 0, (size_t)n_images * (32 + 16 + 4), s) != hipSuccess)
    return wg::check_launch("hipMemsetAsync(sharpyuv)");
  const int64_t cells = (int64_t)uvw * uvh * n_images;
  if (lut)
    hipLaunchKernelGGL(k_sharp_init<true>, dim3(wg::blocks_for(cells, 256)), dim3(256), 0, s, a, n_images);
  else
    hipLaunchKernelGGL(k_sharp_init<false>, dim3(wg::blocks_for(cells, 256)), dim3(256), 0, s, a, n_images);
  int rc = wg::check_launch("k_sharp_init");
  if (rc != WG_OK) return rc;
  // the pipeline's waits need every image's four workgroups resident at
  // once: launch at most as many images as the device holds
  const size_t lds_rows = sizeof(int16_t) * 3 * (size_t)L.uv_rs;
  const bool wide = uvw > 2 * ITER_THREADS;
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, wide ? k_sharp_pipe<8, false> : k_sharp_pipe<2, false>,
                                                   ITER_THREADS, lds_rows) != hipSuccess || per_cu <= 0)
    return wg::check_launch("sharpyuv occupancy");
  const int chunk = std::max(8, (per_cu * cus / 32) * 8);  // images per launch (groups of eight = 32 blocks)
  for (int i0 = 0; i0 < n_images; i0 += chunk) {
    SharpArgs c = a;
    c.n_img = std::min(chunk, n_images - i0);
    c.best_y += i0 * a.img_y;
    c.target_y += i0 * a.img_y;
    c.best_uv += i0 * a.img_uv;
    c.target_uv += i0 * a.img_uv;
    c.sums += 4 * i0;
    c.prog += 4 * i0;
    c.iters += i0;
    const unsigned grid = (unsigned)((c.n_img + 7) / 8 * 32);
    if (wide && lut)
      hipLaunchKernelGGL((k_sharp_pipe<8, true>), dim3(grid), dim3(ITER_THREADS), lds_rows, s, c);
    else if (wide)
      hipLaunchKernelGGL((k_sharp_pipe<8, false>), dim3(grid), dim3(ITER_THREADS), lds_rows, s, c);
    else if (lut)
      hipLaunchKernelGGL((k_sharp_pipe<2, true>), dim3(grid), dim3(ITER_THREADS), lds_rows, s, c);
    else
      hipLaunchKernelGGL((k_sharp_pipe<2, false>), dim3(grid), dim3(ITER_THREADS), lds_rows, s, c);
    rc = wg::check_launch("k_sharp_pipe");
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
  if (hipMemcpyAsync(out, tail + (size_t)n_images * 48, sizeof(int32_t) * n_images, hipMemcpyDeviceToHost, s) !=
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
