// sharpyuv.hip -- SharpYUV RGB -> YUV420 on gfx950,
// sRGB transfer, any conversion matrix (sharpyuv/sharpyuv.go:170-432).
//
//   k_sharp_init   import + gray Y, target W, target / initial chroma
//                  residuals (convertSharp phase 1, :196-222): one thread per
//                  2x2 block, fully parallel
//   k_sharp_iter   the iterative refinement (:224-264).  Each iteration sweeps
//                  the row pairs in order and updates the chroma residuals in
//                  place, so row pair j reads row pair j-1's values from the
//                  SAME iteration (Gauss-Seidel); the sweep is sequential by
//                  construction.  One workgroup per image walks it, the whole
//                  width in parallel, the updated row kept in LDS as the next
//                  row's "prev", the next row's inputs prefetched into
//                  registers while the current one computes.  The early exit
//                  needs the iteration's global |dY| sum, reduced in-workgroup.
//   k_sharp_final  W/RGB -> YUV with the matrix (:390-432), per pixel
//
// All arithmetic is integer (the reference's int / int64 / int16 with wrap);
// the gamma tables are built on the host (sharpyuv_host.cpp) like
// initGammaTables (gamma.go:48-88) and staged in LDS.
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
__device__ __forceinline__ int gray(int64_t r, int64_t g, int64_t b) {
  return (int)((13933 * r + 46871 * g + 4732 * b + 32768) >> 16);
}
__device__ __forceinline__ int clip_bd(int v) { return min(max(v, 0), MAXY); }

// Per image working set, in the reference's layout (sharpyuv.go:186-193):
// best_y / target_y: w*h uint16; best_uv / target_uv: per UV row, 3 planes of
// uvw int16 (R-W, G-W, B-W).
struct SharpArgs {
  const uint8_t* rgb;
  int64_t rgb_pitch;
  int rgb_stride, width, height, w, h, uvw, uvh;
  uint16_t* best_y;
  uint16_t* target_y;
  int16_t* best_uv;
  int16_t* target_uv;
  int64_t y_pitch, uv_pitch;  // elements per image of the working buffers
  const SharpTabs* tabs;
  int* iters;  // per image: iterations run (diagnostic)
};

__device__ __forceinline__ void load_tabs(SharpTabs& dst, const SharpTabs* src) {
  for (int i = threadIdx.x; i < G2L_N; i += blockDim.x) dst.g2l[i] = src->g2l[i];
  for (int i = threadIdx.x; i < L2G_N; i += blockDim.x) dst.l2g[i] = src->l2g[i];
  __syncthreads();
}

// phase 1: thread = one UV position (i, jUV) of one image
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
  uint16_t* by = a.best_y + img * a.y_pitch;
  uint16_t* ty = a.target_y + img * a.y_pitch;
  uint32_t lin[2][2][3];
  for (int r = 0; r < 2; r++)
    for (int k = 0; k < 2; k++) {
      const int64_t o = (int64_t)(j + r) * a.w + 2 * i + k;
      by[o] = (uint16_t)gray(c[r][k][0], c[r][k][1], c[r][k][2]);  // storeGray
      for (int ch = 0; ch < 3; ch++) lin[r][k][ch] = to_linear(t.g2l, c[r][k][ch]);
      ty[o] = (uint16_t)from_linear(t.l2g, (uint32_t)gray(lin[r][k][0], lin[r][k][1], lin[r][k][2]));  // updateW
    }
  int rgbv[3];  // updateChroma (:303-315): scaleDown in linear light
  for (int ch = 0; ch < 3; ch++)
    rgbv[ch] = from_linear(t.l2g, (lin[0][0][ch] + lin[0][1][ch] + lin[1][0][ch] + lin[1][1][ch] + 2) >> 2);
  const int gv = gray(rgbv[0], rgbv[1], rgbv[2]);
  int16_t* tuv = a.target_uv + img * a.uv_pitch + (int64_t)ju * 3 * a.uvw;
  int16_t* buv = a.best_uv + img * a.uv_pitch + (int64_t)ju * 3 * a.uvw;
  for (int ch = 0; ch < 3; ch++) {
    const int16_t d = (int16_t)(rgbv[ch] - gv);
    tuv[ch * a.uvw + i] = d;
    buv[ch * a.uvw + i] = d;
  }
}

constexpr int ITER_THREADS = 1024;

// phase 2: one workgroup per image.  Thread t owns UV columns t + k*1024,
// k < MAX_COLS: MAX_COLS = 2 covers widths up to 4096 without spilling; 8
// covers up to 16384.
template <int MAX_COLS>
__global__ __launch_bounds__(ITER_THREADS) void k_sharp_iter(SharpArgs a) {
  __shared__ SharpTabs t;
  extern __shared__ int16_t rows[];  // prev / cur / next UV rows: 3 rows x 3 planes x uvw
  __shared__ unsigned long long part[ITER_THREADS / 64];
  __shared__ int stop;
  load_tabs(t, a.tabs);
  const int img = blockIdx.x, tid = threadIdx.x;
  const int uvw = a.uvw, uvh = a.uvh, w = a.w;
  uint16_t* by = a.best_y + img * a.y_pitch;
  const uint16_t* ty = a.target_y + img * a.y_pitch;
  int16_t* buv = a.best_uv + img * a.uv_pitch;
  const int16_t* tuv = a.target_uv + img * a.uv_pitch;
  int16_t* lds_row[3] = {rows, rows + 3 * uvw, rows + 6 * uvw};  // rotating prev / cur / next
  const uint64_t threshold = (uint64_t)3 * w * a.h;
  uint64_t prev_sum = ~0ull;
  int iters = 0;

  for (int it = 0; it < 4; it++) {
    uint64_t my_sum = 0;
    int pi = 0, ci = 1, ni = 2;
    // rows 0 and 1 of this iteration's state: prev(row 0) = cur(row 0) = row 0
    for (int i = tid; i < 3 * uvw; i += ITER_THREADS) {
      const int16_t v0 = buv[i];
      lds_row[ci][i] = v0;
      lds_row[pi][i] = v0;
      lds_row[ni][i] = uvh > 1 ? buv[3 * uvw + i] : v0;
    }
    __syncthreads();
    for (int ju = 0; ju < uvh; ju++) {
      const int16_t* P = lds_row[pi];
      const int16_t* C = lds_row[ci];
      const int16_t* N = lds_row[ni];
      const int j = 2 * ju;
      // prefetch the row after next (the next step's "next") into registers
      int16_t pf[MAX_COLS][3];
      int16_t upd[MAX_COLS][3];  // the updated row: written to LDS only after every thread read P/C/N
      const bool have_nn = ju + 2 < uvh;
#pragma unroll
      for (int k = 0; k < MAX_COLS; k++) {
        const int i = tid + k * ITER_THREADS;
        if (have_nn && i < uvw)
          for (int ch = 0; ch < 3; ch++) pf[k][ch] = buv[(int64_t)(ju + 2) * 3 * uvw + ch * uvw + i];
      }
#pragma unroll
      for (int k = 0; k < MAX_COLS; k++) {
        const int i = tid + k * ITER_THREADS;
        if (i >= uvw) continue;
        // interpolateTwoRows (:322-359) for pixels x = 2i, 2i+1 of rows j, j+1
        int iv[2][2][3];
        const int64_t y0 = (int64_t)j * w + 2 * i, y1 = y0 + w;
        const int by00 = by[y0], by01 = by[y0 + 1], by10 = by[y1], by11 = by[y1 + 1];
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
            yv[r][c] = from_linear(t.l2g, (uint32_t)gray(lin[r][c][0], lin[r][c][1], lin[r][c][2]));
          }
        const int64_t ys[2][2] = {{y0, y0 + 1}, {y1, y1 + 1}};
        const int byv[2][2] = {{by00, by01}, {by10, by11}};
        for (int r = 0; r < 2; r++)
          for (int c = 0; c < 2; c++) {
            const int d = (int)ty[ys[r][c]] - yv[r][c];
            by[ys[r][c]] = (uint16_t)clip_bd(byv[r][c] + d);
            my_sum += (uint64_t)(d < 0 ? -d : d);
          }
        // updateChroma -> bestRGBUV, sharpYUVUpdateRGB (:383-388), in place
        int rgbv[3];
        for (int ch = 0; ch < 3; ch++)
          rgbv[ch] = from_linear(t.l2g, (lin[0][0][ch] + lin[0][1][ch] + lin[1][0][ch] + lin[1][1][ch] + 2) >> 2);
        const int gv = gray(rgbv[0], rgbv[1], rgbv[2]);
        for (int ch = 0; ch < 3; ch++) {
          const int64_t o = (int64_t)ju * 3 * uvw + ch * uvw + i;
          const int16_t src = (int16_t)(rgbv[ch] - gv);
          const int16_t d = (int16_t)(tuv[o] - src);
          const int16_t nv = (int16_t)(C[ch * uvw + i] + d);
          buv[o] = nv;
          upd[k][ch] = nv;
        }
      }
      __syncthreads();  // every read of P/C/N for this step is done
      // rotate: prev <- updated cur (into the old prev slot), cur <- next,
      // next <- prefetched row (or, on the last row pair, a copy of cur)
      const int npi = pi, nci = ni, nni = ci;
#pragma unroll
      for (int k = 0; k < MAX_COLS; k++) {
        const int i = tid + k * ITER_THREADS;
        if (i < uvw)
          for (int ch = 0; ch < 3; ch++) {
            lds_row[npi][ch * uvw + i] = upd[k][ch];
            lds_row[nni][ch * uvw + i] = have_nn ? pf[k][ch] : lds_row[nci][ch * uvw + i];
          }
      }
      pi = npi;
      ci = nci;
      ni = nni;
      __syncthreads();
    }
    // iteration's |dY| sum and the early exit (:254-263)
    unsigned long long s = my_sum;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if ((tid & 63) == 0) part[tid >> 6] = s;
    __syncthreads();
    if (tid == 0) {
      uint64_t sum = 0;
      for (int k = 0; k < ITER_THREADS / 64; k++) sum += part[k];
      stop = (it > 0 && (sum < threshold || sum > prev_sum)) ? 1 : 0;
      part[0] = sum;
    }
    __syncthreads();
    prev_sum = part[0];
    iters++;
    const int brk = stop;
    __syncthreads();
    if (brk) break;
  }
  if (tid == 0 && a.iters) a.iters[img] = iters;
}

struct FinalArgs {
  const uint16_t* best_y;
  const int16_t* best_uv;
  uint8_t* y;
  uint8_t* u;
  uint8_t* v;
  int64_t y_pitch, uv_pitch, out_y_pitch, out_uv_pitch;
  int y_stride, uv_stride, width, height, w, uvw, uvh;
  int m[12];
};

// convertWRGBToYUV (:390-432): thread per Y pixel; threads of even (x, y)
// also produce the U / V sample.
__global__ __launch_bounds__(256) void k_sharp_final(FinalArgs a, int n_img) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)a.width * a.height;
  if (gid >= per * n_img) return;
  const int img = (int)(gid / per);
  const int64_t p = gid - img * per;
  const int j = (int)(p / a.width), i = (int)(p - (int64_t)j * a.width);
  const uint16_t* by = a.best_y + img * a.y_pitch;
  const int16_t* buv = a.best_uv + img * a.uv_pitch;
  constexpr int SHIFT = 16 + SFIX;
  const int64_t rounder = (int64_t)1 << (SHIFT - 1);
  const int uvi = (j / 2) * 3 * a.uvw + (i >> 1);
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

}  // namespace

namespace wg {
const void* sharpyuv_tables_device();  // sharpyuv_host.cpp: g2l[1026] then l2g[514] (uint32)
}

extern "C" size_t wg_sharpyuv_work_bytes(int32_t width, int32_t height, int32_t n_images) {
  if (width <= 0 || height <= 0 || n_images <= 0) return 0;
  const size_t w = (size_t)((width + 1) & ~1), h = (size_t)((height + 1) & ~1);
  const size_t per = 2 * (w * h * 2) + 2 * (3 * (w / 2) * (h / 2) * 2);
  return n_images * ((per + 255) & ~(size_t)255) + 4 * (size_t)n_images;
}

extern "C" int wg_sharpyuv_convert(const uint8_t* rgb, int32_t width, int32_t height, int32_t rgb_stride,
                                   int64_t rgb_pitch, const int32_t* matrix_host, int32_t n_images, uint8_t* y,
                                   int32_t y_stride, int64_t y_pitch, uint8_t* u, uint8_t* v, int32_t uv_stride,
                                   int64_t uv_pitch, void* work, void* stream) {
  WG_REQUIRE(rgb && matrix_host && y && u && v && work && width > 0 && height > 0 && n_images > 0);
  WG_REQUIRE(rgb_stride >= 3 * width && y_stride >= width && uv_stride >= (width + 1) / 2);
  const int w = (width + 1) & ~1, h = (height + 1) & ~1;
  const int uvw = w / 2, uvh = h / 2;
  WG_REQUIRE(uvw <= 8 * ITER_THREADS);
  const void* tabs = wg::sharpyuv_tables_device();
  if (!tabs) return WG_EHIP;
  hipStream_t s = wg::as_stream(stream);
  const size_t per = ((size_t)2 * (w * (size_t)h * 2) + 2 * (3 * (size_t)uvw * uvh * 2) + 255) & ~(size_t)255;
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
  // per image: best_y | target_y | best_uv | target_uv  (pitches in elements)
  a.best_y = reinterpret_cast<uint16_t*>(base);
  a.target_y = a.best_y + (size_t)w * h;
  a.best_uv = reinterpret_cast<int16_t*>(a.target_y + (size_t)w * h);
  a.target_uv = a.best_uv + (size_t)3 * uvw * uvh;
  a.y_pitch = (int64_t)(per / 2);
  a.uv_pitch = (int64_t)(per / 2);
  a.tabs = static_cast<const SharpTabs*>(tabs);
  a.iters = reinterpret_cast<int*>(base + per * n_images);
  const int64_t cells = (int64_t)uvw * uvh * n_images;
  hipLaunchKernelGGL(k_sharp_init, dim3(wg::blocks_for(cells, 256)), dim3(256), 0, s, a, n_images);
  int rc = wg::check_launch("k_sharp_init");
  if (rc != WG_OK) return rc;
  const size_t lds_rows = sizeof(int16_t) * 9 * (size_t)uvw;
  if (uvw <= 2 * ITER_THREADS)
    hipLaunchKernelGGL(k_sharp_iter<2>, dim3((unsigned)n_images), dim3(ITER_THREADS), lds_rows, s, a);
  else
    hipLaunchKernelGGL(k_sharp_iter<8>, dim3((unsigned)n_images), dim3(ITER_THREADS), lds_rows, s, a);
  rc = wg::check_launch("k_sharp_iter");
  if (rc != WG_OK) return rc;
  FinalArgs f;
  f.best_y = a.best_y;
  f.best_uv = a.best_uv;
  f.y = y;
  f.u = u;
  f.v = v;
  f.y_pitch = a.y_pitch;
  f.uv_pitch = a.uv_pitch;
  f.out_y_pitch = y_pitch;
  f.out_uv_pitch = uv_pitch;
  f.y_stride = y_stride;
  f.uv_stride = uv_stride;
  f.width = width;
  f.height = height;
  f.w = w;
  f.uvw = uvw;
  f.uvh = uvh;
  for (int k = 0; k < 12; k++) f.m[k] = matrix_host[k];
  const int64_t px = (int64_t)width * height * n_images;
  hipLaunchKernelGGL(k_sharp_final, dim3(wg::blocks_for(px, 256)), dim3(256), 0, s, f, n_images);
  return wg::check_launch("k_sharp_final");
}
