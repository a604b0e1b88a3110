// ssim.hip -- whole-plane SSIM on gfx950.  The reference's SSIM primitives
// are SSIMGet / SSIMGetClipped (internal/dsp/ssim.go:116-160); the plane sum
// is libwebp's AccumulateSSIM as fixed in SURVEY.md 8(a) A22: a 7x7 hat
// window per pixel, clipped at the borders (an interior window equals
// SSIMGet since N = 256 there).
//
// A 16x16 tile of pixels per 256-thread workgroup; the 22x22 source tiles
// (3-pixel halo) of both planes are staged in LDS, and the window sums are
// separable (a horizontal, then a vertical 7-tap hat pass).  Window
// statistics are exact integers (any summation order), the per-pixel SSIM is
// the same float64 expression as the reference; the plane sum is a per-tile
// partial plus a second deterministic pass.
#include "wg_common.h"
#include "wg_dsp.h"

namespace {
using namespace wg;

constexpr int TILE = 16, HALO = 3, TS = TILE + 2 * HALO;  // 22

struct SsimArgs {
  const uint8_t *a, *b;
  int64_t a_pitch, b_pitch;
  int a_stride, b_stride, w, h, tiles_x, tiles_y;
  int ty0;  // first tile row; tiles_y tile rows from there
  double* partial;
};

__global__ __launch_bounds__(256) void k_plane_ssim(const SsimArgs p) {
  __shared__ uint8_t ta[TS * TS], tb[TS * TS];
  __shared__ uint32_t hs[5][TS][TILE];  // horizontal 7-tap hat sums of x, y, xx, xy, yy per (row, output column)
  __shared__ double red[4];
  const int tiles = p.tiles_x * p.tiles_y;
  const int img = blockIdx.x / tiles;
  const int tile = blockIdx.x % tiles;
  const int tx0 = (tile % p.tiles_x) * TILE, ty0 = (tile / p.tiles_x + p.ty0) * TILE;
  const uint8_t* A = p.a + img * p.a_pitch;
  const uint8_t* B = p.b + img * p.b_pitch;
  for (int i = threadIdx.x; i < TS * TS; i += blockDim.x) {
    const int yy = ty0 - HALO + i / TS, xx = tx0 - HALO + i % TS;
    const bool in = xx >= 0 && xx < p.w && yy >= 0 && yy < p.h;
    ta[i] = in ? A[(int64_t)yy * p.a_stride + xx] : 0;
    tb[i] = in ? B[(int64_t)yy * p.b_stride + xx] : 0;
  }
  __syncthreads();
  // The hat weights are separable (kw[dx] * kw[dy]) and pixels outside the
  // image are staged as 0, so a clipped window's sums are a 7-tap horizontal
  // pass followed by a 7-tap vertical one, and its weight is the product of
  // the in-image tap sums: the same integers as the 49-term window of
  // SSIMGetClipped (ssim.go:132-160), at 5 x (7 + 7 x 22/16) MACs per pixel
  // instead of 6 x 49.
  constexpr uint32_t kw[7] = {1, 2, 3, 4, 3, 2, 1};
  for (int i = threadIdx.x; i < TS * TILE; i += blockDim.x) {
    const int r = i / TILE, cx = i % TILE;
    const uint8_t* pa = ta + r * TS + cx;
    const uint8_t* pb = tb + r * TS + cx;
    uint32_t sx = 0, sy = 0, sxx = 0, sxy = 0, syy = 0;
#pragma unroll
    for (int dx = 0; dx < 7; dx++) {
      const uint32_t x = pa[dx], y = pb[dx], wx = kw[dx] * x, wy = kw[dx] * y;
      sx += wx;
      sy += wy;
      sxx += wx * x;
      sxy += wx * y;
      syy += wy * y;
    }
    hs[0][r][cx] = sx;
    hs[1][r][cx] = sy;
    hs[2][r][cx] = sxx;
    hs[3][r][cx] = sxy;
    hs[4][r][cx] = syy;
  }
  __syncthreads();
  const int lx = threadIdx.x % TILE, ly = threadIdx.x / TILE;
  const int xo = tx0 + lx, yo = ty0 + ly;
  double v = 0.0;
  if (xo < p.w && yo < p.h) {
    SsimStats s = {0, 0, 0, 0, 0, 0};
    uint32_t wxs = 0, wys = 0;
#pragma unroll
    for (int d = 0; d < 7; d++) {
      const uint32_t k = kw[d];
      s.xm += k * hs[0][ly + d][lx];
      s.ym += k * hs[1][ly + d][lx];
      s.xxm += k * hs[2][ly + d][lx];
      s.xym += k * hs[3][ly + d][lx];
      s.yym += k * hs[4][ly + d][lx];
      const int xx = xo - 3 + d, yy = yo - 3 + d;
      wxs += (xx >= 0 && xx < p.w) ? k : 0u;
      wys += (yy >= 0 && yy < p.h) ? k : 0u;
    }
    s.w = wxs * wys;
    v = ssim_calc(s, s.w);  // SSIMFromStatsClipped; s.w == 256 for interior windows
  }
  // block reduction (fixed order -> deterministic)
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) p.partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void k_sum_partials(const double* partial, int per_img, double* out) {
  __shared__ double red[4];
  const int img = blockIdx.x;
  double v = 0.0;
  for (int i = threadIdx.x; i < per_img; i += blockDim.x) v += partial[(int64_t)img * per_img + i];
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) out[img] = (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace

extern "C" size_t wg_plane_ssim_work_bytes(int32_t w, int32_t h, int32_t n_images) {
  if (w <= 0 || h <= 0 || n_images <= 0) return 0;
  return sizeof(double) * (size_t)n_images * ((w + TILE - 1) / TILE) * ((h + TILE - 1) / TILE);
}

extern "C" int wg_plane_ssim_rows(const uint8_t* a, int32_t a_stride, int64_t a_pitch, const uint8_t* b,
                                  int32_t b_stride, int64_t b_pitch, int32_t w, int32_t h, int32_t ty_begin,
                                  int32_t ty_end, int32_t n_images, double* partial, void* stream) {
  WG_REQUIRE(a && b && partial && w > 0 && h > 0 && n_images > 0 && a_stride >= w && b_stride >= w);
  WG_REQUIRE(ty_begin >= 0 && ty_begin < ty_end && ty_end <= (h + TILE - 1) / TILE);
  SsimArgs p;
  p.a = a;
  p.b = b;
  p.a_pitch = a_pitch;
  p.b_pitch = b_pitch;
  p.a_stride = a_stride;
  p.b_stride = b_stride;
  p.w = w;
  p.h = h;
  p.tiles_x = (w + TILE - 1) / TILE;
  p.tiles_y = ty_end - ty_begin;
  p.ty0 = ty_begin;
  p.partial = partial;
  const int per = p.tiles_x * p.tiles_y;
  hipLaunchKernelGGL(k_plane_ssim, dim3((unsigned)(per * n_images)), dim3(256), 0, wg::as_stream(stream), p);
  return wg::check_launch("k_plane_ssim");
}

extern "C" int wg_plane_ssim_reduce(const double* partial, int64_t per_image, int32_t n_images, double* out,
                                    void* stream) {
  WG_REQUIRE(partial && out && per_image > 0 && per_image < (1ll << 31) && n_images > 0);
  hipLaunchKernelGGL(k_sum_partials, dim3((unsigned)n_images), dim3(256), 0, wg::as_stream(stream), partial,
                     (int)per_image, out);
  return wg::check_launch("k_sum_partials");
}

extern "C" int wg_plane_ssim(const uint8_t* a, int32_t a_stride, int64_t a_pitch, const uint8_t* b, int32_t b_stride,
                             int64_t b_pitch, int32_t w, int32_t h, int32_t n_images, double* out, void* work,
                             void* stream) {
  WG_REQUIRE(a && b && out && work && w > 0 && h > 0 && n_images > 0 && a_stride >= w && b_stride >= w);
  const int tiles_y = (h + TILE - 1) / TILE;
  double* partial = static_cast<double*>(work);
  int rc = wg_plane_ssim_rows(a, a_stride, a_pitch, b, b_stride, b_pitch, w, h, 0, tiles_y, n_images, partial, stream);
  if (rc) return rc;
  return wg_plane_ssim_reduce(partial, (int64_t)((w + TILE - 1) / TILE) * tiles_y, n_images, out, stream);
}
