// ssim.hip -- whole-plane SSIM on gfx950.  The reference's SSIM primitives
// are SSIMGet / SSIMGetClipped (internal/dsp/ssim.go:116-160); the plane sum
// is libwebp's AccumulateSSIM as fixed in SURVEY.md 8(a) A22: a 7x7 hat
// window per pixel, clipped at the borders (an interior window equals
// SSIMGet since N = 256 there).
//
// One wave per (58-column strip, 32-row band): lane L owns column
// 58 s - 3 + L and walks down the band's rows plus the 3-row halo.  The hat
// weights are separable (kw[dx] * kw[dy]) and the 7-tap hat (1 2 3 4 3 2 1)
// is a 4-tap box applied twice, so per row a lane
//   - loads its two bytes (pixels outside the image are 0) and forms
//     x, y, xx, xy, yy;
//   - runs the vertical hat as two running 4-row box sums (register rings of
//     four rows; exact integers, so the order does not matter);
//   - takes the horizontal hat of the five vertical sums across lanes with
//     wave-wide DPP shifts (lanes 3..60 hold complete windows: the strip's
//     58 outputs).
// The clipped window's weight is the product of the in-image tap sums, so
// the statistics equal the 49-term sums of SSIMGetClipped (ssim.go:132-160).
// The per-pixel SSIM is the reference's float64 expression; interior windows
// (N = 256) use 32-bit products where they fit.  Partial sums per (16-row
// tile row, strip) are reduced by a second, fixed-order pass.
#include "wg_common.h"
#include "wg_instr.h"
#include "wg_dsp.h"

#include <cstdlib>

namespace {
using namespace wg;

constexpr int TILE = 16;   // rows per partial sum: the _rows entry point's tile row
constexpr int STRIP = 58;  // output columns per wave: 64 lanes less a 3-column halo each side

struct SsimArgs {
  const uint8_t *a, *b;
  int64_t a_pitch, b_pitch;
  int a_stride, b_stride, w, h, strips, groups, group;  // group: tile rows per wave
  int ty0, tiles_y;  // tiles_y tile rows from ty0
  double* partial;
};

// (bound_ctrl: the lane with no source reads 0; only lanes 3..60 are used)
__device__ __forceinline__ uint32_t from_left(uint32_t v) {  // lane L - 1 (wave_shr:1)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t from_right(uint32_t v) {  // lane L + 1 (wave_shl:1)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, true);
}

// ssim_calc (wg_dsp.h; ssim.go:48-83) with N = 256: x_m^2, y_m^2, x_m y_m and
// the N-scaled moments fit 32 bits (x_m <= 256 * 255 < 2^24, so 24-bit
// multiplies), and by Cauchy-Schwarz N xx_m >= x_m^2 exactly (the weights sum
// to N).  The reference converts the uint64 products fnum, fden to float64;
// their factors are exact in float64, so one correctly rounded multiply
// gives the same double.
__device__ __forceinline__ double ssim_interior(uint32_t xm, uint32_t ym, uint32_t xxm, uint32_t xym, uint32_t yym) {
  constexpr uint32_t c3 = 64 * 65536, c2_256 = 60 * 65536 / 256;  // c2 = 60 N^2 is a multiple of 256
  constexpr double c1 = 20.0 * 65536;
  const uint32_t xmxm = (uint32_t)__umul24(xm, xm), ymym = (uint32_t)__umul24(ym, ym), xmym = (uint32_t)__umul24(xm, ym);
  const uint64_t sq = (uint64_t)xmxm + ymym;
  const uint32_t sxx = (xxm << 8) - xmxm, syy = (yym << 8) - ymym, xy8 = xym << 8;
  const uint32_t sxy_pos = xy8 > xmym ? xy8 - xmym : 0u;  // max(N xy_m - x_m y_m, 0) < 2^32
  // (2 sxy + c2) >> 8 and (sxx + syy + c2) >> 8 with c2 / 256 added after the shift
  const uint32_t num_s = (sxy_pos >> 7) + c2_256;
  const uint32_t den_s = (uint32_t)(((uint64_t)sxx + syy) >> 8) + c2_256;
  const double fnum = (2.0 * (double)xmym + c1) * (double)num_s;
  const double fden = ((double)xmxm + (double)ymym + c1) * (double)den_s;  // > 0
  return sq < c3 ? 1.0 : fnum / fden;
}

__device__ __forceinline__ uint32_t hat_weight(int v, int n) {  // in-image taps of the hat at v - 3 .. v + 3
  constexpr uint32_t kw[7] = {1, 2, 3, 4, 3, 2, 1};
  uint32_t s = 0;
#pragma unroll
  for (int d = 0; d < 7; d++) s += (v - 3 + d >= 0 && v - 3 + d < n) ? kw[d] : 0u;
  return s;
}

__device__ __forceinline__ double wave_sum(double v) {  // fixed order: the same bits for the same inputs
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

__global__ __launch_bounds__(64) void k_plane_ssim(const SsimArgs p) {
  const int per = p.strips * p.groups;
  const int img = blockIdx.x / per, rem = blockIdx.x % per;
  const int g = rem / p.strips, s = rem % p.strips;  // strips fastest: neighbouring waves share rows in L2
  const int lane = threadIdx.x;
  const int x = s * STRIP - 3 + lane;
  const bool col_in = x >= 0 && x < p.w;
  const bool out_lane = lane >= 3 && lane < 3 + STRIP && x < p.w;
  const int t0 = p.ty0 + g * p.group, t1 = min(t0 + p.group, p.ty0 + p.tiles_y);
  const int y0 = t0 * TILE, y1 = min(t1 * TILE, p.h);
  const int n_in = y1 - y0 + 6;  // rows y0 - 3 .. y1 + 2
  const uint8_t* A = p.a + img * p.a_pitch;
  const uint8_t* B = p.b + img * p.b_pitch;
  const uint32_t xo = col_in ? (uint32_t)x : 0u;
  const uint32_t wx = hat_weight(x, p.w);
  const bool fast_x = s * STRIP - 3 >= 3 && s * STRIP + STRIP + 2 < p.w;  // every output lane's taps inside
  // row r of both planes: a wave-uniform row address plus the lane's column
  // (rows and columns outside the image read as 0, from a clamped address)
  // row r of both planes, raw: a wave-uniform row address plus the lane's
  // column (a plane's offsets fit 31 bits, wg_plane_ssim_rows checks); the
  // mask for rows / columns outside the image is applied at use, so the
  // loads of a block stay in flight while the block before it is processed
  // (the row loop runs in blocks of 8, so it may ask for up to 7 rows past
  // y1 + 2: clamped to the rows the band owns with its halo, which a band
  // buffer of wg_plane_ssim_devices holds; their outputs are not kept)
  const int r_lo = max(y0 - 3, 0), r_hi = min(y1 + 2, p.h - 1);
  // (WG_BOUNDS) the rows the launch's band owns with its halo
  [[maybe_unused]] const int band_lo = max(p.ty0 * TILE - 3, 0), band_hi = min((p.ty0 + p.tiles_y) * TILE + 3, p.h);
  auto load = [&](int r, uint32_t& va, uint32_t& vb) {
    const int rc = min(max(r, r_lo), r_hi);
    const uint8_t *qa = A + (uint32_t)(rc * p.a_stride) + xo, *qb = B + (uint32_t)(rc * p.b_stride) + xo;
    va = WG_CHK(qa, 1, A + (int64_t)band_lo * p.a_stride, (int64_t)(band_hi - band_lo) * p.a_stride, "k_plane_ssim a")
             ? *qa : 0u;
    vb = WG_CHK(qb, 1, B + (int64_t)band_lo * p.b_stride, (int64_t)(band_hi - band_lo) * p.b_stride, "k_plane_ssim b")
             ? *qb : 0u;
  };
  // running sums: Bv = box4 of the rows' stats, Tv = box4 of Bv = the vertical
  // hat.  Stat 0 packs x | y << 16: every partial sum of x or y stays below
  // 2^16 (the full hat: 256 * 255) and never goes negative, so 32-bit adds
  // and subtractions of packed words are exact per half (add first, then
  // subtract what leaves the window).
  uint32_t hq[4][4], hb[4][4], Bv[4] = {0, 0, 0, 0}, Tv[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int i = 0; i < 4; i++) hq[k][i] = hb[k][i] = 0;
  double acc = 0.0;
  // four input rows j0 .. j0 + 3 (rows past n_in only feed outputs beyond y1, which are skipped)
  auto block = [&](int j0, const uint32_t (&ra)[4], const uint32_t (&rb)[4]) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int j = j0 + k, r = y0 - 3 + j;
      const uint32_t m = (col_in && r >= 0 && r < p.h) ? 0xffu : 0u;
      const uint32_t xv = ra[k] & m, yv = rb[k] & m;
      const uint32_t q[4] = {xv | yv << 16, (uint32_t)__umul24(xv, xv), (uint32_t)__umul24(xv, yv),
                             (uint32_t)__umul24(yv, yv)};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        Bv[i] = (Bv[i] + q[i]) - hq[k][i];
        hq[k][i] = q[i];
        Tv[i] = (Tv[i] + Bv[i]) - hb[k][i];
        hb[k][i] = Bv[i];
      }
      const int y = y0 + j - 6;  // the output row whose window ends at this input row
      if (j < 6 || y >= y1) continue;
      // horizontal hat of the vertical sums, stage by stage over the four
      // (independent DPP chains interleave, no hazard stalls)
      uint32_t st[4], t[4], u[4];
#pragma unroll
      for (int i = 0; i < 4; i++) t[i] = Tv[i] + from_left(Tv[i]);  // L-1, L
#pragma unroll
      for (int i = 0; i < 4; i++) u[i] = from_left(t[i]);
#pragma unroll
      for (int i = 0; i < 4; i++) u[i] = t[i] + from_left(u[i]);  // L-3 .. L
#pragma unroll
      for (int i = 0; i < 4; i++) t[i] = u[i] + from_right(u[i]);  // box(L), box(L+1)
#pragma unroll
      for (int i = 0; i < 4; i++) u[i] = from_right(t[i]);
#pragma unroll
      for (int i = 0; i < 4; i++) st[i] = t[i] + from_right(u[i]);  // box(L) .. box(L+3)
      const uint32_t sx = st[0] & 0xffff, sy = st[0] >> 16;
      double v;
      if (fast_x && y >= 3 && y + 3 < p.h) {
        v = ssim_interior(sx, sy, st[1], st[2], st[3]);
      } else {
        const uint32_t n = wx * hat_weight(y, p.h);
        const SsimStats ss = {n, sx, sy, st[1], st[2], st[3]};
        v = ssim_calc(ss, n);  // SSIMFromStatsClipped
      }
      acc += v;  // (finite in every lane: fden > 0; lanes without an output are dropped below)
      if (((y + 1) % TILE) == 0 || y + 1 == y1) {  // the tile row is complete
        const double tot = wave_sum(out_lane ? acc : 0.0);
        acc = 0.0;
        double* const q = p.partial + ((int64_t)img * p.tiles_y + (y / TILE - p.ty0)) * p.strips + s;
        if (lane == 0 && WG_CHK(q, 8, p.partial, 8ll * (blockIdx.x / per + 1) * p.tiles_y * p.strips, "k_plane_ssim partial"))
          *q = tot;
      }
    }
  };
  // two register sets, each block's loads issued one block ahead: no
  // register copies, so no wait on loads still in flight
  uint32_t pa[4], pb[4], qa[4], qb[4];
#pragma unroll
  for (int k = 0; k < 4; k++) load(y0 - 3 + k, pa[k], pb[k]);
  for (int j0 = 0; j0 < n_in; j0 += 8) {
#pragma unroll
    for (int k = 0; k < 4; k++) load(y0 + 1 + j0 + k, qa[k], qb[k]);
    block(j0, pa, pb);
#pragma unroll
    for (int k = 0; k < 4; k++) load(y0 + 5 + j0 + k, pa[k], pb[k]);
    block(j0 + 4, qa, qb);
  }
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

extern "C" int32_t wg_plane_ssim_row_partials(int32_t w) { return w > 0 ? (w + STRIP - 1) / STRIP : 0; }

extern "C" size_t wg_plane_ssim_work_bytes(int32_t w, int32_t h, int32_t n_images) {
  if (w <= 0 || h <= 0 || n_images <= 0) return 0;
  return sizeof(double) * (size_t)n_images * wg_plane_ssim_row_partials(w) * ((h + TILE - 1) / TILE);
}

extern "C" int wg_plane_ssim_rows(const uint8_t* a, int32_t a_stride, int64_t a_pitch, const uint8_t* b,
                                  int32_t b_stride, int64_t b_pitch, int32_t w, int32_t h, int32_t ty_begin,
                                  int32_t ty_end, int32_t n_images, double* partial, void* stream) {
  WG_REQUIRE(a && b && partial && w > 0 && h > 0 && n_images > 0 && a_stride >= w && b_stride >= w);
  WG_REQUIRE(ty_begin >= 0 && ty_begin < ty_end && ty_end <= (h + TILE - 1) / TILE);
  WG_REQUIRE((int64_t)a_stride * h < (1ll << 31) && (int64_t)b_stride * h < (1ll << 31));
  SsimArgs p;
  p.a = a;
  p.b = b;
  p.a_pitch = a_pitch;
  p.b_pitch = b_pitch;
  p.a_stride = a_stride;
  p.b_stride = b_stride;
  p.w = w;
  p.h = h;
  p.strips = wg_plane_ssim_row_partials(w);
  p.ty0 = ty_begin;
  p.tiles_y = ty_end - ty_begin;
  static const int group = [] {  // tile rows per wave (A/B knob WG_SSIM_GROUP, default 2)
    const char* e = getenv("WG_SSIM_GROUP");
    const int g = e ? atoi(e) : 2;
    return g >= 1 && g <= 16 ? g : 2;
  }();
  p.group = group;
  p.groups = (p.tiles_y + group - 1) / group;
  p.partial = partial;
  const int64_t waves = (int64_t)p.strips * p.groups * n_images;
  WG_REQUIRE(waves < (1ll << 31));
  hipLaunchKernelGGL(k_plane_ssim, dim3((unsigned)waves), dim3(64), 0, wg::as_stream(stream), p);
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
  return wg_plane_ssim_reduce(partial, (int64_t)wg_plane_ssim_row_partials(w) * tiles_y, n_images, out, stream);
}
