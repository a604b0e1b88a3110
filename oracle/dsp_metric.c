/*
 * dsp_metric.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates internal/dsp/ssim.go (SSE, TDisto, SSIM).
 */
#include "oracle.h"

#define BPS OR_BPS

static int sse_block(const uint8_t* a, const uint8_t* b, int n) {
  int s = 0;
  for (int y = 0; y < n; y++)
    for (int x = 0; x < n; x++) {
      int d = a[x + y * BPS] - b[x + y * BPS];
      s += d * d;
    }
  return s;
}
int or_sse4x4(const uint8_t* a, const uint8_t* b) { return sse_block(a, b, 4); }     /* :188 */
int or_sse16x16(const uint8_t* a, const uint8_t* b) { return sse_block(a, b, 16); }  /* :220 */

static const int k_weight_y[16] = {38, 32, 20, 9, 32, 28, 17, 7, 20, 17, 10, 4, 9, 7, 4, 2}; /* :257 */

static int ttransform(const uint8_t* in) { /* tTransform :266-304 */
  int tmp[16];
  for (int i = 0; i < 4; i++) {
    const uint8_t* r = in + i * BPS;
    int a0 = r[0] + r[2], a1 = r[1] + r[3], a2 = r[1] - r[3], a3 = r[0] - r[2];
    tmp[4 * i + 0] = a0 + a1;
    tmp[4 * i + 1] = a3 + a2;
    tmp[4 * i + 2] = a3 - a2;
    tmp[4 * i + 3] = a0 - a1;
  }
  int sum = 0;
  for (int i = 0; i < 4; i++) {
    int a0 = tmp[i] + tmp[8 + i], a1 = tmp[4 + i] + tmp[12 + i];
    int a2 = tmp[4 + i] - tmp[12 + i], a3 = tmp[i] - tmp[8 + i];
    int b[4] = {a0 + a1, a3 + a2, a3 - a2, a0 - a1};
    for (int k = 0; k < 4; k++) sum += k_weight_y[4 * k + i] * (b[k] < 0 ? -b[k] : b[k]);
  }
  return sum;
}
int or_tdisto4x4(const uint8_t* a, const uint8_t* b) { /* :315 */
  int d = ttransform(b) - ttransform(a);
  return (d < 0 ? -d : d) >> 5;
}
int or_tdisto16x16(const uint8_t* a, const uint8_t* b) { /* :327 */
  int d = 0;
  for (int y = 0; y < 16; y += 4)
    for (int x = 0; x < 16; x += 4) d += or_tdisto4x4(a + x + y * BPS, b + x + y * BPS);
  return d;
}

/* DistoStats :12 and ssimCalculation :48-83 */
typedef struct { uint32_t w, xm, ym, xxm, xym, yym; } stats_t;
static double ssim_calc(const stats_t* s, uint32_t n) {
  uint64_t w2 = (uint64_t)n * n;
  uint64_t c1 = 20 * w2, c2 = 60 * w2, c3 = 8 * 8 * w2;
  uint64_t xmxm = (uint64_t)s->xm * s->xm, ymym = (uint64_t)s->ym * s->ym;
  if (xmxm + ymym < c3) return 1.0;
  int64_t xmym = (int64_t)s->xm * (int64_t)s->ym;
  int64_t sxy = (int64_t)s->xym * (int64_t)n - xmym;
  uint64_t sxx = (uint64_t)s->xxm * n - xmxm;
  uint64_t syy = (uint64_t)s->yym * n - ymym;
  uint64_t sxy_pos = sxy > 0 ? (uint64_t)sxy : 0;
  uint64_t num_s = (2 * sxy_pos + c2) >> 8;
  uint64_t den_s = (sxx + syy + c2) >> 8;
  uint64_t fnum = (2 * (uint64_t)xmym + c1) * num_s;
  uint64_t fden = (xmxm + ymym + c1) * den_s;
  if (fden == 0) return 1.0;
  return (double)fnum / (double)fden;
}
static const uint32_t k_hat[7] = {1, 2, 3, 4, 3, 2, 1}; /* ssimWeight :43 */
static inline void acc(stats_t* s, uint32_t x, uint32_t y, uint32_t w) {
  s->w += w; s->xm += w * x; s->ym += w * y;
  s->xxm += w * x * x; s->xym += w * x * y; s->yym += w * y * y;
}
double or_ssim_get(const uint8_t* s1, int st1, const uint8_t* s2, int st2) { /* :116 */
  stats_t s = {0};
  for (int y = 0; y < 7; y++)
    for (int x = 0; x < 7; x++) acc(&s, s1[x + y * st1], s2[x + y * st2], k_hat[x] * k_hat[y]);
  return s.w == 0 ? 0.0 : ssim_calc(&s, 256);
}
double or_ssim_get_clipped(const uint8_t* s1, int st1, const uint8_t* s2, int st2, int xo, int yo, int W,
                           int H) { /* :132 */
  stats_t s = {0};
  int ymin = yo - 3 < 0 ? 0 : yo - 3, ymax = yo + 3 > H - 1 ? H - 1 : yo + 3;
  int xmin = xo - 3 < 0 ? 0 : xo - 3, xmax = xo + 3 > W - 1 ? W - 1 : xo + 3;
  for (int y = ymin; y <= ymax; y++)
    for (int x = xmin; x <= xmax; x++)
      acc(&s, s1[x + y * st1], s2[x + y * st2], k_hat[3 + x - xo] * k_hat[3 + y - yo]);
  return ssim_calc(&s, s.w);
}

/* libwebp AccumulateSSIM (picture_psnr_enc.c), the plane definition fixed in
 * interior windows use SSIMGet, a 3-px border band uses
 * SSIMGetClipped; summed in raster order. */
double or_plane_ssim(const uint8_t* a, int sa, const uint8_t* b, int sb, int w, int h) {
  const int w0 = w < 3 ? w : 3, w1 = w - 3 - 1;
  const int h0 = h < 3 ? h : 3, h1 = h - 3 - 1;
  double sum = 0.0;
  int x, y;
  for (y = 0; y < h0; y++)
    for (x = 0; x < w; x++) sum += or_ssim_get_clipped(a, sa, b, sb, x, y, w, h);
  for (; y < h1; y++) {
    for (x = 0; x < w0; x++) sum += or_ssim_get_clipped(a, sa, b, sb, x, y, w, h);
    for (; x < w1; x++)
      sum += or_ssim_get(a + (x - 3) + (y - 3) * sa, sa, b + (x - 3) + (y - 3) * sb, sb);
    for (; x < w; x++) sum += or_ssim_get_clipped(a, sa, b, sb, x, y, w, h);
  }
  for (; y < h; y++)
    for (x = 0; x < w; x++) sum += or_ssim_get_clipped(a, sa, b, sb, x, y, w, h);
  return sum;
}

/* DistoStats.Accumulate over a block (SSIMFromBlocks :103-112): Go's uint32
 * fields wrap exactly like these */
void or_disto_stats(const uint8_t* pix, int ps, const uint8_t* ref, int rs, int w, int h, uint32_t out[6]) {
  stats_t s = {0};
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) acc(&s, pix[x + y * ps], ref[x + y * rs], 1);
  out[0] = s.w, out[1] = s.xm, out[2] = s.ym, out[3] = s.xxm, out[4] = s.xym, out[5] = s.yym;
}
/* SSIMFromStats :88 (clipped = 0) / SSIMFromStatsClipped :97 (clipped = 1) */
double or_ssim_from_stats(const uint32_t st[6], int clipped) {
  const stats_t s = {st[0], st[1], st[2], st[3], st[4], st[5]};
  if (clipped) return ssim_calc(&s, s.w);
  return s.w == 0 ? 0.0 : ssim_calc(&s, 256);
}
/* PSNRFromSSE :163-170 with Go's math.Log10 = log2(x) * (Ln2/Ln10) (src/math/log10.go) */
double or_go_log2(double x);
double or_psnr_from_sse(uint64_t sse, int64_t count) {
  if (sse == 0 || count == 0) return 99.0;
  const double mse = (double)sse / (double)count;
  return 10.0 * (or_go_log2(255.0 * 255.0 / mse) * 0x1.34413509f79ffp-2 /* Ln2/Ln10 */);
}

uint64_t or_sse_plane(const uint8_t* a, int sa, const uint8_t* b, int sb, int w, int h) { /* SSE :172 */
  uint64_t s = 0;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int d = a[x + y * sa] - b[x + y * sb];
      s += (uint64_t)(d * d);
    }
  return s;
}
