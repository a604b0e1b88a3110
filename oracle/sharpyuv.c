/* sharpyuv.c -- TEST INFRASTRUCTURE ONLY.  C restatement of the reference's
 * SharpYUV RGB -> YUV420 conversion, sRGB transfer:
 *
 *   sharpyuv/sharpyuv.go:39-64   Convert
 *                        :68-115  convertStandard (SharpEnabled = false)
 *                        :140-168 getPrecisionShift, rgbToGray, scaleDown
 *                        :170-269 convertSharp (import, 4 Gauss-Seidel
 *                                 iterations with early exit, final matrix)
 *                        :271-432 importOneRow, storeGray, updateW,
 *                                 updateChroma, filter2, interpolateTwoRows,
 *                                 sharpYUVUpdateY/RGB, convertWRGBToYUV
 *   sharpyuv/gamma.go:48-123     initGammaTables, shiftVal,
 *                                 fixedPointInterpolation, to/fromLinearSrgb
 *   sharpyuv/csp.go:62-90        conversion matrices
 *
 * The gamma tables come from math.Pow in the reference; here libm pow (the
 * values are rounded to integers, so an ulp difference could only matter at
 * a rounding boundary; the tables are exported so tests can compare).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define YUV_FIX 16
#define YUV_HALF (1 << (YUV_FIX - 1))
#define G2L_BITS 10
#define G2L_SIZE (1 << G2L_BITS)
#define L2G_BITS 9
#define L2G_SIZE (1 << L2G_BITS)
#define G2L_VALUE_BITS 16

static uint32_t g2l[G2L_SIZE + 2], l2g[L2G_SIZE + 2];
static int tables_ready = 0;

/* initGammaTables (gamma.go:48-88) */
static void init_tables(void) {
  if (tables_ready) return;
  const double a = 0.09929682680944, thresh = 0.018053968510807;
  const double gamma_f = 1.0 / 0.45, final_scale = (double)(1u << G2L_VALUE_BITS);
  const double norm = 1.0 / (double)G2L_SIZE, a_rec = 1.0 / (1.0 + a);
  for (int v = 0; v <= G2L_SIZE; v++) {
    const double g = norm * (double)v;
    const double value = g <= thresh * 4.5 ? g / 4.5 : pow(a_rec * (g + a), gamma_f);
    g2l[v] = (uint32_t)(value * final_scale + 0.5);
  }
  g2l[G2L_SIZE + 1] = g2l[G2L_SIZE];
  const double scale = 1.0 / (double)L2G_SIZE;
  for (int v = 0; v <= L2G_SIZE; v++) {
    const double g = scale * (double)v;
    const double value = g <= thresh ? 4.5 * g : (1.0 + a) * pow(g, 1.0 / gamma_f) - a;
    l2g[v] = (uint32_t)(final_scale * value + 0.5);
  }
  l2g[L2G_SIZE + 1] = l2g[L2G_SIZE];
  tables_ready = 1;
}

void or_sharpyuv_tables(uint32_t* g2l_out, uint32_t* l2g_out) {
  init_tables();
  memcpy(g2l_out, g2l, sizeof(g2l));
  memcpy(l2g_out, l2g, sizeof(l2g));
}

static int shift_val(int v, int shift) { return shift >= 0 ? v << shift : v >> -shift; }

/* fixedPointInterpolation (gamma.go:97-109) */
static uint32_t fp_interp(int v, const uint32_t* tab, int pos_shr, int val_shift) {
  const int pos = shift_val(v, -pos_shr);
  const uint32_t x = (uint32_t)(v - shift_val(pos, pos_shr));
  const uint32_t v0 = (uint32_t)shift_val((int)tab[pos], val_shift);
  const uint32_t v1 = (uint32_t)shift_val((int)tab[pos + 1], val_shift);
  const uint32_t v2 = (v1 - v0) * x;
  const int half = pos_shr > 0 ? 1 << (pos_shr - 1) : 0;
  return v0 + ((v2 + (uint32_t)half) >> pos_shr);
}
/* toLinearSrgb / fromLinearSrgb (gamma.go:111-123) */
static uint32_t to_linear(uint16_t v, int bit_depth) {
  const int shift = G2L_BITS - bit_depth;
  if (shift > 0) return g2l[(int)v << shift];
  return fp_interp((int)v, g2l, -shift, 0);
}
static uint16_t from_linear(uint32_t value, int bit_depth) {
  return (uint16_t)fp_interp((int)value, l2g, G2L_VALUE_BITS - L2G_BITS, bit_depth - G2L_VALUE_BITS);
}

/* ---- the other transfer functions, gamma.go:125-446 (float32 arithmetic like
 * the Go code: every float32 operation rounds; powf/log10f/exp/log go through
 * float64 libm and round back, like Go's float32(math.Pow(float64(.), .))) ---- */
static int g_long_double = 0; /* tests: evaluate pow/log10/exp/log in long double to probe rounding margins */
void or_sharpyuv_tf_long_double(int on) { g_long_double = on; }
static float powf_go(float b, float e) {
  return g_long_double ? (float)(double)powl((long double)b, (long double)e) : (float)pow((double)b, (double)e);
}
static float log10f_go(float x) { return g_long_double ? (float)(double)log10l((long double)x) : (float)log10((double)x); }
static float clampf_go(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
static float minf_go(float a, float b) { return a < b ? a : b; }
static float maxf_go(float a, float b) { return a > b ? a : b; }
static float roundf_go(float x) { /* :159-164 */
  return x < 0 ? (float)ceil((double)(x - 0.5f)) : (float)floor((double)(x + 0.5f));
}
/* Constant expressions are exact in Go and rounded once to float32; the
 * literals below are those products / quotients written out (e.g.
 * 4.5*0.018053968510807 = 0.0812428582986315). */
static float to_linear_tf(float g, int tf) {
  switch (tf) {
    case 1: case 6: case 14: case 15: /* toLinear709 :167-176 */
      if (g < 0) return 0;
      if (g < 0.0812428582986315f) return g / 4.5f;
      if (g < 1) return powf_go((g + 0.09929682680944f) / 1.09929682680944f, (float)(1.0 / 0.45));
      return 1;
    case 4: return powf_go(clampf_go(g, 0, 1), 2.2f);                  /* :190 */
    case 5: return powf_go(clampf_go(g, 0, 1), 2.8f);                  /* :199 */
    case 7:                                                          /* :208-217 */
      if (g < 0) return 0;
      if (g < 0.09128634211778f) return g / 4.0f;
      if (g < 1) return powf_go((g + 0.111572195921731f) / 1.111572195921731f, (float)(1.0 / 0.45));
      return 1;
    case 9: /* :231-237 */
      if (g <= 0) return 0.005f;
      return powf_go(10.0f, 2.0f * (minf_go(g, 1.0f) - 1.0f));
    case 10: /* :247-253 */
      if (g <= 0) return 0.00158113883f;
      return powf_go(10.0f, 2.5f * (minf_go(g, 1.0f) - 1.0f));
    case 11: /* :263-270 */
      if (g <= -0.0812428582986315f) return powf_go((-g + 0.09929682680944f) / -1.09929682680944f, (float)(1.0 / 0.45));
      if (g < 0.0812428582986315f) return g / 4.5f;
      return powf_go((g + 0.09929682680944f) / 1.09929682680944f, (float)(1.0 / 0.45));
    case 12: /* :282-293 */
      if (g < -0.25f) return -0.25f;
      if (g < 0) return powf_go((g - 0.02482420670236f) / -0.27482420670236f, (float)(1.0 / 0.45)) / -4.0f;
      if (g < 0.0812428582986315f) return g / 4.5f;
      if (g < 1) return powf_go((g + 0.09929682680944f) / 1.09929682680944f, (float)(1.0 / 0.45));
      return 1;
    case 16: /* PQ :309-317 */
      if (g > 0) {
        const float pg = powf_go(g, (float)(32.0 / 2523.0));
        const float num = maxf_go(pg - 0.8359375f, 0.0f);
        const float den = maxf_go(18.8515625f - 18.6875f * pg, 1.401298464324817e-45f);
        return powf_go(num / den, (float)(4096.0 / 653.0));
      }
      return 0;
    case 17: return powf_go(maxf_go(g, 0), 2.6f) / 0.91655527974030934f; /* :330 */
    case 18: /* HLG :339-346 */
      if (g < 0) return 0;
      if (g <= 0.5f) return powf_go((g * g) * (float)(1.0 / 3.0), 1.2f);
      {
        const double e = g_long_double ? (double)expl((long double)((g - 0.55991073f) / 0.17883277f))
                                       : exp((double)((g - 0.55991073f) / 0.17883277f));
        return powf_go(((float)e + 0.28466892f) / 12.0f, 1.2f);
      }
    default: return 0;
  }
}
static float from_linear_tf(float l, int tf) {
  switch (tf) {
    case 1: case 6: case 14: case 15: /* fromLinear709 :178-187 */
      if (l < 0) return 0;
      if (l < 0.018053968510807f) return l * 4.5f;
      if (l < 1) return 1.09929682680944f * powf_go(l, 0.45f) - 0.09929682680944f;
      return 1;
    case 4: return powf_go(clampf_go(l, 0, 1), (float)(1.0 / 2.2)); /* :194 */
    case 5: return powf_go(clampf_go(l, 0, 1), (float)(1.0 / 2.8)); /* :203 */
    case 7:                                                        /* :219-228 */
      if (l < 0) return 0;
      if (l < 0.022821585529445f) return l * 4.0f;
      if (l < 1) return 1.111572195921731f * powf_go(l, 0.45f) - 0.111572195921731f;
      return 1;
    case 9: /* :239-244 */
      if (l < 0.01f) return 0;
      return 1.0f + log10f_go(minf_go(l, 1.0f)) / 2.0f;
    case 10: /* :255-260 */
      if (l < 0.00316227766f) return 0;
      return 1.0f + log10f_go(minf_go(l, 1.0f)) / 2.5f;
    case 11: /* :272-279 */
      if (l <= -0.018053968510807f) return -1.09929682680944f * powf_go(-l, 0.45f) + 0.09929682680944f;
      if (l < 0.018053968510807f) return l * 4.5f;
      return 1.09929682680944f * powf_go(l, 0.45f) - 0.09929682680944f;
    case 12: /* :295-306 */
      if (l < -0.25f) return -0.25f;
      if (l < 0) return -0.27482420670236f * powf_go(-4.0f * l, 0.45f) + 0.02482420670236f;
      if (l < 0.018053968510807f) return l * 4.5f;
      if (l < 1) return 1.09929682680944f * powf_go(l, 0.45f) - 0.09929682680944f;
      return 1;
    case 16: /* PQ :319-327 */
      if (l > 0) {
        const float pl = powf_go(l, (float)(653.0 / 4096.0));
        const float num = 0.8359375f + 18.8515625f * pl;
        const float den = 1.0f + 18.6875f * pl;
        return powf_go(num / den, (float)(2523.0 / 32.0));
      }
      return 0;
    case 17: return powf_go(0.91655527974030934f * maxf_go(l, 0), (float)(1.0 / 2.6)); /* :334 */
    case 18: /* HLG :348-356 */
      l = powf_go(l, (float)(1.0 / 1.2));
      if (l < 0) return 0;
      if (l <= (float)(1.0 / 12.0)) return (float)sqrt((double)(3.0f * l));
      return 0.17883277f * (float)(g_long_double ? (double)logl((long double)(12.0f * l - 0.28466892f))
                                                 : log((double)(12.0f * l - 0.28466892f))) + 0.55991073f;
    default: return 0;
  }
}
/* GammaToLinear / LinearToGamma (gamma.go:360-446) */
uint32_t or_sharpyuv_gamma_to_linear(uint16_t v, int bit_depth, int tf) {
  init_tables();
  if (tf == 13) return to_linear(v, bit_depth);
  if (tf == 8) return v;
  const float vf = (float)v / (float)((1 << bit_depth) - 1);
  return (uint32_t)(int64_t)roundf_go(to_linear_tf(vf, tf) * 65535.0f);
}
uint16_t or_sharpyuv_linear_to_gamma(uint32_t v, int bit_depth, int tf) {
  init_tables();
  if (tf == 13) return from_linear(v, bit_depth);
  if (tf == 8) return (uint16_t)v;
  const float vf = (float)v / 65535.0f;
  return (uint16_t)(int64_t)roundf_go(from_linear_tf(vf, tf) * (float)((1 << bit_depth) - 1));
}
static int g_tf = 13; /* transfer of the conversion in progress (the oracle is single-threaded per call) */
static uint32_t to_lin(uint16_t v, int bd) { return g_tf == 13 ? to_linear(v, bd) : or_sharpyuv_gamma_to_linear(v, bd, g_tf); }
static uint16_t from_lin(uint32_t v, int bd) { return g_tf == 13 ? from_linear(v, bd) : or_sharpyuv_linear_to_gamma(v, bd, g_tf); }

static int rgb_to_gray(int64_t r, int64_t g, int64_t b) {
  return (int)((13933 * r + 46871 * g + 4732 * b + YUV_HALF) >> YUV_FIX);
}
static uint32_t scale_down(uint16_t a, uint16_t b, uint16_t c, uint16_t d, int bd) {
  const uint32_t la = to_lin(a, bd), lb = to_lin(b, bd), lc = to_lin(c, bd), ld = to_lin(d, bd);
  return from_lin((la + lb + lc + ld + 2) >> 2, bd);
}
static uint16_t clip_bd(int y, int bd) {
  const int mx = (1 << bd) - 1;
  return (uint16_t)(y < 0 ? 0 : (y > mx ? mx : y));
}
static uint8_t clip_u8(int32_t v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

static void import_row(const uint8_t* rgb, int row, int stride, int pic_w, int w, int sfix, uint16_t* dst) {
  const uint8_t* p = rgb + (size_t)row * stride;
  for (int i = 0; i < pic_w; i++) {
    dst[i] = (uint16_t)shift_val(p[3 * i + 0], sfix);
    dst[i + w] = (uint16_t)shift_val(p[3 * i + 1], sfix);
    dst[i + 2 * w] = (uint16_t)shift_val(p[3 * i + 2], sfix);
  }
  if (pic_w < w) {
    dst[pic_w] = dst[pic_w - 1];
    dst[pic_w + w] = dst[pic_w + w - 1];
    dst[pic_w + 2 * w] = dst[pic_w + 2 * w - 1];
  }
}
static void store_gray(const uint16_t* src, uint16_t* y, int w) {
  for (int i = 0; i < w; i++) y[i] = (uint16_t)rgb_to_gray(src[i], src[i + w], src[i + 2 * w]);
}
static void update_w(const uint16_t* src, uint16_t* dst, int w, int bd) {
  for (int i = 0; i < w; i++) {
    const uint32_t r = to_lin(src[i], bd), g = to_lin(src[i + w], bd), b = to_lin(src[i + 2 * w], bd);
    dst[i] = from_lin((uint32_t)rgb_to_gray(r, g, b), bd);
  }
}
static void update_chroma(const uint16_t* s1, const uint16_t* s2, int16_t* dst, int uvw, int bd) {
  const int w = uvw * 2;
  for (int i = 0; i < uvw; i++) {
    const int i2 = 2 * i;
    const int r = (int)scale_down(s1[i2], s1[i2 + 1], s2[i2], s2[i2 + 1], bd);
    const int g = (int)scale_down(s1[i2 + w], s1[i2 + w + 1], s2[i2 + w], s2[i2 + w + 1], bd);
    const int b = (int)scale_down(s1[i2 + 2 * w], s1[i2 + 2 * w + 1], s2[i2 + 2 * w], s2[i2 + 2 * w + 1], bd);
    const int gray = rgb_to_gray(r, g, b);
    dst[i] = (int16_t)(r - gray);
    dst[i + uvw] = (int16_t)(g - gray);
    dst[i + 2 * uvw] = (int16_t)(b - gray);
  }
}
static uint16_t filter2(int a, int b, int w0, int bd) { return clip_bd(((a * 3 + b + 2) >> 2) + w0, bd); }
static void interpolate_two_rows(const uint16_t* best_y, const int16_t* prev, const int16_t* cur, const int16_t* next,
                                 int w, uint16_t* out1, uint16_t* out2, int bd) {
  const int uvw = w >> 1, flen = (w - 1) >> 1;
  for (int k = 0; k < 3; k++) {
    const int ku = k * uvw, kw = k * w;
    out1[kw] = filter2(cur[ku], prev[ku], best_y[0], bd);
    out2[kw] = filter2(cur[ku], next[ku], best_y[w], bd);
    for (int i = 0; i < flen; i++) {
      const int a0 = cur[ku + i], a1 = cur[ku + i + 1], b0 = prev[ku + i], b1 = prev[ku + i + 1];
      const int v0 = (a0 * 9 + a1 * 3 + b0 * 3 + b1 + 8) >> 4;
      const int v1 = (a1 * 9 + a0 * 3 + b1 * 3 + b0 + 8) >> 4;
      out1[kw + 2 * i + 1] = clip_bd(best_y[2 * i + 1] + v0, bd);
      out1[kw + 2 * i + 2] = clip_bd(best_y[2 * i + 2] + v1, bd);
      const int n0 = next[ku + i], n1 = next[ku + i + 1];
      const int nv0 = (a0 * 9 + a1 * 3 + n0 * 3 + n1 + 8) >> 4;
      const int nv1 = (a1 * 9 + a0 * 3 + n1 * 3 + n0 + 8) >> 4;
      out2[kw + 2 * i + 1] = clip_bd(best_y[w + 2 * i + 1] + nv0, bd);
      out2[kw + 2 * i + 2] = clip_bd(best_y[w + 2 * i + 2] + nv1, bd);
    }
    if ((w & 1) == 0) {
      out1[kw + w - 1] = filter2(cur[ku + uvw - 1], prev[ku + uvw - 1], best_y[w - 1], bd);
      out2[kw + w - 1] = filter2(cur[ku + uvw - 1], next[ku + uvw - 1], best_y[2 * w - 1], bd);
    }
  }
}
static uint64_t update_y(const uint16_t* target, const uint16_t* src, uint16_t* dst, int len, int bd) {
  uint64_t diff = 0;
  const int max_y = (1 << bd) - 1;
  for (int i = 0; i < len; i++) {
    const int d = (int)target[i] - (int)src[i];
    const int ny = (int)dst[i] + d;
    dst[i] = (uint16_t)(ny < 0 ? 0 : (ny > max_y ? max_y : ny));
    diff += (uint64_t)(d < 0 ? -d : d);
  }
  return diff;
}
static void update_rgb(const int16_t* target, const int16_t* src, int16_t* dst, int len) {
  for (int i = 0; i < len; i++) {
    const int16_t d = (int16_t)(target[i] - src[i]); /* int16 arithmetic wraps, as in Go */
    dst[i] = (int16_t)(dst[i] + d);
  }
}

/* matrix: rgb_to_y[4], rgb_to_u[4], rgb_to_v[4] (csp.go ConversionMatrix) */
static void convert_wrgb_to_yuv(const uint16_t* best_y, const int16_t* best_uv, uint8_t* y, int y_stride, uint8_t* u,
                                uint8_t* v, int uv_stride, int width, int height, int w, int uvw, int uvh, int sfix,
                                const int32_t* m) {
  const int64_t rounder = (int64_t)1 << (YUV_FIX + sfix - 1);
  const int64_t y_off = shift_val(m[3], sfix), u_off = shift_val(m[7], sfix), v_off = shift_val(m[11], sfix);
  for (int j = 0; j < height; j++)
    for (int i = 0; i < width; i++) {
      const int uvi = (j / 2) * 3 * uvw + (i >> 1);
      const int64_t wv = best_y[j * w + i];
      const int64_t r = best_uv[uvi] + wv, g = best_uv[uvi + uvw] + wv, b = best_uv[uvi + 2 * uvw] + wv;
      const int64_t yv = (int64_t)m[0] * r + (int64_t)m[1] * g + (int64_t)m[2] * b + y_off + rounder;
      y[(size_t)j * y_stride + i] = clip_u8((int32_t)(yv >> (YUV_FIX + sfix)));
    }
  for (int j = 0; j < uvh; j++)
    for (int i = 0; i < uvw; i++) {
      const int uvi = j * 3 * uvw + i;
      const int64_t r = best_uv[uvi], g = best_uv[uvi + uvw], b = best_uv[uvi + 2 * uvw];
      const int64_t uv = (int64_t)m[4] * r + (int64_t)m[5] * g + (int64_t)m[6] * b + u_off + rounder;
      const int64_t vv = (int64_t)m[8] * r + (int64_t)m[9] * g + (int64_t)m[10] * b + v_off + rounder;
      u[(size_t)j * uv_stride + i] = clip_u8((int32_t)(uv >> (YUV_FIX + sfix)));
      v[(size_t)j * uv_stride + i] = clip_u8((int32_t)(vv >> (YUV_FIX + sfix)));
    }
}

/* convertStandard (sharpyuv.go:68-115) */
static int32_t rgb_to_yuv_component(int32_t r, int32_t g, int32_t b, const int32_t* c) {
  const int64_t luma = (int64_t)c[0] * r + (int64_t)c[1] * g + (int64_t)c[2] * b + (int64_t)c[3] + YUV_HALF;
  return (int32_t)(luma >> YUV_FIX);
}
void or_sharpyuv_convert_standard(const uint8_t* rgb, int width, int height, int rgb_stride, uint8_t* y, int y_stride,
                                  uint8_t* u, uint8_t* v, int uv_stride, const int32_t* m) {
  for (int j = 0; j < height; j++)
    for (int i = 0; i < width; i++) {
      const uint8_t* p = rgb + (size_t)j * rgb_stride + 3 * i;
      y[(size_t)j * y_stride + i] = clip_u8(rgb_to_yuv_component(p[0], p[1], p[2], m));
    }
  const int uvw = (width + 1) >> 1, uvh = (height + 1) >> 1;
  for (int j = 0; j < uvh; j++)
    for (int i = 0; i < uvw; i++) {
      int32_t sr = 0, sg = 0, sb = 0, n = 0;
      for (int dy = 0; dy < 2; dy++) {
        const int yy = 2 * j + dy;
        if (yy >= height) continue;
        for (int dx = 0; dx < 2; dx++) {
          const int xx = 2 * i + dx;
          if (xx >= width) continue;
          const uint8_t* p = rgb + (size_t)yy * rgb_stride + 3 * xx;
          sr += p[0];
          sg += p[1];
          sb += p[2];
          n++;
        }
      }
      const int32_t ar = (sr + n / 2) / n, ag = (sg + n / 2) / n, ab = (sb + n / 2) / n;
      u[(size_t)j * uv_stride + i] = clip_u8(rgb_to_yuv_component(ar, ag, ab, m + 4));
      v[(size_t)j * uv_stride + i] = clip_u8(rgb_to_yuv_component(ar, ag, ab, m + 8));
    }
}

int or_sharpyuv_convert(const uint8_t* rgb, int width, int height, int rgb_stride, uint8_t* y, int y_stride,
                        uint8_t* u, uint8_t* v, int uv_stride, const int32_t* matrix) {
  return or_sharpyuv_convert_tf(rgb, width, height, rgb_stride, y, y_stride, u, v, uv_stride, matrix, 13);
}

/* convertSharp (sharpyuv.go:170-269) with transfer function tf (H.273 code,
 * gamma.go:11-28).  Returns the number of iterations run. */
int or_sharpyuv_convert_tf(const uint8_t* rgb, int width, int height, int rgb_stride, uint8_t* y, int y_stride,
                           uint8_t* u, uint8_t* v, int uv_stride, const int32_t* matrix, int tf) {
  init_tables();
  g_tf = tf;
  const int w = (width + 1) & ~1, h = (height + 1) & ~1;
  const int uvw = w >> 1, uvh = h >> 1, sfix = 2, bd = 8 + sfix;
  uint16_t* tmp1 = malloc(sizeof(uint16_t) * 3 * w);
  uint16_t* tmp2 = malloc(sizeof(uint16_t) * 3 * w);
  uint16_t* best_y = malloc(sizeof(uint16_t) * w * h);
  uint16_t* target_y = malloc(sizeof(uint16_t) * w * h);
  int16_t* best_uv = malloc(sizeof(int16_t) * 3 * uvw * uvh);
  int16_t* target_uv = malloc(sizeof(int16_t) * 3 * uvw * uvh);
  uint16_t* best_rgb_y = malloc(sizeof(uint16_t) * 2 * w);
  int16_t* best_rgb_uv = malloc(sizeof(int16_t) * 3 * uvw);
  for (int j = 0; j < height; j += 2) {
    const int last = j == height - 1;
    import_row(rgb, j, rgb_stride, width, w, sfix, tmp1);
    if (!last) import_row(rgb, j + 1, rgb_stride, width, w, sfix, tmp2);
    else memcpy(tmp2, tmp1, sizeof(uint16_t) * 3 * w);
    const int boff = (j / 2) * 2 * w, uoff = (j / 2) * 3 * uvw;
    store_gray(tmp1, best_y + boff, w);
    store_gray(tmp2, best_y + boff + w, w);
    update_w(tmp1, target_y + boff, w, bd);
    update_w(tmp2, target_y + boff + w, w, bd);
    update_chroma(tmp1, tmp2, target_uv + uoff, uvw, bd);
    memcpy(best_uv + uoff, target_uv + uoff, sizeof(int16_t) * 3 * uvw);
  }
  const uint64_t thr = (uint64_t)3 * w * h;
  uint64_t prev_sum = ~(uint64_t)0;
  int iters = 0;
  for (int it = 0; it < 4; it++) {
    uint64_t sum = 0;
    for (int j = 0; j < h; j += 2) {
      const int ju = j / 2;
      const int cur = ju * 3 * uvw;
      const int prev = ju > 0 ? (ju - 1) * 3 * uvw : cur;
      const int next = j < h - 2 ? (ju + 1) * 3 * uvw : cur;
      interpolate_two_rows(best_y + j * w, best_uv + prev, best_uv + cur, best_uv + next, w, tmp1, tmp2, bd);
      update_w(tmp1, best_rgb_y, w, bd);
      update_w(tmp2, best_rgb_y + w, w, bd);
      update_chroma(tmp1, tmp2, best_rgb_uv, uvw, bd);
      sum += update_y(target_y + j * w, best_rgb_y, best_y + j * w, 2 * w, bd);
      update_rgb(target_uv + ju * 3 * uvw, best_rgb_uv, best_uv + cur, 3 * uvw);
    }
    iters++;
    if (it > 0 && (sum < thr || sum > prev_sum)) break;
    prev_sum = sum;
  }
  convert_wrgb_to_yuv(best_y, best_uv, y, y_stride, u, v, uv_stride, width, height, w, uvw, uvh, sfix, matrix);
  free(tmp1);
  free(tmp2);
  free(best_y);
  free(target_y);
  free(best_uv);
  free(target_uv);
  free(best_rgb_y);
  free(best_rgb_uv);
  return iters;
}
