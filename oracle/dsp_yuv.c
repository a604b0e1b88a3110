/*
 * dsp_yuv.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates internal/dsp/yuv.go (YUV<->RGB, gamma tables, AccumulateRGBA),
 * internal/dsp/random.go, internal/dsp/upsample.go and webp.go:379-450
 * (buildNRGBA).
 */
#include <math.h>
#include <string.h>
#include "oracle.h"

/* ---------------- YUV -> RGB, yuv.go:11-118 ---------------- */
static inline int mult_hi(int v, int c) { return (v * c) >> 8; } /* :38 */
static inline uint8_t clip_yuv(int val) {                          /* vp8kClip lookup :44-58 */
  if (val < 0) return 0;
  if (val > (256 << 6) - 1) return 255;
  return (uint8_t)(val >> 6);
}
void or_yuv_to_rgb(int y, int u, int v, uint8_t* rgb) { /* :71-109 */
  int yy = mult_hi(y, 19077);
  rgb[0] = clip_yuv(yy + mult_hi(v, 26149) - 14234);
  rgb[1] = clip_yuv(yy - mult_hi(u, 6419) - mult_hi(v, 13320) + 8708);
  rgb[2] = clip_yuv(yy + mult_hi(u, 33050) - 17685);
}

/* ---------------- RGB -> YUV, yuv.go:124-171 ---------------- */
static int clip_uv(int uv, int rounding) { /* VP8ClipUV :138 */
  uv = (uv + rounding + (128 << 18)) >> 18;
  return (uv & ~0xff) == 0 ? uv : (uv < 0 ? 0 : 255);
}
int or_rgb_to_y(int r, int g, int b) { return (16839 * r + 33059 * g + 6420 * b + (1 << 15) + (16 << 16)) >> 16; }
int or_rgb_to_u(int r, int g, int b, int rnd) { return clip_uv(-9719 * r - 19081 * g + 28800 * b, rnd); }
int or_rgb_to_v(int r, int g, int b, int rnd) { return clip_uv(28800 * r - 24116 * g - 4684 * b, rnd); }

/* ---------------- gamma tables, yuv.go:176-249 ---------------- */
static uint32_t g_to_lin[256];
static uint32_t lin_to_g[34];
static int gamma_ready = 0;
static void init_gamma(void) { /* InitGammaTables :193-215 (float64 pow, robust to libm) */
  if (gamma_ready) return;
  for (int i = 0; i < 256; i++) {
    double v = (double)i / 255.0;
    double lin = (v <= 0 ? 0.0 : pow(v, 0.80)) * 4095.0;
    g_to_lin[i] = (uint32_t)(lin + 0.5);
  }
  double scale = 128.0 / 4095.0;
  for (int i = 0; i <= 32; i++) {
    double v = scale * (double)i;
    double g = (v <= 0 ? 0.0 : pow(v, 1.0 / 0.80)) * 255.0;
    lin_to_g[i] = (uint32_t)(g + 0.5);
  }
  lin_to_g[33] = 255;
  gamma_ready = 1;
}
uint32_t or_gamma_to_linear(int v) { init_gamma(); return g_to_lin[v & 255]; }
int or_linear_to_gamma(uint32_t base, int shift) { /* :236-249 */
  init_gamma();
  int v = (int)base << shift;
  int pos = v >> (7 + 2);
  if (pos >= 32) pos = 31;
  int x = v & ((128 << 2) - 1);
  int v0 = (int)lin_to_g[pos], v1 = (int)lin_to_g[pos + 1];
  int y = v1 * x + v0 * ((128 << 2) - x);
  return (y + 64) >> 7;
}

/* divideByAlpha :453 with kInvAlpha[a] = floor(2^19 / a) (yuv.go:343-447, checked entry by entry) */
static inline uint32_t inv_alpha(uint32_t a) { return a ? (1u << 19) / a : 0; }
static int lin_to_gamma_weighted(const uint8_t s[4], const uint8_t al[4], uint32_t total) { /* :466 */
  uint32_t sum = 0;
  for (int k = 0; k < 4; k++) sum += (uint32_t)al[k] * g_to_lin[s[k]];
  return or_linear_to_gamma((sum * inv_alpha(total)) >> (19 - 2), 0);
}

void or_accumulate_rgba(const uint8_t* r, const uint8_t* g, const uint8_t* b, const uint8_t* a,
                        int stride, uint16_t* dst, int width) { /* :486-547 */
  init_gamma();
  const uint8_t* ch[3] = {r, g, b};
  int j = 0;
  for (int i = 0; i < (width >> 1); i++, j += 2, dst += 4) {
    uint32_t ta = (uint32_t)a[j] + a[j + 1] + a[j + stride] + a[j + stride + 1];
    for (int c = 0; c < 3; c++) {
      const uint8_t* p = ch[c];
      if (ta == 4 * 255 || ta == 0) {
        dst[c] = (uint16_t)or_linear_to_gamma(g_to_lin[p[j]] + g_to_lin[p[j + 1]] +
                                              g_to_lin[p[j + stride]] + g_to_lin[p[j + stride + 1]], 0);
      } else {
        uint8_t s[4] = {p[j], p[j + 1], p[j + stride], p[j + stride + 1]};
        uint8_t al[4] = {a[j], a[j + 1], a[j + stride], a[j + stride + 1]};
        dst[c] = (uint16_t)lin_to_gamma_weighted(s, al, ta);
      }
    }
    dst[3] = (uint16_t)ta;
  }
  if (width & 1) { /* odd last column :519-546 */
    uint32_t ta = 2 * ((uint32_t)a[j] + a[j + stride]);
    for (int c = 0; c < 3; c++) {
      const uint8_t* p = ch[c];
      if (ta == 4 * 255 || ta == 0) {
        dst[c] = (uint16_t)or_linear_to_gamma(g_to_lin[p[j]] + g_to_lin[p[j + stride]], 1);
      } else {
        uint8_t s[4] = {p[j], p[j], p[j + stride], p[j + stride]};
        uint8_t al[4] = {a[j], a[j], a[j + stride], a[j + stride]};
        dst[c] = (uint16_t)lin_to_gamma_weighted(s, al, ta);
      }
    }
    dst[3] = (uint16_t)ta;
  }
}

void or_convert_rgba32_to_uv(const uint16_t* rgb, uint8_t* u, uint8_t* v, int width) { /* :553 */
  const int rnd = (1 << 15) << 2;
  for (int i = 0; i < width; i++) {
    u[i] = (uint8_t)or_rgb_to_u(rgb[4 * i], rgb[4 * i + 1], rgb[4 * i + 2], rnd);
    v[i] = (uint8_t)or_rgb_to_v(rgb[4 * i], rgb[4 * i + 1], rgb[4 * i + 2], rnd);
  }
}

/* ConvertARGBToY (yuv.go:270-278): packed 0xAARRGGBB -> RGBToY per pixel */
void or_convert_argb_to_y(const uint32_t* argb, uint8_t* y, int width) {
  for (int i = 0; i < width; i++) {
    const uint32_t p = argb[i];
    y[i] = (uint8_t)or_rgb_to_y((int)((p >> 16) & 0xff), (int)((p >> 8) & 0xff), (int)(p & 0xff));
  }
}

/* ConvertARGBToUV (yuv.go:291-330): a pixel pair per U/V sample, its
 * channels doubled into the sum-of-4 scale (the odd last pixel x4); do_store
 * writes the sample, else averages it into u/v ((old + new + 1) >> 1) */
void or_convert_argb_to_uv(const uint32_t* argb, uint8_t* u, uint8_t* v, int src_width, int do_store) {
  const int uv_width = src_width >> 1, rnd = (1 << 15) << 2;
  for (int i = 0; i <= uv_width; i++) {
    int r, g, b;
    if (i < uv_width) {
      const uint32_t v0 = argb[2 * i], v1 = argb[2 * i + 1];
      r = (int)((v0 >> 15) & 0x1fe) + (int)((v1 >> 15) & 0x1fe);
      g = (int)((v0 >> 7) & 0x1fe) + (int)((v1 >> 7) & 0x1fe);
      b = (int)((v0 << 1) & 0x1fe) + (int)((v1 << 1) & 0x1fe);
    } else {
      if (!(src_width & 1)) break;
      const uint32_t v0 = argb[2 * uv_width];
      r = (int)((v0 >> 14) & 0x3fc);
      g = (int)((v0 >> 6) & 0x3fc);
      b = (int)((v0 << 2) & 0x3fc);
    }
    const int tu = or_rgb_to_u(r, g, b, rnd), tv = or_rgb_to_v(r, g, b, rnd);
    if (do_store) {
      u[i] = (uint8_t)tu;
      v[i] = (uint8_t)tv;
    } else {
      u[i] = (uint8_t)((u[i] + tu + 1) >> 1);
      v[i] = (uint8_t)((v[i] + tv + 1) >> 1);
    }
  }
}

/* ---------------- VP8Random, random.go ---------------- */
void or_convert_rgba32_to_uv_dithered(const uint16_t* rgb, uint8_t* u, uint8_t* v, int width, or_random* rg) { /* :568 */
  for (int i = 0; i < width; i++) {
    const int r = rgb[4 * i], g = rgb[4 * i + 1], b = rgb[4 * i + 2];
    u[i] = (uint8_t)or_rgb_to_u(r, g, b, or_random_bits2(rg, 18, rg->amp));
    v[i] = (uint8_t)or_rgb_to_v(r, g, b, or_random_bits2(rg, 18, rg->amp));
  }
}

static const uint32_t k_random_table[55] = { /* random.go:24-35 (libwebp random_utils.c) */
  0x0de15230, 0x03b31886, 0x775faccb, 0x1c88626a, 0x68385c55, 0x14b3b828, 0x4a85fef8, 0x49ddb84b,
  0x64fcf397, 0x5c550289, 0x4a290000, 0x0d7ec1da, 0x5940b7ab, 0x5492577d, 0x4e19ca72, 0x38d38c69,
  0x0c01ee65, 0x32a1755f, 0x5437f652, 0x5abb2c32, 0x0faa57b1, 0x73f533e7, 0x685feeda, 0x7563cce2,
  0x6e990e83, 0x4730a7ed, 0x4fc0d9c6, 0x496b153c, 0x4f1403fa, 0x541afb0c, 0x73990b32, 0x26d7cb1c,
  0x6fcc3706, 0x2cbb77d8, 0x75762f2a, 0x6425ccdd, 0x24b35461, 0x0a7d8715, 0x220414a8, 0x141ebf67,
  0x56b41583, 0x73e502e3, 0x44cab16f, 0x28264d42, 0x73baaefb, 0x0a50ebed, 0x1d6ab6fb, 0x0d3ad40b,
  0x35db3b68, 0x2b081e83, 0x77ce6b95, 0x5181e5f0, 0x78853bbc, 0x009f9494, 0x27e5ed3c};
void or_random_init(or_random* rg, float dithering) { /* :39 */
  memcpy(rg->tab, k_random_table, sizeof(k_random_table));
  rg->index1 = 0;
  rg->index2 = 31;
  if (dithering < 0.0f) rg->amp = 0;
  else if (dithering > 1.0f) rg->amp = 1 << 8;
  else rg->amp = (int)((float)(1 << 8) * dithering);
}
int or_random_bits2(or_random* rg, int num_bits, int amp) { /* :54 */
  int64_t diff = (int64_t)rg->tab[rg->index1] - (int64_t)rg->tab[rg->index2];
  if (diff < 0) diff += (int64_t)1 << 31;
  rg->tab[rg->index1] = (uint32_t)diff;
  if (++rg->index1 == 55) rg->index1 = 0;
  if (++rg->index2 == 55) rg->index2 = 0;
  int64_t d = (int64_t)(int32_t)((uint32_t)diff << 1) >> (32 - num_bits);
  d = (d * amp) >> 8;
  d += (int64_t)1 << (num_bits - 1);
  return (int)d;
}

/* ---------------- fancy upsampler, upsample.go:45-236 ----------------
 * Per-channel form of the packed-UV diamond kernel (the u/v halves never
 * carry into each other, SURVEY 7 traps). */
typedef void (*emit_fn)(uint8_t* dst, int x, int y, int u, int v, const uint8_t* alpha);
static void emit_rgb(uint8_t* dst, int x, int y, int u, int v, const uint8_t* alpha) {
  (void)alpha;
  or_yuv_to_rgb(y, u, v, dst + 3 * x);
}
static void emit_nrgba(uint8_t* dst, int x, int y, int u, int v, const uint8_t* alpha) {
  or_yuv_to_rgb(y, u, v, dst + 4 * x);
  dst[4 * x + 3] = alpha ? alpha[x] : 255;
}

static void upsample_pair(const uint8_t* ty, const uint8_t* by, const uint8_t* tu, const uint8_t* tv,
                          const uint8_t* bu, const uint8_t* bv, uint8_t* td, uint8_t* bd,
                          const uint8_t* at, const uint8_t* ab, int width, emit_fn emit) {
  if (width <= 0) return;
  const uint8_t* cin[2][2] = {{tu, bu}, {tv, bv}}; /* [channel][top/bottom chroma row] */
  int last_pair = (width - 1) >> 1;
  int tl[2], l[2];
  int out_t[2][2], out_b[2][2];
  for (int c = 0; c < 2; c++) { tl[c] = cin[c][0][0]; l[c] = cin[c][1][0]; }
  /* first pixel, vertical interpolation only */
  emit(td, 0, ty[0], (3 * tl[0] + l[0] + 2) >> 2, (3 * tl[1] + l[1] + 2) >> 2, at);
  if (by) emit(bd, 0, by[0], (3 * l[0] + tl[0] + 2) >> 2, (3 * l[1] + tl[1] + 2) >> 2, ab);
  for (int x = 1; x <= last_pair; x++) {
    for (int c = 0; c < 2; c++) {
      int t = cin[c][0][x], cur = cin[c][1][x];
      int avg = tl[c] + t + l[c] + cur + 8;
      int diag12 = (avg + 2 * (t + l[c])) >> 3;
      int diag03 = (avg + 2 * (tl[c] + cur)) >> 3;
      out_t[c][0] = (diag12 + tl[c]) >> 1;
      out_t[c][1] = (diag03 + t) >> 1;
      out_b[c][0] = (diag03 + l[c]) >> 1;
      out_b[c][1] = (diag12 + cur) >> 1;
      tl[c] = t;
      l[c] = cur;
    }
    emit(td, 2 * x - 1, ty[2 * x - 1], out_t[0][0], out_t[1][0], at);
    emit(td, 2 * x, ty[2 * x], out_t[0][1], out_t[1][1], at);
    if (by) {
      emit(bd, 2 * x - 1, by[2 * x - 1], out_b[0][0], out_b[1][0], ab);
      emit(bd, 2 * x, by[2 * x], out_b[0][1], out_b[1][1], ab);
    }
  }
  if ((width & 1) == 0) { /* last pixel for even widths */
    emit(td, width - 1, ty[width - 1], (3 * tl[0] + l[0] + 2) >> 2, (3 * tl[1] + l[1] + 2) >> 2, at);
    if (by) emit(bd, width - 1, by[width - 1], (3 * l[0] + tl[0] + 2) >> 2, (3 * l[1] + tl[1] + 2) >> 2, ab);
  }
}

void or_upsample_line_pair_rgb(const uint8_t* ty, const uint8_t* by, const uint8_t* tu, const uint8_t* tv,
                               const uint8_t* bu, const uint8_t* bv, uint8_t* td, uint8_t* bd, int width) {
  upsample_pair(ty, by, tu, tv, bu, bv, td, bd, NULL, NULL, width, emit_rgb);
}
void or_upsample_line_pair_nrgba(const uint8_t* ty, const uint8_t* by, const uint8_t* tu, const uint8_t* tv,
                                 const uint8_t* bu, const uint8_t* bv, uint8_t* td, uint8_t* bd,
                                 const uint8_t* at, const uint8_t* ab, int width) {
  upsample_pair(ty, by, tu, tv, bu, bv, td, bd, at, ab, width, emit_nrgba);
}

/* PointSampleRow (upsample.go:238-245): nearest chroma sample, RGB 3 B/px */
void or_point_sample_row(const uint8_t* y, const uint8_t* u, const uint8_t* v, uint8_t* dst, int width) {
  for (int x = 0; x < width; x++) or_yuv_to_rgb(y[x], u[x >> 1], v[x >> 1], dst + 3 * x);
}

/* buildNRGBA webp.go:379-450 */
void or_build_nrgba(int w, int h, const uint8_t* y, int ys, const uint8_t* u, const uint8_t* v, int uvs,
                    const uint8_t* alpha, uint8_t* out) {
#define YR(r) (y + (size_t)(r) * ys)
#define UR(r) (u + (size_t)(r) * uvs)
#define VR(r) (v + (size_t)(r) * uvs)
#define AR(r) (alpha ? alpha + (size_t)(r) * w : NULL)
#define OR(r) (out + (size_t)(r) * 4 * w)
  or_upsample_line_pair_nrgba(YR(0), NULL, UR(0), VR(0), UR(0), VR(0), OR(0), NULL, AR(0), NULL, w);
  if (h == 1) return;
  int r = 0;
  for (; r + 2 < h; r += 2) {
    int ct = r / 2, cb = ct + 1;
    or_upsample_line_pair_nrgba(YR(r + 1), YR(r + 2), UR(ct), VR(ct), UR(cb), VR(cb), OR(r + 1), OR(r + 2),
                                AR(r + 1), AR(r + 2), w);
  }
  if ((h & 1) == 0) {
    int lc = (h - 1) / 2;
    or_upsample_line_pair_nrgba(YR(h - 1), NULL, UR(lc), VR(lc), UR(lc), VR(lc), OR(h - 1), NULL, AR(h - 1),
                                NULL, w);
  }
#undef YR
#undef UR
#undef VR
#undef AR
#undef OR
}
