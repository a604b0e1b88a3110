/* oracle/alpha.c -- TEST INFRASTRUCTURE ONLY (see oracle/oracle.h).
 * C restatement of the reference's alpha-plane filters and alpha
 * processing:
 *   internal/lossy/alpha.go      filters :387-454, unfilters :128-203,
 *                                estimateBestFilter :321-385, getNumColors :302-317
 *   internal/dsp/alpha_proc.go   premultiply :13-135, dispatch / extract :140-227
 * Parity: restatement of the Go source (libwebp's filters_utils.c /
 * alpha_processing.c semantics, which the Go code mirrors); unfilter(filter(x))
 * == x is checked for every filter. */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

static uint8_t clip255(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

/* alphaFilterHorizontal / Vertical / Gradient (:387-454); filter 0 copies */
void or_alpha_filter(int filter, const uint8_t* in, int width, int height, uint8_t* out) {
  if (filter == 0) {
    memcpy(out, in, (size_t)width * height);
    return;
  }
  out[0] = in[0];
  for (int i = 1; i < width; i++) out[i] = (uint8_t)(in[i] - in[i - 1]);
  for (int y = 1; y < height; y++) {
    const uint8_t* src = in + (size_t)y * width;
    const uint8_t* prev = src - width;
    uint8_t* dst = out + (size_t)y * width;
    if (filter == 2) {
      for (int x = 0; x < width; x++) dst[x] = (uint8_t)(src[x] - prev[x]);
      continue;
    }
    dst[0] = (uint8_t)(src[0] - prev[0]);
    for (int x = 1; x < width; x++) {
      const int pred = filter == 1 ? src[x - 1] : clip255(src[x - 1] + prev[x] - prev[x - 1]);
      dst[x] = (uint8_t)(src[x] - pred);
    }
  }
}

/* alphaUnfilterHorizontal / Vertical / Gradient (:128-203), in place */
void or_alpha_unfilter(int filter, uint8_t* data, int width, int height) {
  if (filter == 0) return;
  if (filter == 1) {
    for (int y = 0; y < height; y++) {
      uint8_t* row = data + (size_t)y * width;
      if (y > 0) row[0] = (uint8_t)(row[0] + row[-width]);
      for (int x = 1; x < width; x++) row[x] = (uint8_t)(row[x] + row[x - 1]);
    }
    return;
  }
  for (int x = 1; x < width; x++) data[x] = (uint8_t)(data[x] + data[x - 1]);
  for (int y = 1; y < height; y++) {
    uint8_t* curr = data + (size_t)y * width;
    const uint8_t* prev = curr - width;
    if (filter == 2) {
      for (int x = 0; x < width; x++) curr[x] = (uint8_t)(curr[x] + prev[x]);
      continue;
    }
    uint8_t top = prev[0], top_left = top, left = top;
    for (int x = 0; x < width; x++) {
      top = prev[x];
      left = (uint8_t)(curr[x] + clip255(left + top - top_left));
      top_left = top;
      curr[x] = left;
    }
  }
}

/* estimateBestFilter (:321-385): 0 none, 1 horizontal, 2 vertical, 3 gradient */
int or_alpha_estimate_best_filter(const uint8_t* data, int width, int height) {
  int bins[4][16];
  memset(bins, 0, sizeof(bins));
  for (int j = 2; j < height - 1; j += 2) {
    const uint8_t* p = data + (size_t)j * width;
    int mean = p[0];
    for (int i = 2; i < width - 1; i += 2) {
      const int cur = p[i];
      const int d0 = abs(cur - mean) >> 4, d1 = abs(cur - p[i - 1]) >> 4, d2 = abs(cur - p[i - width]) >> 4;
      const int d3 = abs(cur - clip255(p[i - 1] + p[i - width] - p[i - width - 1])) >> 4;
      if (d0 < 16) bins[0][d0] = 1;
      if (d1 < 16) bins[1][d1] = 1;
      if (d2 < 16) bins[2][d2] = 1;
      if (d3 < 16) bins[3][d3] = 1;
      mean = (3 * mean + cur + 2) >> 2;
    }
  }
  int best = 0, best_score = 0x7fffffff;
  for (int f = 0; f < 4; f++) {
    int score = 0;
    for (int i = 0; i < 16; i++)
      if (bins[f][i]) score += i;
    if (score < best_score) {
      best_score = score;
      best = f;
    }
  }
  return best;
}

/* getNumColors (:302-317) */
int or_alpha_num_colors(const uint8_t* data, int width, int height) {
  int seen[256] = {0}, n = 0;
  for (size_t i = 0; i < (size_t)width * height; i++) seen[data[i]] = 1;
  for (int i = 0; i < 256; i++) n += seen[i];
  return n;
}

/* alphaMult / alphaGetScale (alpha_proc.go:13-26) */
static uint32_t a_mult(uint8_t x, uint32_t mult) { return ((uint32_t)x * mult + (1u << 23)) >> 24; }
static uint32_t a_scale(uint32_t a, int inverse) { return inverse ? (255u << 24) / a : a * ((1u << 24) / 255); }

/* ApplyAlphaMultiply (:74-104): 4-byte pixels, alpha at offset 0 (alpha_first) or 3 */
void or_apply_alpha_multiply(uint8_t* rgba, int alpha_first, int width, int height, int stride, int inverse) {
  const int rgb_off = alpha_first ? 1 : 0, a_off = alpha_first ? 0 : 3;
  for (int y = 0; y < height; y++) {
    uint8_t* row = rgba + (size_t)y * stride;
    for (int i = 0; i < width; i++) {
      uint8_t* p = row + 4 * i;
      const uint32_t a = p[a_off];
      if (a == 255) continue;
      if (a == 0) {
        p[rgb_off] = p[rgb_off + 1] = p[rgb_off + 2] = 0;
        continue;
      }
      const uint32_t s = a_scale(a, inverse);
      for (int c = 0; c < 3; c++) p[rgb_off + c] = (uint8_t)a_mult(p[rgb_off + c], s);
    }
  }
}

/* MultARGBRow (:28-46) over n pixels */
void or_mult_argb(uint32_t* argb, size_t n, int inverse) {
  for (size_t i = 0; i < n; i++) {
    const uint32_t p = argb[i];
    if (p >= 0xff000000u) continue;
    if (p <= 0x00ffffffu) {
      argb[i] = 0;
      continue;
    }
    const uint32_t s = a_scale((p >> 24) & 0xff, inverse);
    argb[i] = (p & 0xff000000u) | a_mult((uint8_t)p, s) | a_mult((uint8_t)(p >> 8), s) << 8 |
              a_mult((uint8_t)(p >> 16), s) << 16;
  }
}

/* ApplyAlphaMultiply4444 (:106-135) */
void or_apply_alpha_multiply_4444(uint8_t* data, int width, int height, int stride) {
  for (int y = 0; y < height; y++) {
    uint8_t* row = data + (size_t)y * stride;
    for (int x = 0; x < width; x++) {
      uint8_t* p = row + 2 * x;
      const uint8_t rg = p[0], ba = p[1], a = ba & 0x0f;
      if (a == 0x0f) continue;
      if (a == 0) {
        p[0] = p[1] = 0;
        continue;
      }
      /* Go: byte arithmetic, (r * a + 7) / 15 in uint8 -- r * a + 7 <= 217, no wrap */
      const uint8_t r = (uint8_t)(((rg >> 4) & 0x0f) * a + 7) / 15, g = (uint8_t)((rg & 0x0f) * a + 7) / 15;
      const uint8_t b = (uint8_t)(((ba >> 4) & 0x0f) * a + 7) / 15;
      p[0] = (uint8_t)(r << 4 | g);
      p[1] = (uint8_t)(b << 4 | a);
    }
  }
}

/* DispatchAlpha (:140-155): returns whether any alpha != 0xff */
int or_dispatch_alpha(const uint8_t* alpha, int alpha_stride, int width, int height, uint8_t* dst, int dst_stride,
                      int alpha_off) {
  uint32_t mask = 0xff;
  for (int y = 0; y < height; y++)
    for (int x = 0; x < width; x++) {
      const uint32_t v = alpha[(size_t)y * alpha_stride + x];
      dst[(size_t)y * dst_stride + 4 * x + alpha_off] = (uint8_t)v;
      mask &= v;
    }
  return mask != 0xff;
}

/* ExtractAlpha (:158-176): returns 1 when every alpha is 0xff */
int or_extract_alpha(const uint8_t* src, int src_stride, int width, int height, uint8_t* alpha, int alpha_stride,
                     int alpha_off) {
  uint8_t mask = 0xff;
  for (int y = 0; y < height; y++)
    for (int x = 0; x < width; x++) {
      const uint8_t a = src[(size_t)y * src_stride + 4 * x + alpha_off];
      alpha[(size_t)y * alpha_stride + x] = a;
      mask &= a;
    }
  return mask == 0xff;
}

/* HasAlpha8b / HasAlpha32b (:178-197): any byte at i * step (step 1 or 4) != 0xff */
int or_has_alpha(const uint8_t* src, size_t length, int step) {
  for (size_t i = 0; i < length; i++)
    if (src[i * step] != 0xff) return 1;
  return 0;
}

/* AlphaReplace (:199-206) */
void or_alpha_replace(uint32_t* argb, size_t length, uint32_t color) {
  for (size_t i = 0; i < length; i++)
    if ((argb[i] >> 24) == 0) argb[i] = color;
}

/* DispatchAlphaToGreen (:209-219) */
void or_dispatch_alpha_to_green(const uint8_t* alpha, int alpha_stride, int width, int height, uint32_t* dst,
                                int dst_stride) {
  for (int y = 0; y < height; y++)
    for (int x = 0; x < width; x++) dst[(size_t)y * dst_stride + x] = (uint32_t)alpha[(size_t)y * alpha_stride + x] << 8;
}

/* ExtractGreen (:221-226) */
void or_extract_green(const uint32_t* argb, uint8_t* alpha, size_t size) {
  for (size_t i = 0; i < size; i++) alpha[i] = (uint8_t)(argb[i] >> 8);
}

/* PackRGB (:229-238) */
void or_pack_rgb(const uint8_t* r, const uint8_t* g, const uint8_t* b, size_t length, int step, uint32_t* out) {
  for (size_t i = 0; i < length; i++) {
    const size_t o = i * step;
    out[i] = 0xff000000u | (uint32_t)r[o] << 16 | (uint32_t)g[o] << 8 | b[o];
  }
}
