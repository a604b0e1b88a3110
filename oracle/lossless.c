/* lossless.c -- TEST INFRASTRUCTURE ONLY.  C restatement of the reference's
 * VP8L predictor transform:
 *
 *   forward  internal/lossless/encode_predictor.go:35-180 (subPixels, avg2,
 *            selectPred, clampAddSubFull/Half, predictPixel),
 *            :194-277 (estimateEntropy), :298-363 (copyImageWithPrediction),
 *            :378-455 (ResidualImage), :461-470 (SubtractGreen)
 *   entropy  internal/lossless/encode_histogram.go:355-377 (fastSLog2 + LUT)
 *   inverse  internal/lossless/decode_transform.go:202-451
 *            (predictorInverseTransform, addPixels, average2, selectPredictor,
 *            clampedAddSubtract*)
 *
 * The fastSLog2 LUT is i * math.Log2(i) from Go's standard library (third-
 * party to the reference; Go src/math/log.go + log2 in src/math/log10.go,
 * the FreeBSD e_log.c algorithm, which the amd64 assembly mirrors).  It is
 * restated here (go_log / go_log2) with -ffp-contract=off so the doubles are
 * the reference's.  Parity status of the LUT: unpinned by execution (no Go
 * toolchain in the image); cross-checked against libm log2 in tests.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define ARGB_BLACK 0xff000000u

/* ---------------- Go math.Log / math.Log2 (src/math/log.go) ---------------- */
static double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01;
  const double L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01;
  const double L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01;
  const double L7 = 1.479819860511658591e-01;
  if (isnan(x) || isinf(x)) return x;
  if (x < 0) return NAN;
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = frexp(x, &ki);
  if (f1 < 0.70710678118654752440 /* Go Sqrt2/2 */) {
    f1 *= 2;
    ki--;
  }
  const double f = f1 - 1;
  const double k = (double)ki;
  const double s = f / (2 + f);
  const double s2 = s * s;
  const double s4 = s2 * s2;
  const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const double R = t1 + t2;
  const double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

double or_go_log2(double x) {
  int e;
  const double frac = frexp(x, &e);
  if (frac == 0.5) return (double)(e - 1);
  
  return go_log(frac) * 0x1.71547652b82fep+0 /* Go const 1/Ln2, correctly rounded */ + (double)e;
}

/* fastSLog2LUT (encode_histogram.go:359-368) */
void or_vp8l_slog2_lut(double* out, int n) {
  out[0] = 0;
  for (int i = 1; i < n; i++) {
    const double fv = (double)i;
    out[i] = fv * or_go_log2(fv);
  }
}

static double* slog2_lut(void) {
  static double* lut = NULL;
  if (!lut) {
    lut = (double*)malloc(65536 * sizeof(double));
    or_vp8l_slog2_lut(lut, 65536);
  }
  return lut;
}

static double fast_slog2(uint32_t v) {
  if (v < 65536) return slog2_lut()[v];
  const double fv = (double)v;
  return fv * or_go_log2(fv);
}

/* ---------------- pixel arithmetic ---------------- */
static uint32_t sub_pixels(uint32_t a, uint32_t b) {
  const uint32_t ag = 0x00ff00ffu + (a & 0xff00ff00u) - (b & 0xff00ff00u);
  const uint32_t rb = 0xff00ff00u + (a & 0x00ff00ffu) - (b & 0x00ff00ffu);
  return (ag & 0xff00ff00u) | (rb & 0x00ff00ffu);
}
static uint32_t add_pixels(uint32_t a, uint32_t b) {
  const uint32_t ag = (a & 0xff00ff00u) + (b & 0xff00ff00u);
  const uint32_t rb = (a & 0x00ff00ffu) + (b & 0x00ff00ffu);
  return (ag & 0xff00ff00u) | (rb & 0x00ff00ffu);
}
static uint32_t avg2(uint32_t a, uint32_t b) { return (((a ^ b) & 0xfefefefeu) >> 1) + (a & b); }
static uint32_t select_pred(uint32_t l, uint32_t t, uint32_t tl) {
  int pa = 0;
  for (int s = 0; s < 32; s += 8) {
    const int a = abs((int)((t >> s) & 0xff) - (int)((tl >> s) & 0xff));
    const int b = abs((int)((l >> s) & 0xff) - (int)((tl >> s) & 0xff));
    pa += b - a;
  }
  return pa <= 0 ? t : l;
}
static int clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
static uint32_t clamp_add_sub_full(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r = 0;
  for (int s = 0; s < 32; s += 8)
    r |= (uint32_t)clamp255((int)((a >> s) & 0xff) + (int)((b >> s) & 0xff) - (int)((c >> s) & 0xff)) << s;
  return r;
}
static uint32_t clamp_add_sub_half(uint32_t avg, uint32_t c) {
  uint32_t r = 0;
  for (int s = 0; s < 32; s += 8) {
    const int va = (int)((avg >> s) & 0xff), vc = (int)((c >> s) & 0xff);
    r |= (uint32_t)clamp255(va + (va - vc) / 2) << s; /* Go '/' truncates toward zero, as C */
  }
  return r;
}

/* predictPixel (encode_predictor.go:148-180) */
uint32_t or_vp8l_predict(int mode, uint32_t l, uint32_t t, uint32_t tr, uint32_t tl) {
  switch (mode) {
    case 0: return ARGB_BLACK;
    case 1: return l;
    case 2: return t;
    case 3: return tr;
    case 4: return tl;
    case 5: return avg2(avg2(l, tr), t);
    case 6: return avg2(l, tl);
    case 7: return avg2(l, t);
    case 8: return avg2(tl, t);
    case 9: return avg2(t, tr);
    case 10: return avg2(avg2(l, tl), avg2(t, tr));
    case 11: return select_pred(l, t, tl);
    case 12: return clamp_add_sub_full(l, t, tl);
    case 13: return clamp_add_sub_half(avg2(l, t), tl);
    default: return ARGB_BLACK;
  }
}

static int subsample(int size, int bits) { return (size + (1 << bits) - 1) >> bits; }

/* estimateEntropy (encode_predictor.go:194-277) */
double or_vp8l_estimate_entropy(const uint32_t* argb, int width, int height, int tx, int ty, int bits, int mode) {
  const int ts = 1 << bits;
  const int x0 = tx * ts, y0 = ty * ts;
  const int x1 = x0 + ts > width ? width : x0 + ts;
  const int y1 = y0 + ts > height ? height : y0 + ts;
  const int ystep = (y1 - y0 > 16) ? 2 : 1;
  uint32_t hist[4 * 256];
  memset(hist, 0, sizeof(hist));
  uint32_t count = 0;
  for (int y = y0; y < y1; y += ystep) {
    const uint32_t* row = argb + (size_t)y * width;
    const uint32_t* prev = y > 0 ? row - width : NULL;
    for (int x = x0; x < x1; x++) {
      uint32_t l = 0, t = 0, tr = 0, tl = 0;
      if (x > 0) l = row[x - 1];
      if (y > 0) {
        t = prev[x];
        if (x > 0) tl = prev[x - 1];
        tr = (x < width - 1) ? prev[x + 1] : t;
      }
      const uint32_t res = sub_pixels(row[x], or_vp8l_predict(mode, l, t, tr, tl));
      hist[0 * 256 + ((res >> 24) & 0xff)]++;
      hist[1 * 256 + ((res >> 16) & 0xff)]++;
      hist[2 * 256 + ((res >> 8) & 0xff)]++;
      hist[3 * 256 + (res & 0xff)]++;
      count++;
    }
  }
  if (count == 0) return 0;
  double entropy = 0.0;
  for (int ch = 0; ch < 4; ch++) {
    double ce = fast_slog2(count);
    for (int i = 0; i < 256; i++)
      if (hist[ch * 256 + i] > 0) ce -= fast_slog2(hist[ch * 256 + i]);
    entropy += ce;
  }
  return entropy;
}

/* copyImageWithPrediction (encode_predictor.go:298-363) */
static void copy_image_with_prediction(const uint32_t* argb, int width, int height, int bits, const uint32_t* modes,
                                       uint32_t* out) {
  const int tpr = subsample(width, bits);
  for (int y = 0; y < height; y++) {
    const uint32_t* cur = argb + (size_t)y * width;
    const uint32_t* up = y > 0 ? cur - width : NULL; /* up[width] == cur[0] */
    for (int x = 0; x < width; x++) {
      const int mode = (int)((modes[(y >> bits) * tpr + (x >> bits)] >> 8) & 0xff);
      uint32_t pred;
      if (y == 0) pred = x == 0 ? ARGB_BLACK : cur[x - 1];
      else if (x == 0) pred = up[0];
      else {
        const uint32_t tr = (x < width - 1) ? up[x + 1] : up[width];
        pred = or_vp8l_predict(mode, cur[x - 1], up[x], tr, up[x - 1]);
      }
      out[(size_t)y * width + x] = sub_pixels(cur[x], pred);
    }
  }
}

/* ResidualImage (encode_predictor.go:378-455): modes[tiles] (mode << 8 |
 * 0xff000000) and residuals[w*h]. */
void or_vp8l_residual_image(const uint32_t* argb, int width, int height, int bits, int quality, uint32_t* modes,
                            uint32_t* residuals) {
  const int tx_n = subsample(width, bits), ty_n = subsample(height, bits);
  const int max_mode = quality < 25 ? 4 : (quality < 50 ? 8 : 14);
  for (int ty = 0; ty < ty_n; ty++)
    for (int tx = 0; tx < tx_n; tx++) {
      int best = 0;
      double best_cost = 1.7976931348623157e308;
      for (int m = 0; m < max_mode; m++) {
        const double c = or_vp8l_estimate_entropy(argb, width, height, tx, ty, bits, m);
        if (c < best_cost) {
          best_cost = c;
          best = m;
        }
      }
      modes[ty * tx_n + tx] = ((uint32_t)best << 8) | ARGB_BLACK;
    }
  copy_image_with_prediction(argb, width, height, bits, modes, residuals);
}

/* predictorInverseTransform (decode_transform.go:202-360), whole image. */
void or_vp8l_inverse_predictor(const uint32_t* modes, int bits, int width, int height, const uint32_t* in,
                               uint32_t* out) {
  const int tpr = subsample(width, bits);
  out[0] = add_pixels(in[0], ARGB_BLACK);
  for (int x = 1; x < width; x++) out[x] = add_pixels(in[x], out[x - 1]);
  for (int y = 1; y < height; y++) {
    const uint32_t* ir = in + (size_t)y * width;
    uint32_t* o = out + (size_t)y * width;
    const uint32_t* t = o - width;
    o[0] = add_pixels(ir[0], t[0]);
    for (int x = 1; x < width; x++) {
      const int mode = (int)((modes[(y >> bits) * tpr + (x >> bits)] >> 8) & 0xf);
      const uint32_t tr = (x < width - 1) ? t[x + 1] : o[0];
      uint32_t pred;
      switch (mode) {
        case 1: pred = o[x - 1]; break;
        case 2: pred = t[x]; break;
        case 3: pred = tr; break;
        case 4: pred = t[x - 1]; break;
        case 5: pred = avg2(avg2(o[x - 1], tr), t[x]); break;
        case 6: pred = avg2(o[x - 1], t[x - 1]); break;
        case 7: pred = avg2(o[x - 1], t[x]); break;
        case 8: pred = avg2(t[x - 1], t[x]); break;
        case 9: pred = avg2(t[x], tr); break;
        case 10: pred = avg2(avg2(o[x - 1], t[x - 1]), avg2(t[x], tr)); break;
        case 11: pred = select_pred(o[x - 1], t[x], t[x - 1]); break;
        case 12: pred = clamp_add_sub_full(o[x - 1], t[x], t[x - 1]); break;
        case 13: pred = clamp_add_sub_half(avg2(o[x - 1], t[x]), t[x - 1]); break;
        default: pred = ARGB_BLACK; break;
      }
      o[x] = add_pixels(ir[x], pred);
    }
  }
}

/* SubtractGreen (encode_predictor.go:461-470) / AddGreenToBlueAndRed (dsp/lossless_dsp.go:12) */
void or_vp8l_subtract_green(uint32_t* argb, size_t n) {
  for (size_t i = 0; i < n; i++) {
    const uint32_t p = argb[i], g = (p >> 8) & 0xff;
    argb[i] = (p & 0xff00ff00u) | ((((p >> 16) & 0xff) - g) & 0xff) << 16 | (((p & 0xff) - g) & 0xff);
  }
}
void or_vp8l_add_green(uint32_t* argb, size_t n) {
  for (size_t i = 0; i < n; i++) {
    const uint32_t p = argb[i], g = (p >> 8) & 0xff;
    argb[i] = (p & 0xff00ff00u) | ((((p >> 16) & 0xff) + g) & 0xff) << 16 | (((p & 0xff) + g) & 0xff);
  }
}

/* ---------------------------------------------------------------------------
 * Cross-colour transform.
 * ColorSpaceTransform   internal/lossless/encode_predictor.go:727-770
 * findBestMultipliers   :514-585,  findBestMultiplier :590-619,
 * multiplierCost        :645-718 (the threshold early exit returns a partial
 *                       sum above the running best, which never changes the
 *                       argmin, so the full sum is used here),
 * applyColorTransformPixel :497-507, encColorTransformDelta :478-480,
 * packMultipliers       :489-493 (no alpha byte).
 * ------------------------------------------------------------------------- */
static uint8_t cc_delta(int m, uint8_t c) { return (uint8_t)((m * (int)(int8_t)c) >> 5); }

static int64_t cc_cost(int m, const uint8_t* src, const uint8_t* dst, int n) {
  int64_t total = 0;
  for (int i = 0; i < n; i++) {
    uint8_t r = (uint8_t)(dst[i] - cc_delta(m, src[i]));
    if (r > 128) r = (uint8_t)(-r);
    total += r;
  }
  return total;
}

static int cc_best_multiplier(const uint8_t* src, const uint8_t* dst, int n) {
  int best_m = 0;
  int64_t best = INT64_MAX;
  for (int m = -128; m <= 127; m += 8) {
    const int64_t c = cc_cost(m, src, dst, n);
    if (c < best) {
      best = c;
      best_m = m;
    }
  }
  const int coarse = best_m;
  for (int m = coarse - 7; m <= coarse + 7; m++) {
    if (m < -128 || m > 127) continue;
    const int64_t c = cc_cost(m, src, dst, n);
    if (c < best) {
      best = c;
      best_m = m;
    }
  }
  return best_m;
}

void or_vp8l_color_space_transform(uint32_t* argb, int width, int height, int bits, uint32_t* data) {
  const int tw = subsample(width, bits), th = subsample(height, bits), ts = 1 << bits;
  uint8_t* buf = (uint8_t*)malloc((size_t)5 * ts * ts);
  uint8_t *g = buf, *r = buf + ts * ts, *b = buf + 2 * ts * ts, *ar = buf + 3 * ts * ts, *ab = buf + 4 * ts * ts;
  for (int ty = 0; ty < th; ty++)
    for (int tx = 0; tx < tw; tx++) {
      const int x0 = tx * ts, y0 = ty * ts;
      const int x1 = x0 + ts < width ? x0 + ts : width, y1 = y0 + ts < height ? y0 + ts : height;
      int n = 0;
      for (int y = y0; y < y1; y++)
        for (int x = x0; x < x1; x++) {
          const uint32_t px = argb[(size_t)y * width + x];
          g[n] = (uint8_t)(px >> 8);
          r[n] = (uint8_t)(px >> 16);
          b[n] = (uint8_t)px;
          n++;
        }
      int g2r = 0, g2b = 0, r2b = 0;
      if (n > 0) {
        g2r = cc_best_multiplier(g, r, n);
        for (int i = 0; i < n; i++) ar[i] = (uint8_t)(r[i] - cc_delta(g2r, g[i]));
        g2b = cc_best_multiplier(g, b, n);
        for (int i = 0; i < n; i++) ab[i] = (uint8_t)(b[i] - cc_delta(g2b, g[i]));
        r2b = cc_best_multiplier(ar, ab, n);
      }
      data[ty * tw + tx] = (uint32_t)(uint8_t)g2r | (uint32_t)(uint8_t)g2b << 8 | (uint32_t)(uint8_t)r2b << 16;
      for (int y = y0; y < y1; y++)
        for (int x = x0; x < x1; x++) {
          const uint32_t px = argb[(size_t)y * width + x];
          const uint8_t gr = (uint8_t)(px >> 8), rd = (uint8_t)(px >> 16), bl = (uint8_t)px;
          const int nr = (rd - (int)(int8_t)cc_delta(g2r, gr)) & 0xff;
          int nb = (bl - (int)(int8_t)cc_delta(g2b, gr)) & 0xff;
          nb = (nb - (int)(int8_t)cc_delta(r2b, rd)) & 0xff;
          argb[(size_t)y * width + x] = (px & 0xff00ff00u) | ((uint32_t)nr << 16) | (uint32_t)nb;
        }
    }
  free(buf);
}

/* colorSpaceInverseTransform (internal/lossless/decode_transform.go:454-520) */
void or_vp8l_color_space_inverse(const uint32_t* data, int bits, int width, int height, const uint32_t* src,
                                 uint32_t* dst) {
  const int tw = subsample(width, bits);
  for (int y = 0; y < height; y++)
    for (int x = 0; x < width; x++) {
      const uint32_t code = data[(y >> bits) * tw + (x >> bits)];
      const int g2r = (int8_t)code, g2b = (int8_t)(code >> 8), r2b = (int8_t)(code >> 16);
      const uint32_t px = src[(size_t)y * width + x];
      const int green = (int8_t)(px >> 8);
      int red = (px >> 16) & 0xff, blue = px & 0xff;
      red += (g2r * green) >> 5;
      red &= 0xff;
      blue += (g2b * green) >> 5;
      blue += (r2b * (int)(int8_t)red) >> 5;
      blue &= 0xff;
      dst[(size_t)y * width + x] = (px & 0xff00ff00u) | ((uint32_t)red << 16) | (uint32_t)blue;
    }
}

/* colorIndexInverseTransform (internal/lossless/decode_transform.go:560-612):
 * xbits = the transform's Bits (0..3: 8 >> xbits bits per index); src rows
 * hold subsample(width, xbits) packed words; out-of-palette indices leave
 * dst untouched. */
void or_vp8l_color_index_inverse(const uint32_t* palette, int palette_size, int xbits, int width, int height,
                                 const uint32_t* src, uint32_t* dst) {
  const int bpp = 8 >> xbits, ppb = 1 << xbits, packed_w = subsample(width, xbits);
  const uint32_t mask = (1u << bpp) - 1;
  for (int y = 0; y < height; y++) {
    const uint32_t* s = src + (size_t)y * packed_w;
    uint32_t packed = 0;
    for (int x = 0; x < width; x++) {
      if ((x & (ppb - 1)) == 0) packed = (s[x >> xbits] >> 8) & 0xff;
      const uint32_t idx = bpp < 8 ? (packed & mask) : packed;
      if ((int)idx < palette_size) dst[(size_t)y * width + x] = palette[idx];
      if (bpp < 8) packed >>= bpp;
    }
  }
}
