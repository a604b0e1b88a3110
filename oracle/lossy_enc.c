/*
 * lossy_enc.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates the VP8 encoder's DSP drivers:
 *   importImage (non-dithered, direct RGBA path)  internal/lossy/encode.go:671-902
 *   computeAlphas + per-MB analysis              internal/lossy/encode_analysis.go:245-700
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define BPS OR_BPS

void or_import_rgba(const uint8_t* rgba, int w, int h, int stride, int has_alpha, uint8_t* Y, uint8_t* U,
                    uint8_t* V) {
  const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4;
  const int padw = mbw * 16, padh = mbh * 16;
  const int ys = padw, uvs = mbw * 8, uvw = (padw + 1) >> 1;
  /* Y plane, encode.go:757-793: rows clamp to h-1, columns replicate Y[w-1] */
  for (int y = 0; y < padh; y++) {
    int sy = y < h ? y : h - 1;
    const uint8_t* row = rgba + (size_t)sy * stride;
    uint8_t* dst = Y + (size_t)y * ys;
    for (int x = 0; x < w; x++) dst[x] = (uint8_t)or_rgb_to_y(row[4 * x], row[4 * x + 1], row[4 * x + 2]);
    for (int x = w; x < padw; x++) dst[x] = dst[w - 1];
  }
  /* U/V planes, encode.go:836-902: two padded planar rows -> AccumulateRGBA -> ConvertRGBA32ToUV */
  uint8_t* pr = (uint8_t*)malloc((size_t)padw * 2 * 4);
  uint8_t *pg = pr + 2 * padw, *pb = pg + 2 * padw, *pa = pb + 2 * padw;
  uint16_t* tmp = (uint16_t*)malloc((size_t)uvw * 4 * sizeof(uint16_t));
  for (int yp = 0; yp < padh / 2; yp++) {
    for (int r = 0; r < 2; r++) {
      int sy = yp * 2 + r;
      if (sy >= h) sy = h - 1;
      const uint8_t* row = rgba + (size_t)sy * stride;
      for (int x = 0; x < padw; x++) {
        int sx = x < w ? x : w - 1;
        pr[r * padw + x] = row[4 * sx];
        pg[r * padw + x] = row[4 * sx + 1];
        pb[r * padw + x] = row[4 * sx + 2];
        pa[r * padw + x] = has_alpha ? row[4 * sx + 3] : 0xff;
      }
    }
    or_accumulate_rgba(pr, pg, pb, pa, padw, tmp, padw);
    or_convert_rgba32_to_uv(tmp, U + (size_t)yp * uvs, V + (size_t)yp * uvs, uvw);
  }
  free(pr);
  free(tmp);
}

/* ---------------- analysis, encode_analysis.go ---------------- */
enum { MAX_COEFF_THRESH = 31, ALPHA_SCALE = 2 * 255, MAX_ALPHA = 255 }; /* :320-323 */

/* collectHistogramAlphaWith :559-600 over nblk blocks (pairs of src/pred offsets) */
static int histo_alpha(int* distribution) {
  int max_value = 0, last_nz = 1;
  for (int k = 0; k <= MAX_COEFF_THRESH; k++)
    if (distribution[k] > 0) {
      if (distribution[k] > max_value) max_value = distribution[k];
      last_nz = k;
    }
  int alpha = max_value > 1 ? ALPHA_SCALE * last_nz / max_value : 0;
  return alpha > MAX_ALPHA ? MAX_ALPHA : alpha;
}
static void histo_add(int* distribution, const int16_t* c) {
  for (int k = 0; k < 16; k++) {
    int v = c[k] < 0 ? -c[k] : c[k];
    v >>= 3;
    if (v > MAX_COEFF_THRESH) v = MAX_COEFF_THRESH;
    distribution[v]++;
  }
}

typedef struct { const uint8_t *y, *u, *v; int w, h, mbw, mbh, ys, uvs; } plane_t;

/* generateI16Prediction :455-552 (DC: rounded average, TM: 128 borders) */
static void i16_pred(const plane_t* P, int mbx, int mby, int mode, uint8_t* pred) {
  int x0 = mbx * 16, y0 = mby * 16;
  if (mode == 0) {
    int dc = 128, sum = 0, count = 0;
    if (mby > 0)
      for (int i = 0; i < 16; i++) {
        int sx = x0 + i < P->w ? x0 + i : P->w - 1;
        sum += P->y[(y0 - 1) * P->ys + sx];
        count++;
      }
    if (mbx > 0)
      for (int j = 0; j < 16; j++) {
        int sy = y0 + j < P->h ? y0 + j : P->h - 1;
        sum += P->y[sy * P->ys + x0 - 1];
        count++;
      }
    if (count > 0) dc = (sum + count / 2) / count;
    for (int j = 0; j < 16; j++)
      for (int i = 0; i < 16; i++) pred[j * BPS + i] = (uint8_t)dc;
  } else {
    int top[16], left[16], tl = 128;
    if (mby > 0) {
      for (int i = 0; i < 16; i++) {
        int sx = x0 + i < P->w ? x0 + i : P->w - 1;
        top[i] = P->y[(y0 - 1) * P->ys + sx];
      }
      tl = mbx > 0 ? P->y[(y0 - 1) * P->ys + x0 - 1] : top[0];
    } else {
      for (int i = 0; i < 16; i++) top[i] = 128;
    }
    for (int j = 0; j < 16; j++) {
      int sy = y0 + j < P->h ? y0 + j : P->h - 1;
      left[j] = mbx > 0 ? P->y[sy * P->ys + x0 - 1] : 128;
    }
    for (int j = 0; j < 16; j++)
      for (int i = 0; i < 16; i++) pred[j * BPS + i] = (uint8_t)or_clip8b(top[i] + left[j] - tl);
  }
}

/* computeMBAlphaDCTWith :407-452 */
static int mb_luma_alpha(const plane_t* P, int mbx, int mby) {
  uint8_t src[16 * BPS], pred[16 * BPS];
  int16_t c[16];
  int x0 = mbx * 16, y0 = mby * 16;
  for (int j = 0; j < 16; j++) {
    int sy = y0 + j < P->h ? y0 + j : P->h - 1;
    for (int i = 0; i < 16; i++) {
      int sx = x0 + i < P->w ? x0 + i : P->w - 1;
      src[j * BPS + i] = P->y[sy * P->ys + sx];
    }
  }
  int best = MAX_ALPHA + 1;
  for (int mode = 0; mode < 2; mode++) {
    if (mode == 1 && (mbx == 0 || mby == 0)) continue;
    i16_pred(P, mbx, mby, mode, pred);
    int dist[MAX_COEFF_THRESH + 1] = {0};
    for (int by = 0; by < 4; by++)
      for (int bx = 0; bx < 4; bx++) {
        int off = by * 4 * BPS + bx * 4;
        or_ftransform(src + off, pred + off, c);
        histo_add(dist, c);
      }
    int a = histo_alpha(dist);
    if (a < best) best = a;
  }
  return best > MAX_ALPHA ? MAX_ALPHA : best;
}

/* computeMBUVAlphaDCTWith :613-700 */
static int mb_uv_alpha(const plane_t* P, int mbx, int mby) {
  uint8_t su[8 * BPS], sv[8 * BPS], pu[8 * BPS], pv[8 * BPS];
  int16_t c[16];
  int ux0 = mbx * 8, uy0 = mby * 8, hmax = P->mbh * 8, wmax = P->mbw * 8;
  for (int j = 0; j < 8; j++) {
    int sy = uy0 + j < hmax ? uy0 + j : hmax - 1;
    for (int i = 0; i < 8; i++) {
      int sx = ux0 + i < wmax ? ux0 + i : wmax - 1;
      su[j * BPS + i] = P->u[sy * P->uvs + sx];
      sv[j * BPS + i] = P->v[sy * P->uvs + sx];
    }
  }
  int dcu = 128, dcv = 128, sumu = 0, sumv = 0, count = 0;
  if (mby > 0)
    for (int i = 0; i < 8; i++)
      if (ux0 + i < wmax) {
        sumu += P->u[(uy0 - 1) * P->uvs + ux0 + i];
        sumv += P->v[(uy0 - 1) * P->uvs + ux0 + i];
        count++;
      }
  if (mbx > 0)
    for (int j = 0; j < 8; j++)
      if (uy0 + j < hmax) {
        sumu += P->u[(uy0 + j) * P->uvs + ux0 - 1];
        sumv += P->v[(uy0 + j) * P->uvs + ux0 - 1];
        count++;
      }
  if (count > 0) {
    dcu = (sumu + count / 2) / count;
    dcv = (sumv + count / 2) / count;
  }
  for (int j = 0; j < 8; j++)
    for (int i = 0; i < 8; i++) {
      pu[j * BPS + i] = (uint8_t)dcu;
      pv[j * BPS + i] = (uint8_t)dcv;
    }
  int dist[MAX_COEFF_THRESH + 1] = {0};
  for (int by = 0; by < 2; by++)
    for (int bx = 0; bx < 2; bx++) {
      int off = by * 4 * BPS + bx * 4;
      or_ftransform(su + off, pu + off, c);
      histo_add(dist, c);
      or_ftransform(sv + off, pv + off, c);
      histo_add(dist, c);
    }
  return histo_alpha(dist);
}

int or_compute_alphas(const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h, int32_t* alphas,
                      int32_t* lum, int32_t* uva) { /* computeAlphas :245-307 */
  plane_t P;
  P.y = y; P.u = u; P.v = v; P.w = w; P.h = h;
  P.mbw = (w + 15) >> 4; P.mbh = (h + 15) >> 4;
  P.ys = 16 * P.mbw; P.uvs = 8 * P.mbw;
  int total = P.mbw * P.mbh;
  long long uv_sum = 0;
  for (int mby = 0; mby < P.mbh; mby++)
    for (int mbx = 0; mbx < P.mbw; mbx++) {
      int idx = mby * P.mbw + mbx;
      int la = mb_luma_alpha(&P, mbx, mby);
      int ua = mb_uv_alpha(&P, mbx, mby);
      int mixed = MAX_ALPHA - ((3 * la + ua + 2) >> 2);
      if (mixed < 0) mixed = 0;
      if (mixed > MAX_ALPHA) mixed = MAX_ALPHA;
      alphas[idx] = mixed;
      if (lum) lum[idx] = la;
      if (uva) uva[idx] = ua;
      uv_sum += ua;
    }
  return total > 0 ? (int)(uv_sum / total) : 0;
}

/* ---------------- dithered import (Preprocessing bit 1) ---------------- */
/* webp.Encode's dithering amplitude, encode.go (root):517-521, float32:
 * x = quality / 100; dithering = 1 + (0.5 - 1) * x^2 * x^2 */
float or_dithering_strength(float quality) {
  const float x = quality / 100.0f;
  const float x2 = x * x;
  return 1.0f + (0.5f - 1.0f) * x2 * x2;
}

/* importImage's dithered path (internal/lossy/encode.go:690-695, :793-809,
 * :903-940): one VP8Random stream per image (InitRandom), Y first over every
 * padded pixel in raster order (RGBToYRounding with RandomBits(16)), then per
 * row pair ConvertRGBA32ToUVDithered (RandomBits(18) for U, then V, per chroma
 * pixel; yuv.go:568-576). */
void or_import_rgba_dithered(const uint8_t* rgba, int w, int h, int stride, int has_alpha, float dithering, uint8_t* Y,
                             uint8_t* U, uint8_t* V) {
  const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4;
  const int padw = mbw * 16, padh = mbh * 16;
  const int ys = padw, uvs = mbw * 8, uvw = (padw + 1) >> 1;
  or_random rg;
  or_random_init(&rg, dithering);
  for (int y = 0; y < padh; y++) {
    const int sy = y < h ? y : h - 1;
    const uint8_t* row = rgba + (size_t)sy * stride;
    for (int x = 0; x < padw; x++) {
      const int sx = x < w ? x : w - 1;
      const int rnd = or_random_bits2(&rg, 16, rg.amp);
      Y[(size_t)y * ys + x] =
          (uint8_t)((16839 * row[4 * sx] + 33059 * row[4 * sx + 1] + 6420 * row[4 * sx + 2] + rnd + (16 << 16)) >> 16);
    }
  }
  uint8_t* pr = (uint8_t*)malloc((size_t)padw * 2 * 4);
  uint8_t *pg = pr + 2 * padw, *pb = pg + 2 * padw, *pa = pb + 2 * padw;
  uint16_t* tmp = (uint16_t*)malloc((size_t)uvw * 4 * sizeof(uint16_t));
  for (int yp = 0; yp < padh / 2; yp++) {
    for (int r = 0; r < 2; r++) {
      int sy = yp * 2 + r;
      if (sy >= h) sy = h - 1;
      const uint8_t* row = rgba + (size_t)sy * stride;
      for (int x = 0; x < padw; x++) {
        const int sx = x < w ? x : w - 1;
        pr[r * padw + x] = row[4 * sx];
        pg[r * padw + x] = row[4 * sx + 1];
        pb[r * padw + x] = row[4 * sx + 2];
        pa[r * padw + x] = has_alpha ? row[4 * sx + 3] : 0xff;
      }
    }
    or_accumulate_rgba(pr, pg, pb, pa, padw, tmp, padw);
    for (int i = 0; i < uvw; i++) {
      const int r = tmp[4 * i], g = tmp[4 * i + 1], b = tmp[4 * i + 2];
      U[(size_t)yp * uvs + i] = (uint8_t)or_rgb_to_u(r, g, b, or_random_bits2(&rg, 18, rg.amp));
      V[(size_t)yp * uvs + i] = (uint8_t)or_rgb_to_v(r, g, b, or_random_bits2(&rg, 18, rg.amp));
    }
  }
  free(pr);
  free(tmp);
}
