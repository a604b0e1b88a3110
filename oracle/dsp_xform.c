/*
 * dsp_xform.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates internal/dsp/transforms.go and cliptables.go:Clip8b.
 */
#include "oracle.h"

/* Clip8b, internal/dsp/cliptables.go:37-44 */
int or_clip8b(int64_t v) { return v < 0 ? 0 : (v > 255 ? 255 : (int)v); }

/* mul1/mul2 (transforms.go:20-27): Go does these in 64-bit int. */
static inline int64_t mul1(int64_t a) { return ((a * 20091) >> 16) + a; }
static inline int64_t mul2(int64_t a) { return (a * 35468) >> 16; }

/* Shared 4x4 inverse DCT core: vertical pass then horizontal pass (+4 rounding),
 * returns the 16 residuals (>>3 applied). transforms.go:37-136 and :265-366
 * compute exactly this; they differ only in where the residual is added. */
static void idct4x4(const int16_t* in, int64_t res[16]) {
  int64_t tmp[16];
  for (int c = 0; c < 4; c++) {             /* vertical pass, transforms.go:45-92 */
    int64_t a = (int64_t)in[c] + in[8 + c];
    int64_t b = (int64_t)in[c] - in[8 + c];
    int64_t cc = mul2(in[4 + c]) - mul1(in[12 + c]);
    int64_t d = mul1(in[4 + c]) + mul2(in[12 + c]);
    tmp[0 + c] = a + d;
    tmp[4 + c] = b + cc;
    tmp[8 + c] = b - cc;
    tmp[12 + c] = a - d;
  }
  for (int r = 0; r < 4; r++) {             /* horizontal pass, transforms.go:95-135 */
    const int64_t* t = tmp + 4 * r;
    int64_t dc = t[0] + 4;
    int64_t a = dc + t[2];
    int64_t b = dc - t[2];
    int64_t cc = mul2(t[1]) - mul1(t[3]);
    int64_t d = mul1(t[1]) + mul2(t[3]);
    res[4 * r + 0] = (a + d) >> 3;
    res[4 * r + 1] = (b + cc) >> 3;
    res[4 * r + 2] = (b - cc) >> 3;
    res[4 * r + 3] = (a - d) >> 3;
  }
}

/* transformOne: dst += residual, clipped (store() transforms.go:30-33). */
static void transform_one(const int16_t* in, uint8_t* dst) {
  int64_t res[16];
  idct4x4(in, res);
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++)
      dst[c + r * OR_BPS] = (uint8_t)or_clip8b(dst[c + r * OR_BPS] + res[4 * r + c]);
}

void or_transform(const int16_t* in, uint8_t* dst, int do_two) { /* transformTwo :139 */
  transform_one(in, dst);
  if (do_two) transform_one(in + 16, dst + 4);
}

/* store(dst, off, x) adds x>>3 (transforms.go:30-33) */
static inline void store(uint8_t* dst, int off, int64_t x) {
  dst[off] = (uint8_t)or_clip8b(dst[off] + (x >> 3));
}

void or_transform_dc(const int16_t* in, uint8_t* dst) { /* :148-166 */
  int64_t dc = (int64_t)in[0] + 4;
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) store(dst, c + r * OR_BPS, dc);
}

void or_transform_ac3(const int16_t* in, uint8_t* dst) { /* :170-193 */
  int64_t a = (int64_t)in[0] + 4;
  int64_t c4 = mul2(in[4]), d4 = mul1(in[4]);
  int64_t c1 = mul2(in[1]), d1 = mul1(in[1]);
  const int64_t row[4] = {a + d4, a + c4, a - c4, a - d4};
  const int64_t col[4] = {d1, c1, -c1, -d1};
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) store(dst, c + r * OR_BPS, row[r] + col[c]);
}

void or_transform_uv(const int16_t* in, uint8_t* dst) { /* :197-200 */
  or_transform(in, dst, 1);
  or_transform(in + 32, dst + 4 * OR_BPS, 1);
}

void or_transform_dcuv(const int16_t* in, uint8_t* dst) { /* :203-216 */
  if (in[0]) or_transform_dc(in, dst);
  if (in[16]) or_transform_dc(in + 16, dst + 4);
  if (in[32]) or_transform_dc(in + 32, dst + 4 * OR_BPS);
  if (in[48]) or_transform_dc(in + 48, dst + 4 * OR_BPS + 4);
}

void or_transform_wht(const int16_t* in, int16_t* out) { /* :223-252 */
  int64_t tmp[16];
  for (int i = 0; i < 4; i++) {
    int64_t a0 = (int64_t)in[i] + in[12 + i];
    int64_t a1 = (int64_t)in[4 + i] + in[8 + i];
    int64_t a2 = (int64_t)in[4 + i] - in[8 + i];
    int64_t a3 = (int64_t)in[i] - in[12 + i];
    tmp[i] = a0 + a1;
    tmp[8 + i] = a0 - a1;
    tmp[4 + i] = a3 + a2;
    tmp[12 + i] = a3 - a2;
  }
  for (int i = 0; i < 4; i++) {
    int64_t dc = tmp[4 * i] + 3;
    int64_t a0 = dc + tmp[4 * i + 3];
    int64_t a1 = tmp[4 * i + 1] + tmp[4 * i + 2];
    int64_t a2 = tmp[4 * i + 1] - tmp[4 * i + 2];
    int64_t a3 = dc - tmp[4 * i + 3];
    int16_t* o = out + 64 * i;               /* int16() wraps, as in Go */
    o[0] = (int16_t)((a0 + a1) >> 3);
    o[16] = (int16_t)((a3 + a2) >> 3);
    o[32] = (int16_t)((a0 - a1) >> 3);
    o[48] = (int16_t)((a3 - a2) >> 3);
  }
}

static void itransform_one(const uint8_t* ref, const int16_t* in, uint8_t* dst) { /* :265-366 */
  int64_t res[16];
  idct4x4(in, res);
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++)
      dst[c + r * OR_BPS] = (uint8_t)or_clip8b(ref[c + r * OR_BPS] + res[4 * r + c]);
}

void or_itransform(const uint8_t* ref, const int16_t* in, uint8_t* dst, int do_two) { /* :256 */
  itransform_one(ref, in, dst);
  if (do_two) itransform_one(ref + 4, in + 16, dst + 4);
}

void or_ftransform(const uint8_t* src, const uint8_t* ref, int16_t* out) { /* :371-484 */
  int tmp[16];
  for (int r = 0; r < 4; r++) {             /* horizontal pass */
    const uint8_t* s = src + r * OR_BPS;
    const uint8_t* p = ref + r * OR_BPS;
    int d0 = s[0] - p[0], d1 = s[1] - p[1], d2 = s[2] - p[2], d3 = s[3] - p[3];
    int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
    tmp[4 * r + 0] = (a0 + a1) * 8;
    tmp[4 * r + 1] = (a2 * 2217 + a3 * 5352 + 1812) >> 9;
    tmp[4 * r + 2] = (a0 - a1) * 8;
    tmp[4 * r + 3] = (a3 * 2217 - a2 * 5352 + 937) >> 9;
  }
  for (int c = 0; c < 4; c++) {             /* vertical pass */
    int a0 = tmp[c] + tmp[12 + c];
    int a1 = tmp[4 + c] + tmp[8 + c];
    int a2 = tmp[4 + c] - tmp[8 + c];
    int a3 = tmp[c] - tmp[12 + c];
    out[c] = (int16_t)((a0 + a1 + 7) >> 4);
    out[4 + c] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0));
    out[8 + c] = (int16_t)((a0 - a1 + 7) >> 4);
    out[12 + c] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
  }
}

void or_ftransform2(const uint8_t* src, const uint8_t* ref, int16_t* out) { /* :487-490 */
  or_ftransform(src, ref, out);
  or_ftransform(src + 4, ref + 4, out + 16);
}

void or_ftransform_wht(const int16_t* in, int16_t* out) { /* :500-531, flat stride-4 input */
  int tmp[16];
  for (int i = 0; i < 4; i++) {
    const int16_t* r = in + 4 * i;
    int a0 = r[0] + r[2], a1 = r[1] + r[3], a2 = r[1] - r[3], a3 = r[0] - r[2];
    tmp[4 * i + 0] = a0 + a1;
    tmp[4 * i + 1] = a3 + a2;
    tmp[4 * i + 2] = a3 - a2;
    tmp[4 * i + 3] = a0 - a1;
  }
  for (int i = 0; i < 4; i++) {
    int a0 = tmp[i] + tmp[8 + i], a1 = tmp[4 + i] + tmp[12 + i];
    int a2 = tmp[4 + i] - tmp[12 + i], a3 = tmp[i] - tmp[8 + i];
    out[i] = (int16_t)((a0 + a1) >> 1);
    out[4 + i] = (int16_t)((a3 + a2) >> 1);
    out[8 + i] = (int16_t)((a3 - a2) >> 1);
    out[12 + i] = (int16_t)((a0 - a1) >> 1);
  }
}
