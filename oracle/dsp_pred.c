/*
 * dsp_pred.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates internal/dsp/predict_lossy.go (VP8 intra predictors).
 * Convention (predict_lossy.go:3-13): buf+off is the block origin, top row at
 * off-BPS, left column at off-1, top-left at off-BPS-1.
 */
#include "oracle.h"

#define BPS OR_BPS
static inline uint8_t avg3(int a, int b, int c) { return (uint8_t)((a + 2 * b + c + 2) >> 2); } /* :16 */
static inline uint8_t avg2(int a, int b) { return (uint8_t)((a + b + 1) >> 1); }                 /* :21 */

static void fill(uint8_t* d, int size, int v) {
  for (int j = 0; j < size; j++)
    for (int i = 0; i < size; i++) d[i + j * BPS] = (uint8_t)v;
}

/* Shared body of the 16x16 and 8x8 predictors (:27-181); size = 16 or 8,
 * shift = log2(2*size) for DC, DC-NoTop/NoLeft use shift-1. */
static void pred_square(int mode, uint8_t* d, int size, int shift) {
  const uint8_t* top = d - BPS;
  int sum = 0;
  switch (mode) {
    case 0: /* DC: dc16 :27 / dc8uv :106 */
      for (int i = 0; i < size; i++) sum += top[i] + d[-1 + i * BPS];
      fill(d, size, (sum + size) >> shift);
      break;
    case 1: { /* TM: tm16 :40 / tm8uv :119 */
      int tl = d[-1 - BPS];
      for (int j = 0; j < size; j++) {
        int base = d[-1 + j * BPS] - tl;
        for (int i = 0; i < size; i++) d[i + j * BPS] = (uint8_t)or_clip8b(base + top[i]);
      }
      break;
    }
    case 2: /* VE */
      for (int j = 0; j < size; j++)
        for (int i = 0; i < size; i++) d[i + j * BPS] = top[i];
      break;
    case 3: /* HE */
      for (int j = 0; j < size; j++)
        for (int i = 0; i < size; i++) d[i + j * BPS] = d[-1 + j * BPS];
      break;
    case 4: /* DC NoTop: left only */
      for (int i = 0; i < size; i++) sum += d[-1 + i * BPS];
      fill(d, size, (sum + (size >> 1)) >> (shift - 1));
      break;
    case 5: /* DC NoLeft: top only */
      for (int i = 0; i < size; i++) sum += top[i];
      fill(d, size, (sum + (size >> 1)) >> (shift - 1));
      break;
    default: /* 6: DC NoTopLeft */
      fill(d, size, 128);
      break;
  }
}

void or_pred_luma16(int mode, uint8_t* buf, int off) { pred_square(mode, buf + off, 16, 5); }
void or_pred_chroma8(int mode, uint8_t* buf, int off) { pred_square(mode, buf + off, 8, 4); }

/* 4x4 predictors :185-424.  P(x,y) addresses the block; T[i]=top row (i=-1 is
 * top-left, i up to 7 includes the 4 top-right pixels), L[j]=left column. */
void or_pred_luma4(int mode, uint8_t* buf, int off) {
  uint8_t* d = buf + off;
#define P(x, y) d[(x) + (y) * BPS]
  const int X = d[-1 - BPS];
  const int A = d[0 - BPS], B = d[1 - BPS], C = d[2 - BPS], D = d[3 - BPS];
  const int E = d[4 - BPS], F = d[5 - BPS], G = d[6 - BPS], H = d[7 - BPS];
  const int I = d[-1], J = d[-1 + BPS], K = d[-1 + 2 * BPS], L = d[-1 + 3 * BPS];
  switch (mode) {
    case 0: { /* dc4 :185 */
      int v = (A + B + C + D + I + J + K + L + 4) >> 3;
      fill(d, 4, v);
      break;
    }
    case 1: /* tm4 :197 */
      for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) P(x, y) = (uint8_t)or_clip8b(d[-1 + y * BPS] + d[x - BPS] - X);
      break;
    case 2: { /* ve4 :206, smoothed with avg3 */
      uint8_t v[4] = {avg3(X, A, B), avg3(A, B, C), avg3(B, C, D), avg3(C, D, E)};
      for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) P(x, y) = v[x];
      break;
    }
    case 3: { /* he4 :225 */
      uint8_t v[4] = {avg3(X, I, J), avg3(I, J, K), avg3(J, K, L), avg3(K, L, L)};
      for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) P(x, y) = v[y];
      break;
    }
    case 4: /* rd4 :244: down-right diagonals, index x-y */
      P(0, 3) = avg3(L, K, J);
      P(0, 2) = P(1, 3) = avg3(K, J, I);
      P(0, 1) = P(1, 2) = P(2, 3) = avg3(J, I, X);
      P(0, 0) = P(1, 1) = P(2, 2) = P(3, 3) = avg3(I, X, A);
      P(1, 0) = P(2, 1) = P(3, 2) = avg3(X, A, B);
      P(2, 0) = P(3, 1) = avg3(A, B, C);
      P(3, 0) = avg3(B, C, D);
      break;
    case 5: /* vr4 :272 */
      P(0, 0) = P(1, 2) = avg2(X, A);
      P(1, 0) = P(2, 2) = avg2(A, B);
      P(2, 0) = P(3, 2) = avg2(B, C);
      P(3, 0) = avg2(C, D);
      P(0, 1) = P(1, 3) = avg3(I, X, A);
      P(1, 1) = P(2, 3) = avg3(X, A, B);
      P(2, 1) = P(3, 3) = avg3(A, B, C);
      P(3, 1) = avg3(B, C, D);
      P(0, 2) = avg3(J, I, X);
      P(0, 3) = avg3(K, J, I);
      break;
    case 6: /* ld4 :305: down-left, index x+y */
      P(0, 0) = avg3(A, B, C);
      P(1, 0) = P(0, 1) = avg3(B, C, D);
      P(2, 0) = P(1, 1) = P(0, 2) = avg3(C, D, E);
      P(3, 0) = P(2, 1) = P(1, 2) = P(0, 3) = avg3(D, E, F);
      P(3, 1) = P(2, 2) = P(1, 3) = avg3(E, F, G);
      P(3, 2) = P(2, 3) = avg3(F, G, H);
      P(3, 3) = avg3(G, H, H);
      break;
    case 7: /* vl4 :333 */
      P(0, 0) = avg2(A, B);
      P(1, 0) = P(0, 2) = avg2(B, C);
      P(2, 0) = P(1, 2) = avg2(C, D);
      P(3, 0) = P(2, 2) = avg2(D, E);
      P(0, 1) = avg3(A, B, C);
      P(1, 1) = P(0, 3) = avg3(B, C, D);
      P(2, 1) = P(1, 3) = avg3(C, D, E);
      P(3, 1) = P(2, 3) = avg3(D, E, F);
      P(3, 2) = avg3(E, F, G);
      P(3, 3) = avg3(F, G, H);
      break;
    case 8: /* hd4 :363 */
      P(0, 0) = P(2, 1) = avg2(X, I);
      P(1, 0) = P(3, 1) = avg3(I, X, A);
      P(2, 0) = avg3(X, A, B);
      P(3, 0) = avg3(A, B, C);
      P(0, 1) = P(2, 2) = avg2(I, J);
      P(1, 1) = P(3, 2) = avg3(X, I, J);
      P(0, 2) = P(2, 3) = avg2(J, K);
      P(1, 2) = P(3, 3) = avg3(I, J, K);
      P(0, 3) = avg2(K, L);
      P(1, 3) = avg3(J, K, L);
      break;
    default: /* 9: hu4 :394 */
      P(0, 0) = avg2(I, J);
      P(1, 0) = avg3(I, J, K);
      P(2, 0) = P(0, 1) = avg2(J, K);
      P(3, 0) = P(1, 1) = avg3(J, K, L);
      P(2, 1) = P(0, 2) = avg2(K, L);
      P(3, 1) = P(1, 2) = avg3(K, L, L);
      P(2, 2) = P(3, 2) = P(0, 3) = P(1, 3) = P(2, 3) = P(3, 3) = (uint8_t)L;
      break;
  }
#undef P
}
