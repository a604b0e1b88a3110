// wg_dsp.h -- device-side building blocks of the internal/dsp hot path for
// gfx950.  Lane-level functions shared by the frame kernels and by the
// batched block-level parity entry points, so the parity tests exercise the
// exact code the frame kernels run.
//
// Arithmetic notes (bit-exactness vs the Go reference):
//  * mul1/mul2 (transforms.go:20-27) are computed with v_mul_hi_i32 on a
//    pre-shifted constant: (a*c)>>16 == a + mulhi(a, (c-65536)<<16) for
//    c = 35468, and a + mulhi(a, 20091<<16) for MUL1.  Exact for every int32 a,
//    which covers Go's 64-bit `int` products on full-range int16 inputs.
//  * The clip tables (cliptables.go) are exact clamps on their domains.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define WG_BPS 32

namespace wg {

__device__ __forceinline__ int clip8(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int sclip1(int v) { return min(max(v, -128), 127); }
__device__ __forceinline__ int sclip2(int v) { return min(max(v, -16), 15); }
__device__ __forceinline__ int mul1(int a) { return a + __mulhi(a, 20091 << 16); }
__device__ __forceinline__ int mul2(int a) { return a + __mulhi(a, (35468 - 65536) * 65536); }
// The same on the full-rate 24-bit multiplier (v_mul_hi_i32 and v_mul_lo_u32
// are quarter rate).  For |a| <= 2^15 (an int16 coefficient: callers
// truncate to int16 first, as dequant() does) a * 35468 fits int32 (2^15 *
// 35468 < 2^31; 2^16 * 35468 does not): one v_mul_i32_i24 and a shift.  For |a| < 2^23 (the inverse DCT's
// second pass: at most ~2^17.4 from int16 inputs) the 48-bit product is
// mul_i24 (low 32 bits) + mulhi_i24 (bits 32..47) and bits 16..47 come out
// of one v_alignbit.  Both equal mul1 / mul2 (Go's 64-bit products) on those
// ranges.
// (as inline asm: hipcc turns __mul24 / __umul24 back into v_mul_lo_u32
// wherever it loses the operands' range)
__device__ __forceinline__ int mul_i24(int a, int c) {
  int r;
  asm("v_mul_i32_i24 %0, %1, %2" : "=v"(r) : "v"(c), "v"(a));
  return r;
}
__device__ __forceinline__ int mulhi_i24(int a, int c) {
  int r;
  asm("v_mul_hi_i32_i24 %0, %1, %2" : "=v"(r) : "v"(c), "v"(a));
  return r;
}
__device__ __forceinline__ int mul1_16(int a) { return a + (mul_i24(a, 20091) >> 16); }
__device__ __forceinline__ int mul2_16(int a) { return mul_i24(a, 35468) >> 16; }
__device__ __forceinline__ int mul_sh16_24(int a, int c) {
  return (int)__builtin_amdgcn_alignbit((uint32_t)mulhi_i24(a, c), (uint32_t)mul_i24(a, c), 16);
}
__device__ __forceinline__ int mul1_24(int a) { return a + mul_sh16_24(a, 20091); }
__device__ __forceinline__ int mul2_24(int a) { return mul_sh16_24(a, 35468); }
__device__ __forceinline__ int avg3(int a, int b, int c) { return (a + 2 * b + c + 2) >> 2; }
__device__ __forceinline__ int avg2(int a, int b) { return (a + b + 1) >> 1; }
__device__ __forceinline__ uint32_t pack4(int a, int b, int c, int d) {
  return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24);
}
__device__ __forceinline__ int byte_of(uint32_t w, int i) { return (w >> (8 * i)) & 0xff; }

// ------------------------------------------------------------------------
// Inverse 4x4 DCT, one output row per lane (transforms.go:37-136 / :265-366).
// in[16] raster coefficients (registers; int16 values: every caller's
// coefficients are int16), r = output row.  res[c] = (.. )>>3.
__device__ __forceinline__ void idct_row(const int in[16], int r, int res[4]) {
  int t[4];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const int a = in[c] + in[8 + c];
    const int b = in[c] - in[8 + c];
    const int cc = mul2_16(in[4 + c]) - mul1_16(in[12 + c]);
    const int d = mul1_16(in[4 + c]) + mul2_16(in[12 + c]);
    const int s0 = (r == 0 || r == 3) ? a : b;
    const int s1 = (r == 0 || r == 3) ? d : cc;
    t[c] = (r < 2) ? s0 + s1 : s0 - s1;
  }
  const int dc = t[0] + 4;
  const int a = dc + t[2], b = dc - t[2];
  const int cc = mul2_24(t[1]) - mul1_24(t[3]);
  const int d = mul1_24(t[1]) + mul2_24(t[3]);
  res[0] = (a + d) >> 3;
  res[1] = (b + cc) >> 3;
  res[2] = (b - cc) >> 3;
  res[3] = (a - d) >> 3;
}

// transformAC3 (transforms.go:170-193), one row: only in[0], in[1], in[4].
__device__ __forceinline__ void ac3_row(int in0, int in1, int in4, int r, int res[4]) {
  const int a = in0 + 4;
  const int c4 = mul2_16(in4), d4 = mul1_16(in4);
  const int c1 = mul2_16(in1), d1 = mul1_16(in1);
  const int rv = (r == 0) ? a + d4 : (r == 1) ? a + c4 : (r == 2) ? a - c4 : a - d4;
  res[0] = (rv + d1) >> 3;
  res[1] = (rv + c1) >> 3;
  res[2] = (rv - c1) >> 3;
  res[3] = (rv - d1) >> 3;
}

// Residual of one row of a block according to the decoder's 2-bit nz code
// (doTransform, decode_frame.go:22-43): 3 full, 2 AC3, 1 DC-only, 0 none.
__device__ __forceinline__ void dec_residual_row(const int16_t* __restrict__ co, int code, int r, int res[4]) {
  if (code == 3) {
    int in[16];
    const int4* p = reinterpret_cast<const int4*>(co);
    int4 q0 = p[0], q1 = p[1];
    const int w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
    for (int k = 0; k < 8; k++) {
      in[2 * k] = (int)(int16_t)(w[k] & 0xffff);
      in[2 * k + 1] = w[k] >> 16;
    }
    idct_row(in, r, res);
  } else if (code == 2) {
    const int w0 = reinterpret_cast<const int*>(co)[0];
    ac3_row((int)(int16_t)(w0 & 0xffff), w0 >> 16, co[4], r, res);
  } else if (code == 1) {
    const int add = (co[0] + 4) >> 3;
    res[0] = res[1] = res[2] = res[3] = add;
  } else {
    res[0] = res[1] = res[2] = res[3] = 0;
  }
}

// Inverse WHT of the 16 luma DCs (transforms.go:223-252); out[k] is the DC of
// block k (the reference writes it to out[16*k]); int16 stores wrap.
__device__ __forceinline__ void iwht(const int in[16], int16_t out[16]) {
  int tmp[16];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int a0 = in[i] + in[12 + i], a1 = in[4 + i] + in[8 + i];
    const int a2 = in[4 + i] - in[8 + i], a3 = in[i] - in[12 + i];
    tmp[i] = a0 + a1;
    tmp[8 + i] = a0 - a1;
    tmp[4 + i] = a3 + a2;
    tmp[12 + i] = a3 - a2;
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int dc = tmp[4 * i] + 3;
    const int a0 = dc + tmp[4 * i + 3], a1 = tmp[4 * i + 1] + tmp[4 * i + 2];
    const int a2 = tmp[4 * i + 1] - tmp[4 * i + 2], a3 = dc - tmp[4 * i + 3];
    out[4 * i + 0] = (int16_t)((a0 + a1) >> 3);
    out[4 * i + 1] = (int16_t)((a3 + a2) >> 3);
    out[4 * i + 2] = (int16_t)((a0 - a1) >> 3);
    out[4 * i + 3] = (int16_t)((a3 - a2) >> 3);
  }
}

// Forward WHT on a flat 4x4 DC array (transforms.go:500-531).
__device__ __forceinline__ void fwht(const int in[16], int16_t out[16]) {
  int tmp[16];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int a0 = in[4 * i] + in[4 * i + 2], a1 = in[4 * i + 1] + in[4 * i + 3];
    const int a2 = in[4 * i + 1] - in[4 * i + 3], a3 = in[4 * i] - in[4 * i + 2];
    tmp[4 * i + 0] = a0 + a1;
    tmp[4 * i + 1] = a3 + a2;
    tmp[4 * i + 2] = a3 - a2;
    tmp[4 * i + 3] = a0 - a1;
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int a0 = tmp[i] + tmp[8 + i], a1 = tmp[4 + i] + tmp[12 + i];
    const int a2 = tmp[4 + i] - tmp[12 + i], a3 = tmp[i] - tmp[8 + i];
    out[i] = (int16_t)((a0 + a1) >> 1);
    out[4 + i] = (int16_t)((a3 + a2) >> 1);
    out[8 + i] = (int16_t)((a3 - a2) >> 1);
    out[12 + i] = (int16_t)((a0 - a1) >> 1);
  }
}

// ------------------------------------------------------------------------
// Forward 4x4 DCT of (src - ref), both BPS/stride-strided (transforms.go:371-484).
__device__ __forceinline__ void fdct4x4(const int d[16], int16_t out[16]) {
  int tmp[16];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int d0 = d[4 * r], d1 = d[4 * r + 1], d2 = d[4 * r + 2], d3 = d[4 * r + 3];
    const int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
    tmp[4 * r + 0] = (a0 + a1) * 8;
    tmp[4 * r + 1] = (a2 * 2217 + a3 * 5352 + 1812) >> 9;
    tmp[4 * r + 2] = (a0 - a1) * 8;
    tmp[4 * r + 3] = (a3 * 2217 - a2 * 5352 + 937) >> 9;
  }
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const int a0 = tmp[c] + tmp[12 + c], a1 = tmp[4 + c] + tmp[8 + c];
    const int a2 = tmp[4 + c] - tmp[8 + c], a3 = tmp[c] - tmp[12 + c];
    out[c] = (int16_t)((a0 + a1 + 7) >> 4);
    out[4 + c] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0));
    out[8 + c] = (int16_t)((a0 - a1 + 7) >> 4);
    out[12 + c] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
  }
}

// The same FTransform on packed int16 pairs: dp01[k] = (d[k], d[4 + k])
// (rows 0 and 1 of column k), dp32[k] = (d[12 + k], d[8 + k]) (rows 3 and 2).
// The row pass runs two rows an instruction; its rotations and the column
// pass's four outputs are signed dot products (v_dot2_i32_i16) of the pairs
// (row sums P + Q = (a0, a1), differences P - Q = (a3, a2)).  Every value
// fits int16 (row outputs <= 8160 in magnitude, column sums <= 16320) and
// every dot product is exact in int32: the outputs equal fdct4x4's.
typedef short s16x2_t __attribute__((ext_vector_type(2)));
// VOP3P v_dot2_i32_i16 with its accumulator as an operand (the builtin's
// v_dot2c form accumulates in place: a v_mov of the constant before each)
__device__ __forceinline__ int sdot2_acc(s16x2_t a, s16x2_t b, int c) {
  int r;
  asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ void fdct4x4_rowpair(const s16x2_t d[4], s16x2_t t[4]) {
  const s16x2_t a0 = d[0] + d[3], a1 = d[1] + d[2], a2 = d[1] - d[2], a3 = d[0] - d[3];
  t[0] = (a0 + a1) << (short)3;
  t[2] = (a0 - a1) << (short)3;
  const s16x2_t x = {a2.x, a3.x}, y = {a2.y, a3.y};  // (a2, a3) of each row
  const s16x2_t k1 = {2217, 5352}, k3 = {-5352, 2217};
  t[1] = (s16x2_t){(short)(sdot2_acc(x, k1, 1812) >> 9),
                   (short)(sdot2_acc(y, k1, 1812) >> 9)};
  t[3] = (s16x2_t){(short)(sdot2_acc(x, k3, 937) >> 9),
                   (short)(sdot2_acc(y, k3, 937) >> 9)};
}
__device__ __forceinline__ void fdct4x4_pk(const s16x2_t dp01[4], const s16x2_t dp32[4], int out[16]) {
  s16x2_t P[4], Q[4];  // P[c] = (row 0, row 1), Q[c] = (row 3, row 2) of the row pass
  fdct4x4_rowpair(dp01, P);
  fdct4x4_rowpair(dp32, Q);
  const s16x2_t one = {1, 1}, pm = {1, -1}, k4 = {5352, 2217}, k12 = {2217, -5352};
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const s16x2_t S = P[c] + Q[c], D = P[c] - Q[c];  // (a0, a1), (a3, a2)
    out[c] = (int16_t)(sdot2_acc(S, one, 7) >> 4);
    out[8 + c] = (int16_t)(sdot2_acc(S, pm, 7) >> 4);
    out[4 + c] = (int16_t)((sdot2_acc(D, k4, 12000) >> 16) + (D.x != 0));
    out[12 + c] = (int16_t)(sdot2_acc(D, k12, 51000) >> 16);
  }
}

// ------------------------------------------------------------------------
// 4x4 intra prediction, one row per lane (predict_lossy.go:185-424).
// ctx: X = top-left, T[0..7] = top row incl. top-right, L[0..3] = left column.
// Returns the 4 predicted pixels of row y packed little-endian.
__device__ __forceinline__ uint32_t pred4_row(int mode, int y, int X, const int T[8], const int L[4]) {
  const int A = T[0], B = T[1], C = T[2], D = T[3], E = T[4], F = T[5], G = T[6], H = T[7];
  const int I = L[0], J = L[1], K = L[2], Lq = L[3];
  int p0, p1, p2, p3;
  switch (mode) {
    case 0: {  // dc4
      const int v = (A + B + C + D + I + J + K + Lq + 4) >> 3;
      p0 = p1 = p2 = p3 = v;
      break;
    }
    case 1: {  // tm4
      const int base = L[y] - X;
      p0 = clip8(base + A); p1 = clip8(base + B); p2 = clip8(base + C); p3 = clip8(base + D);
      break;
    }
    case 2:  // ve4
      p0 = avg3(X, A, B); p1 = avg3(A, B, C); p2 = avg3(B, C, D); p3 = avg3(C, D, E);
      break;
    case 3: {  // he4
      const int v = (y == 0) ? avg3(X, I, J) : (y == 1) ? avg3(I, J, K) : (y == 2) ? avg3(J, K, Lq) : avg3(K, Lq, Lq);
      p0 = p1 = p2 = p3 = v;
      break;
    }
    case 4: {  // rd4: value depends on x - y; e[k] for k = x - y + 3
      const int e[7] = {avg3(Lq, K, J), avg3(K, J, I), avg3(J, I, X), avg3(I, X, A),
                        avg3(X, A, B), avg3(A, B, C), avg3(B, C, D)};
      p0 = e[3 - y]; p1 = e[4 - y]; p2 = e[5 - y]; p3 = e[6 - y];
      break;
    }
    case 5: {  // vr4
      const int r0[4] = {avg2(X, A), avg2(A, B), avg2(B, C), avg2(C, D)};
      const int r1[4] = {avg3(I, X, A), avg3(X, A, B), avg3(A, B, C), avg3(B, C, D)};
      if (y == 0) { p0 = r0[0]; p1 = r0[1]; p2 = r0[2]; p3 = r0[3]; }
      else if (y == 1) { p0 = r1[0]; p1 = r1[1]; p2 = r1[2]; p3 = r1[3]; }
      else if (y == 2) { p0 = avg3(J, I, X); p1 = r0[0]; p2 = r0[1]; p3 = r0[2]; }
      else { p0 = avg3(K, J, I); p1 = r1[0]; p2 = r1[1]; p3 = r1[2]; }
      break;
    }
    case 6: {  // ld4: value depends on x + y
      const int e[7] = {avg3(A, B, C), avg3(B, C, D), avg3(C, D, E), avg3(D, E, F),
                        avg3(E, F, G), avg3(F, G, H), avg3(G, H, H)};
      p0 = e[y]; p1 = e[y + 1]; p2 = e[y + 2]; p3 = e[y + 3];
      break;
    }
    case 7: {  // vl4
      const int a2[4] = {avg2(A, B), avg2(B, C), avg2(C, D), avg2(D, E)};
      const int a3[5] = {avg3(A, B, C), avg3(B, C, D), avg3(C, D, E), avg3(D, E, F), avg3(E, F, G)};
      if (y == 0) { p0 = a2[0]; p1 = a2[1]; p2 = a2[2]; p3 = a2[3]; }
      else if (y == 1) { p0 = a3[0]; p1 = a3[1]; p2 = a3[2]; p3 = a3[3]; }
      else if (y == 2) { p0 = a2[1]; p1 = a2[2]; p2 = a2[3]; p3 = avg3(E, F, G); }
      else { p0 = a3[1]; p1 = a3[2]; p2 = a3[3]; p3 = avg3(F, G, H); }
      break;
    }
    case 8: {  // hd4
      const int q[10] = {avg2(X, I), avg3(I, X, A), avg3(X, A, B), avg3(A, B, C),  // row 0
                         avg2(I, J), avg3(X, I, J), avg2(J, K), avg3(I, J, K), avg2(K, Lq), avg3(J, K, Lq)};
      if (y == 0) { p0 = q[0]; p1 = q[1]; p2 = q[2]; p3 = q[3]; }
      else if (y == 1) { p0 = q[4]; p1 = q[5]; p2 = q[0]; p3 = q[1]; }
      else if (y == 2) { p0 = q[6]; p1 = q[7]; p2 = q[4]; p3 = q[5]; }
      else { p0 = q[8]; p1 = q[9]; p2 = q[6]; p3 = q[7]; }
      break;
    }
    default: {  // 9: hu4
      const int u0 = avg2(I, J), u1 = avg3(I, J, K), u2 = avg2(J, K), u3 = avg3(J, K, Lq);
      const int u4 = avg2(K, Lq), u5 = avg3(K, Lq, Lq);
      if (y == 0) { p0 = u0; p1 = u1; p2 = u2; p3 = u3; }
      else if (y == 1) { p0 = u2; p1 = u3; p2 = u4; p3 = u5; }
      else if (y == 2) { p0 = u4; p1 = u5; p2 = Lq; p3 = Lq; }
      else { p0 = p1 = p2 = p3 = Lq; }
      break;
    }
  }
  return pack4(p0, p1, p2, p3);
}

// Gather the 4x4 prediction context of the block at buf+off (BPS stride).
__device__ __forceinline__ void pred4_ctx(const uint8_t* buf, int off, int& X, int T[8], int L[4]) {
  const uint8_t* d = buf + off;
  X = d[-1 - WG_BPS];
#pragma unroll
  for (int i = 0; i < 8; i++) T[i] = d[i - WG_BPS];
#pragma unroll
  for (int j = 0; j < 4; j++) L[j] = d[-1 + j * WG_BPS];
}

// 16x16 / 8x8 prediction of the 4 pixels at (px..px+3, py) of a square
// block of `size` (predict_lossy.go:27-181).  dc = precomputed DC value
// (only used by modes 0, 4, 5, 6).  Mode numbering: DC TM V H NoTop NoLeft NoTopLeft.
__device__ __forceinline__ uint32_t predsq_row4(int mode, const uint8_t* d, int px, int py, int dc) {
  if (mode == 1) {  // TM
    const int base = d[-1 + py * WG_BPS] - d[-1 - WG_BPS];
    const uint8_t* t = d - WG_BPS + px;
    return pack4(clip8(base + t[0]), clip8(base + t[1]), clip8(base + t[2]), clip8(base + t[3]));
  }
  if (mode == 2) {  // VE
    const uint8_t* t = d - WG_BPS + px;
    return pack4(t[0], t[1], t[2], t[3]);
  }
  if (mode == 3) {  // HE
    const int v = d[-1 + py * WG_BPS];
    return pack4(v, v, v, v);
  }
  return 0x01010101u * (uint32_t)dc;
}

// DC value for a square predictor (needs the whole border): sizes 16 / 8.
__device__ __forceinline__ int predsq_dc(int mode, const uint8_t* d, int size) {
  const int shift = (size == 16) ? 5 : 4;
  if (mode == 6) return 128;
  int sum = 0;
  if (mode == 0 || mode == 5)
    for (int i = 0; i < size; i++) sum += d[i - WG_BPS];
  if (mode == 0 || mode == 4)
    for (int j = 0; j < size; j++) sum += d[-1 + j * WG_BPS];
  if (mode == 0) return (sum + size) >> shift;
  return (sum + (size >> 1)) >> (shift - 1);
}

// ------------------------------------------------------------------------
// Loop-filter sample operations (filter.go:13-87).  p is any address space;
// off is the q0 sample, step crosses the edge.
__device__ __forceinline__ bool f_needs(const uint8_t* p, int off, int step, int t2) {
  const int p1 = p[off - 2 * step], p0 = p[off - step], q0 = p[off], q1 = p[off + step];
  return 4 * abs(p0 - q0) + abs(p1 - q1) <= t2;
}
__device__ __forceinline__ bool f_needs2(const uint8_t* p, int off, int step, int t2, int it) {
  const int p3 = p[off - 4 * step], p2 = p[off - 3 * step], p1 = p[off - 2 * step], p0 = p[off - step];
  const int q0 = p[off], q1 = p[off + step], q2 = p[off + 2 * step], q3 = p[off + 3 * step];
  if (4 * abs(p0 - q0) + abs(p1 - q1) > t2) return false;
  return abs(p3 - p2) <= it && abs(p2 - p1) <= it && abs(p1 - p0) <= it && abs(q3 - q2) <= it &&
         abs(q2 - q1) <= it && abs(q1 - q0) <= it;
}
__device__ __forceinline__ bool f_hev(const uint8_t* p, int off, int step, int t) {
  const int p1 = p[off - 2 * step], p0 = p[off - step], q0 = p[off], q1 = p[off + step];
  return abs(p1 - p0) > t || abs(q1 - q0) > t;
}
__device__ __forceinline__ void f_do2(uint8_t* p, int off, int step) {
  const int p1 = p[off - 2 * step], p0 = p[off - step], q0 = p[off], q1 = p[off + step];
  const int a = 3 * (q0 - p0) + sclip1(p1 - q1);
  const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3);
  p[off - step] = clip8(p0 + a2);
  p[off] = clip8(q0 - a1);
}
__device__ __forceinline__ void f_do4(uint8_t* p, int off, int step) {
  const int p1 = p[off - 2 * step], p0 = p[off - step], q0 = p[off], q1 = p[off + step];
  const int a = 3 * (q0 - p0);
  const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3), a3 = (a1 + 1) >> 1;
  p[off - 2 * step] = clip8(p1 + a3);
  p[off - step] = clip8(p0 + a2);
  p[off] = clip8(q0 - a1);
  p[off + step] = clip8(q1 - a3);
}
__device__ __forceinline__ void f_do6(uint8_t* p, int off, int step) {
  const int p2 = p[off - 3 * step], p1 = p[off - 2 * step], p0 = p[off - step];
  const int q0 = p[off], q1 = p[off + step], q2 = p[off + 2 * step];
  const int a = sclip1(3 * (q0 - p0) + sclip1(p1 - q1));
  const int a1 = (27 * a + 63) >> 7, a2 = (18 * a + 63) >> 7, a3 = (9 * a + 63) >> 7;
  p[off - 3 * step] = clip8(p2 + a3);
  p[off - 2 * step] = clip8(p1 + a2);
  p[off - step] = clip8(p0 + a1);
  p[off] = clip8(q0 - a1);
  p[off + step] = clip8(q1 - a2);
  p[off + 2 * step] = clip8(q2 - a3);
}
// One sample of the simple filter (simpleVFilter16Go loop body, filter.go:93-105).
__device__ __forceinline__ void f_simple(uint8_t* p, int off, int step, int thresh) {
  if (f_needs(p, off, step, 2 * thresh + 1)) f_do2(p, off, step);
}
// One sample of filterLoop26 (mb edge) / filterLoop24 (inner), filter.go:144-190.
__device__ __forceinline__ void f_complex(uint8_t* p, int off, int step, int thresh, int ithresh, int hev_t,
                                          bool inner) {
  if (!f_needs2(p, off, step, 2 * thresh + 1, ithresh)) return;
  if (f_hev(p, off, step, hev_t)) f_do2(p, off, step);
  else if (inner) f_do4(p, off, step);
  else f_do6(p, off, step);
}

// ------------------------------------------------------------------------
// Register forms: one line of pixels (a row for the horizontal pass, a column
// for the vertical one) held in v[], an edge between v[K-1] and v[K].  Same
// arithmetic as f_simple / f_complex, written branch-free: conditions are
// combined with `&` (never `&&`) and applied as selects, and a disabled edge
// gets threshold -1 instead of an `if`, so the compiler keeps v[] in place
// (an `if` around array updates made it copy the whole line per edge).
template <int K, int N>
__device__ __forceinline__ void rf_simple(int (&v)[N], int t2) {
  const int p1 = v[K - 2], p0 = v[K - 1], q0 = v[K], q1 = v[K + 1];
  const int a = 3 * (q0 - p0) + sclip1(p1 - q1);
  const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3);
  const bool on = 4 * abs(p0 - q0) + abs(p1 - q1) <= t2;
  v[K - 1] = on ? clip8(p0 + a2) : p0;
  v[K] = on ? clip8(q0 - a1) : q0;
}
template <int K, int N, bool INNER>
__device__ __forceinline__ void rf_complex(int (&v)[N], int t2, int it, int hev_t) {
  const int p3 = v[K - 4], p2 = v[K - 3], p1 = v[K - 2], p0 = v[K - 1];
  const int q0 = v[K], q1 = v[K + 1], q2 = v[K + 2], q3 = v[K + 3];
  const int m = max(max(max(abs(p3 - p2), abs(p2 - p1)), max(abs(p1 - p0), abs(q3 - q2))),
                    max(abs(q2 - q1), abs(q1 - q0)));
  const bool on = (4 * abs(p0 - q0) + abs(p1 - q1) <= t2) & (m <= it);
  const bool hev = max(abs(p1 - p0), abs(q1 - q0)) > hev_t;
  if (INNER) {  // doFilter2 when hev, else doFilter4
    const int a = 3 * (q0 - p0) + (hev ? sclip1(p1 - q1) : 0);
    const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3), a3 = (a1 + 1) >> 1;
    const bool four = on & !hev;
    v[K - 2] = four ? clip8(p1 + a3) : p1;
    v[K - 1] = on ? clip8(p0 + a2) : p0;
    v[K] = on ? clip8(q0 - a1) : q0;
    v[K + 1] = four ? clip8(q1 - a3) : q1;
  } else {  // doFilter2 when hev, else doFilter6
    const int b = 3 * (q0 - p0) + sclip1(p1 - q1);
    const int w = sclip1(b);
    const int h1 = sclip2((b + 4) >> 3), h2 = sclip2((b + 3) >> 3);
    const int a1 = (27 * w + 63) >> 7, a2 = (18 * w + 63) >> 7, a3 = (9 * w + 63) >> 7;
    const bool six = on & !hev;
    v[K - 3] = six ? clip8(p2 + a3) : p2;
    v[K - 2] = six ? clip8(p1 + a2) : p1;
    v[K - 1] = on ? clip8(p0 + (hev ? h2 : a1)) : p0;
    v[K] = on ? clip8(q0 - (hev ? h1 : a1)) : q0;
    v[K + 1] = six ? clip8(q1 - a2) : q1;
    v[K + 2] = six ? clip8(q2 - a3) : q2;
  }
}
// All edges of one 20-pixel line in the reference's order: the MB edge between
// v[3] and v[4], then the inner edges at v[8], v[12], v[16].  Chroma lines
// (12 pixels: MB edge + one inner edge at v[8]) run the same code with
// `luma` false, which turns the edges at v[12] and v[16] off, so luma and
// chroma lanes share one instruction stream.  COMPLEX: filter type 2 (the
// simple filter, type 1, never reaches chroma).
template <bool COMPLEX>
__device__ __forceinline__ void rf_line(int (&v)[20], bool mb_edge, bool inner, bool luma, int limit, int ilevel,
                                        int hev_t) {
  const int t_mb = mb_edge ? 2 * (limit + 4) + 1 : -1;
  const int t_in = inner ? 2 * limit + 1 : -1;
  const int t_l = luma ? t_in : -1;
  if (COMPLEX) {
    rf_complex<4, 20, false>(v, t_mb, ilevel, hev_t);
    rf_complex<8, 20, true>(v, t_in, ilevel, hev_t);
    rf_complex<12, 20, true>(v, t_l, ilevel, hev_t);
    rf_complex<16, 20, true>(v, t_l, ilevel, hev_t);
  } else {
    rf_simple<4, 20>(v, t_mb);
    rf_simple<8, 20>(v, t_in);
    rf_simple<12, 20>(v, t_l);
    rf_simple<16, 20>(v, t_l);
  }
}

// ------------------------------------------------------------------------
// Distortion metrics (ssim.go:188-335), one block per lane.
__device__ __forceinline__ int sse_nxn(const uint8_t* a, const uint8_t* b, int n) {
  int s = 0;
  for (int y = 0; y < n; y++)
    for (int x = 0; x < n; x++) {
      const int d = a[x + y * WG_BPS] - b[x + y * WG_BPS];
      s += d * d;
    }
  return s;
}
__device__ __forceinline__ int ttransform(const uint8_t* in) {
  const int kw[16] = {38, 32, 20, 9, 32, 28, 17, 7, 20, 17, 10, 4, 9, 7, 4, 2};
  int tmp[16];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint8_t* r = in + i * WG_BPS;
    const int a0 = r[0] + r[2], a1 = r[1] + r[3], a2 = r[1] - r[3], a3 = r[0] - r[2];
    tmp[4 * i] = a0 + a1;
    tmp[4 * i + 1] = a3 + a2;
    tmp[4 * i + 2] = a3 - a2;
    tmp[4 * i + 3] = a0 - a1;
  }
  int sum = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int a0 = tmp[i] + tmp[8 + i], a1 = tmp[4 + i] + tmp[12 + i];
    const int a2 = tmp[4 + i] - tmp[12 + i], a3 = tmp[i] - tmp[8 + i];
    sum += kw[i] * abs(a0 + a1) + kw[4 + i] * abs(a3 + a2) + kw[8 + i] * abs(a3 - a2) + kw[12 + i] * abs(a0 - a1);
  }
  return sum;
}
__device__ __forceinline__ int tdisto4x4(const uint8_t* a, const uint8_t* b) {
  return abs(ttransform(b) - ttransform(a)) >> 5;
}

// ------------------------------------------------------------------------
// SSIM statistics (ssim.go:12-83).
struct SsimStats {
  uint32_t w, xm, ym, xxm, xym, yym;
};
__device__ __forceinline__ double ssim_calc(const SsimStats& s, uint32_t n) {
  const uint64_t w2 = (uint64_t)n * n;
  const uint64_t c1 = 20 * w2, c2 = 60 * w2, c3 = 64 * w2;
  const uint64_t xmxm = (uint64_t)s.xm * s.xm, ymym = (uint64_t)s.ym * s.ym;
  if (xmxm + ymym < c3) return 1.0;
  const int64_t xmym = (int64_t)s.xm * (int64_t)s.ym;
  const int64_t sxy = (int64_t)s.xym * (int64_t)n - xmym;
  const uint64_t sxx = (uint64_t)s.xxm * n - xmxm;
  const uint64_t syy = (uint64_t)s.yym * n - ymym;
  const uint64_t sxy_pos = sxy > 0 ? (uint64_t)sxy : 0;
  const uint64_t num_s = (2 * sxy_pos + c2) >> 8;
  const uint64_t den_s = (sxx + syy + c2) >> 8;
  const uint64_t fnum = (2 * (uint64_t)xmym + c1) * num_s;
  const uint64_t fden = (xmxm + ymym + c1) * den_s;
  if (fden == 0) return 1.0;
  return (double)fnum / (double)fden;
}

}  // namespace wg
