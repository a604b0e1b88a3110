// vp8l.hip -- VP8L predictor transform on gfx950.
//
//   k_vp8l_select    ResidualImage phase 1: per tile, the entropy estimate of
//                    every candidate predictor and its argmin
//                    (internal/lossless/encode_predictor.go:194-277, 396-440)
//   k_vp8l_residual  ResidualImage phase 2: residual = ARGB -mod prediction
//                    from ORIGINAL pixels (copyImageWithPrediction :298-363)
//   k_vp8l_inverse   predictorInverseTransform (decode_transform.go:202-360)
//   k_vp8l_green     SubtractGreen (encode_predictor.go:461) / AddGreenToBlueAndRed
//
// Bit-exactness of the mode choice: the entropy is a float64 sum that the
// reference accumulates in a fixed order (count term first, then bins 0..255
// of alpha, red, green, blue); k_vp8l_select keeps exactly that order (one lane
// per channel walks its 256 bins) and takes fastSLog2 values from the same
// LUT the reference builds (i * math.Log2(i), built on the host by
// vp8l_host.cpp's restatement of Go's math.Log2).  No FMA contraction anywhere
// in this file.
#include "wg_common.h"
#include "wg_instr.h"

#pragma clang fp contract(off)

namespace {

constexpr uint32_t ARGB_BLACK = 0xff000000u;

// LDS written by this wave is visible to all its lanes, and the compiler may
// not move LDS accesses across this point.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
constexpr int SLOG2_LUT = 65536;

__device__ __forceinline__ uint32_t sub_pixels(uint32_t a, uint32_t b) {
  const uint32_t ag = 0x00ff00ffu + (a & 0xff00ff00u) - (b & 0xff00ff00u);
  const uint32_t rb = 0xff00ff00u + (a & 0x00ff00ffu) - (b & 0x00ff00ffu);
  return (ag & 0xff00ff00u) | (rb & 0x00ff00ffu);
}
// per-byte a + b mod 256: the low 7 bits of each byte add without carrying
// out of it, and bit 7 is a7 ^ b7 ^ the carry into it (v_xor3 + v_bfi)
__device__ __forceinline__ uint32_t add_pixels(uint32_t a, uint32_t b) {
  const uint32_t s = (a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu);
  return ((a ^ b ^ s) & 0x80808080u) | (s & 0x7f7f7f7fu);
}
// per-byte floor((a + b) / 2): v_lerp_u8 with no rounding bits
__device__ __forceinline__ uint32_t avg2(uint32_t a, uint32_t b) { return __builtin_amdgcn_lerp(a, b, 0u); }
__device__ __forceinline__ int chan(uint32_t v, int s) { return (int)((v >> s) & 0xff); }
// Select (encode_predictor.go:49-95): sum over channels of |l - tl| minus
// that of |t - tl|, as two v_sad_u8 (sum of absolute byte differences)
__device__ __forceinline__ uint32_t select_pred(uint32_t l, uint32_t t, uint32_t tl) {
  const int pa = (int)__builtin_amdgcn_sad_u8(l, tl, 0u) - (int)__builtin_amdgcn_sad_u8(t, tl, 0u);
  return pa <= 0 ? t : l;
}
// The clamped predictors on two 16-bit lanes at a time (bytes 0, 2 and bytes
// 1, 3 of the pixel); every intermediate fits int16.
typedef short v2i16 __attribute__((ext_vector_type(2)));
// bytes 0, 2 (lo) / 1, 3 (hi) of a pixel as two 16-bit lanes, and back (v_perm_b32)
__device__ __forceinline__ v2i16 as_v2(uint32_t x) { return __builtin_bit_cast(v2i16, x); }
__device__ __forceinline__ uint32_t as_u(v2i16 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ v2i16 lanes_lo(uint32_t x) { return as_v2(__builtin_amdgcn_perm(0u, x, 0x0c020c00u)); }
__device__ __forceinline__ v2i16 lanes_hi(uint32_t x) { return as_v2(__builtin_amdgcn_perm(0u, x, 0x0c030c01u)); }
__device__ __forceinline__ uint32_t pack_lanes(v2i16 lo, v2i16 hi) { return __builtin_amdgcn_perm(as_u(hi), as_u(lo), 0x06020400u); }
__device__ __forceinline__ v2i16 clamp255(v2i16 v) {
  const v2i16 zero = {0, 0}, top = {255, 255};
  return __builtin_elementwise_min(__builtin_elementwise_max(v, zero), top);
}
__device__ __forceinline__ uint32_t clamp_add_sub_full(uint32_t a, uint32_t b, uint32_t c) {
  const v2i16 lo = clamp255(lanes_lo(a) + lanes_lo(b) - lanes_lo(c));  // bytes 0, 2
  const v2i16 hi = clamp255(lanes_hi(a) + lanes_hi(b) - lanes_hi(c));  // bytes 1, 3
  return pack_lanes(lo, hi);
}
__device__ __forceinline__ v2i16 half_step(v2i16 va, v2i16 vc) {
  const v2i16 d = va - vc;
  // d / 2 truncating toward zero, as Go's '/': add the sign bit to d before the arithmetic shift
  typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));
  const v2i16 neg = __builtin_bit_cast(v2i16, __builtin_bit_cast(v2u16, d) >> (v2u16){15, 15});
  return clamp255(va + ((d + neg) >> (v2i16){1, 1}));
}
__device__ __forceinline__ uint32_t clamp_add_sub_half(uint32_t avg, uint32_t c) {
  return pack_lanes(half_step(lanes_lo(avg), lanes_lo(c)), half_step(lanes_hi(avg), lanes_hi(c)));
}
// predictPixel (encode_predictor.go:148-180); the decoder's switch
// (decode_transform.go:257-350) computes the same predictors.
__device__ __forceinline__ uint32_t predict(int mode, uint32_t l, uint32_t t, uint32_t tr, uint32_t tl) {
  switch (mode) {
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

// The same predictors for a lane-varying mode with little divergence (the
// inverse walk's lanes sit in up to ~10 tiles at once, and a switch runs the
// union of their cases).  Modes 1-10 are all avg2(avg2(A, B), avg2(C, D)) with
// A..D drawn from (L, T, TR, TL) -- L = avg2(L, L) etc. -- so one branch-free
// form with per-mode input codes (2 bits each: 0 L, 1 T, 2 TR, 3 TL) covers
// them and mode 13's avg2(L, T); only Select (11) and the clamped
// predictors (12, 13) branch.  Modes 0, 14, 15: black.
__device__ __forceinline__ uint32_t predict_lanes(int mode, uint32_t l, uint32_t t, uint32_t tr, uint32_t tl) {
#define PCODE(a, b, c, d) (uint64_t)((a) | (b) << 2 | (c) << 4 | (d) << 6)
  constexpr uint64_t K0 = PCODE(0, 0, 0, 0) | PCODE(0, 0, 0, 0) << 8 | PCODE(1, 1, 1, 1) << 16 |
                          PCODE(2, 2, 2, 2) << 24 | PCODE(3, 3, 3, 3) << 32 | PCODE(0, 2, 1, 1) << 40 |
                          PCODE(0, 0, 3, 3) << 48 | PCODE(0, 0, 1, 1) << 56;  // modes 0-7
  constexpr uint64_t K1 = PCODE(3, 3, 1, 1) | PCODE(1, 1, 2, 2) << 8 | PCODE(0, 3, 1, 2) << 16 |
                          PCODE(0, 0, 1, 1) << 40;  // modes 8-15 (13: avg2(L, T))
#undef PCODE
  const uint32_t code = (uint32_t)((mode < 8 ? K0 : K1) >> (8 * (mode & 7)));
  auto pick = [&](uint32_t i) {
    const uint32_t lo = (i & 1) ? t : l, hi = (i & 1) ? tl : tr;
    return (i & 2) ? hi : lo;
  };
  const uint32_t avg = avg2(avg2(pick(code & 3), pick((code >> 2) & 3)), avg2(pick((code >> 4) & 3), pick((code >> 6) & 3)));
  uint32_t p = (mode == 0 || mode >= 14) ? ARGB_BLACK : avg;
  if (mode == 11) p = select_pred(l, t, tl);
  else if (mode == 12) p = clamp_add_sub_full(l, t, tl);
  else if (mode == 13) p = clamp_add_sub_half(avg, tl);
  return p;
}

// The inverse walk's predictor as one branch-free stream: every candidate
// the modes share is formed once and a per-pixel control word (kPredCtl,
// staged per chunk) picks among them with bit masks -- no lane-varying switch,
// no compare-to-mask hazards.  Modes 1-10 and 13's inner average are
// avg2(P, Q) with P in {L, T, TR, TL, avg2(L, TR), avg2(L, TL)} and Q in
// {L, T, TR, TL, avg2(T, TR)} (avg2(X, X) = X); 11 / 12 / 13 / black override.
enum : uint32_t {
  C_PAVG = 1u << 0,   // P = avg2(L, R1)
  C_PL = 1u << 1,     // P = L (else Pc)
  C_PC_TR = 1u << 2,  // Pc = TR (else T)
  C_PC_TL = 1u << 3,  // Pc = TL
  C_R1_TL = 1u << 4,  // R1 = TL (else TR)
  C_QL = 1u << 5,     // Q = L (else Qc)
  C_Q6 = 1u << 6,     // Qc: 0 T, C_Q6 TR, C_Q7 TL, both avg2(T, TR)
  C_Q7 = 1u << 7,
  C_SEL = 1u << 8,    // Select (11)
  C_CF = 1u << 9,     // ClampAddSubtractFull (12)
  C_CH = 1u << 10,    // ClampAddSubtractHalf (13) of avg2(L, T)
  C_BLACK = 1u << 11, // 0, 14, 15
  C_EDGE = 1u << 12,  // x = width - 1: TR is this row's first pixel
};
constexpr uint32_t kPredCtl[16] = {
    C_BLACK,                          // 0
    C_PL | C_QL,                      // 1 L
    0,                                // 2 T
    C_PC_TR | C_Q6,                   // 3 TR
    C_PC_TL | C_Q7,                   // 4 TL
    C_PAVG,                           // 5 avg2(avg2(L, TR), T)
    C_PL | C_Q7,                      // 6 avg2(L, TL)
    C_PL,                             // 7 avg2(L, T)
    C_PC_TL,                          // 8 avg2(TL, T)
    C_Q6,                             // 9 avg2(T, TR)
    C_PAVG | C_R1_TL | C_Q6 | C_Q7,   // 10 avg2(avg2(L, TL), avg2(T, TR))
    C_SEL,                            // 11
    C_CF,                             // 12
    C_CH | C_PL,                      // 13 (avg2(L, T) first)
    C_BLACK, C_BLACK};
// Go math.Log / math.Log2 (src/math/log.go, log10.go) for counts beyond the
// LUT (tiles of 512 px at bits = 9); same operation sequence as the host LUT.
__device__ double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01;
  const double L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01;
  const double L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01;
  const double L7 = 1.479819860511658591e-01;
  int ki;
  double f1 = frexp(x, &ki);
  if (f1 < 0.70710678118654752440) {
    f1 *= 2;
    ki--;
  }
  const double f = f1 - 1, k = (double)ki;
  const double s = f / (2 + f), s2 = s * s, s4 = s2 * s2;
  const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const double R = t1 + t2, hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}
__device__ double fast_slog2(const double* __restrict__ lut, uint32_t v) {
  if (v < (uint32_t)SLOG2_LUT) return lut[v];
  int e;
  const double fv = (double)v;
  const double frac = frexp(fv, &e);
  const double l2 = frac == 0.5 ? (double)(e - 1) : go_log(frac) * 0x1.71547652b82fep+0 + (double)e;
  return fv * l2;
}

struct SelArgs {
  const uint32_t* argb;
  int64_t pitch;  // pixels per image
  uint32_t* modes;
  const double* lut;
  int width, height, bits, tiles_x, tiles_y, max_mode;
  int ty0, band_tiles;  // tile rows [ty0, ty0 + band_tiles / tiles_x) of each image
};

constexpr int SEL_WAVES = 4;

// One workgroup per tile; wave w evaluates modes w, w+4, ...  Histograms
// (4 x 256 u32) per wave in LDS; the per-channel float64 sums run on lanes
// 0-3, each walking its channel's bins in order.
__global__ __launch_bounds__(64 * SEL_WAVES) void k_vp8l_select(SelArgs a) {
  __shared__ uint32_t hist[SEL_WAVES][4 * 256];
  __shared__ double terms[SEL_WAVES][4 * 256];  // each bin's fastSLog2 term
  __shared__ double chan_cost[SEL_WAVES][4];
  __shared__ double cost[14];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile = blockIdx.x % a.band_tiles + a.ty0 * a.tiles_x;
  const int img = blockIdx.x / a.band_tiles;
  const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
  const uint32_t* argb = a.argb + img * a.pitch;
  const int ts = 1 << a.bits, w = a.width, h = a.height;
  const int x0 = tx * ts, y0 = ty * ts;
  const int x1 = min(x0 + ts, w), y1 = min(y0 + ts, h);
  const int ystep = (y1 - y0 > 16) ? 2 : 1;
  const int tw = x1 - x0, rows = (y1 - y0 + ystep - 1) / ystep;
  const uint32_t count = (uint32_t)(tw * rows);
  uint32_t* hg = hist[wave];
  // (WG_BOUNDS) the rows this launch may read: its band's and the one above
  [[maybe_unused]] const int r_lo = max(a.ty0 * ts - 1, 0), r_hi = min((a.ty0 + a.band_tiles / a.tiles_x) * ts, h);
  [[maybe_unused]] const uint32_t* band_px = argb + (int64_t)r_lo * w;
  [[maybe_unused]] const int64_t band_n = (int64_t)(r_hi - r_lo) * w * 4;
  auto px = [&](const uint32_t* p) { return WG_CHK(p, 4, band_px, band_n, "k_vp8l_select argb") ? *p : 0u; };

  for (int mode = wave; mode < a.max_mode; mode += SEL_WAVES) {
    for (int i = lane; i < 4 * 256; i += 64) hg[i] = 0;
    wave_lds_sync();  // this wave's zeroing lands before its adds
    for (int i = lane; i < tw * rows; i += 64) {
      const int x = x0 + i % tw, y = y0 + (i / tw) * ystep;
      const uint32_t* row = argb + (int64_t)y * w;
      uint32_t l = 0, t = 0, tr = 0, tl = 0;
      if (x > 0) l = px(row + x - 1);
      if (y > 0) {
        const uint32_t* prev = row - w;
        t = px(prev + x);
        if (x > 0) tl = px(prev + x - 1);
        tr = (x < w - 1) ? px(prev + x + 1) : t;
      }
      const uint32_t res = sub_pixels(px(row + x), predict(mode, l, t, tr, tl));
      atomicAdd(&hg[0 * 256 + ((res >> 24) & 0xff)], 1u);
      atomicAdd(&hg[1 * 256 + ((res >> 16) & 0xff)], 1u);
      atomicAdd(&hg[2 * 256 + ((res >> 8) & 0xff)], 1u);
      atomicAdd(&hg[3 * 256 + (res & 0xff)], 1u);
    }
    wave_lds_sync();
    // the terms fastSLog2(v) of every bin, looked up by all lanes at once
    // (0.0 for an empty bin: ce - 0.0 == ce, so the sum below equals the
    // reference's, which skips them); the float64 sum stays serial, in the
    // reference's order, on one lane per channel
    double* tm = terms[wave];
#pragma unroll 4
    for (int i = lane; i < 4 * 256; i += 64) {
      const uint32_t v = hg[i];
      tm[i] = v > 0 ? fast_slog2(a.lut, v) : 0.0;
    }
    wave_lds_sync();
    if (lane < 4) {  // estimateEntropy's float64 sum, in the reference's order
      const double* tc = tm + lane * 256;
      double ce = fast_slog2(a.lut, count);
#pragma unroll 8
      for (int i = 0; i < 256; i++) ce -= tc[i];
      chan_cost[wave][lane] = ce;
    }
    wave_lds_sync();
    if (lane == 0) {
      double e = 0.0;
      for (int c = 0; c < 4; c++) e += chan_cost[wave][c];
      cost[mode] = count == 0 ? 0.0 : e;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int best = 0;
    double best_cost = 1.7976931348623157e308;
    for (int m = 0; m < a.max_mode; m++)
      if (cost[m] < best_cost) {
        best_cost = cost[m];
        best = m;
      }
    a.modes[(int64_t)img * a.tiles_x * a.tiles_y + tile] = ((uint32_t)best << 8) | ARGB_BLACK;
  }
}

// ResidualImage phase 1 for tiles of at most 32 x 32 px (bits <= 5, so every
// histogram count is <= 512): a 2-wave workgroup a tile and one pass over
// its samples for all modes at once.
//   - The tile and its border are staged in LDS with estimateEntropy's edge
//     values already in place (0 left of column 0 and above row 0, the last
//     pixel repeated right of the last column: TR = T there), every load
//     issued before the first store.
//   - Sample lanes: lane l takes one sample (two sample rows of up to 32 per
//     pass; wave h the rows h, h + 2, ...) and forms all 14 predictions at
//     once -- modes 1-4 are its neighbours, the averages share their avg2
//     terms, only Select and the two clamps cost more -- and its 14 residuals
//     go to an LDS transpose buffer (rows of 68 words: the column lanes' 16-B
//     reads of one sample quad land on 14 disjoint bank quads).
//   - Column lanes: lane 4m + c owns the histogram of (mode m, channel c),
//     bins b and b + 128 as the two 16-bit halves of word b & 127, columns 64
//     words apart (every lane adds to its own bank: ds_add_u32, no return, no
//     contention however flat the content); it reads mode m's residuals back
//     and adds channel c's bins (address and increment: two bit-field
//     extracts).  The two waves' adds to one word serialise in the LDS.
//   - After the barrier wave 1 exits and lane 4m + c of wave 0 runs the
//     (mode, channel) float64 sum of estimateEntropy
//     (encode_predictor.go:262-275) in the reference's order: fastSLog2(count)
//     minus the bins 0..255 (an empty bin subtracts fastSLog2(0) = 0.0, which
//     leaves the sum unchanged); the 56 sums run at once (the whole column read
//     first, then the LUT in batches), and each mode's four channel sums are
//     added alpha, red, green, blue from 0.0 as the reference adds them.  The
//     argmin keeps the reference's first strict minimum in mode order
//     (:408-418).
// fastSLog2 of 0..512 is staged in LDS from the same device table.  48.5 KB a
// workgroup, three workgroups (six waves) a CU.  (Round 5 measured the
// alternatives -- one wave a tile with lane (mode, sample) running the
// branch-free predictor of its one mode, and the same on two waves -- at
// 1.27 / 0.60 ms against this kernel's 0.43 ms at 4096^2)
constexpr int SQ_LUT = 513;   // counts 0..512
__device__ __forceinline__ double dpp_quad_f64(double v, int j) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  int lo = (int)(uint32_t)u, hi = (int)(uint32_t)(u >> 32);
  switch (j) {  // (j is a constant at every call)
    case 0: lo = __builtin_amdgcn_mov_dpp(lo, 0x00, 0xf, 0xf, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x00, 0xf, 0xf, false); break;
    case 1: lo = __builtin_amdgcn_mov_dpp(lo, 0x55, 0xf, 0xf, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x55, 0xf, 0xf, false); break;
    case 2: lo = __builtin_amdgcn_mov_dpp(lo, 0xaa, 0xf, 0xf, false); hi = __builtin_amdgcn_mov_dpp(hi, 0xaa, 0xf, 0xf, false); break;
    default: lo = __builtin_amdgcn_mov_dpp(lo, 0xff, 0xf, 0xf, false); hi = __builtin_amdgcn_mov_dpp(hi, 0xff, 0xf, 0xf, false); break;
  }
  return __builtin_bit_cast(double, (uint64_t)(uint32_t)hi << 32 | (uint32_t)lo);
}
constexpr int SQ_SW = 34;     // staged tile row: columns x0 - 1 .. x0 + 32
constexpr int SQ2_COLS = 56;  // (mode, channel) column lanes
constexpr int SQ3_XS = 68;  // transpose buffer row stride (words)
__global__ __launch_bounds__(128) void k_vp8l_select_q3(SelArgs a, int64_t total) {
  __shared__ uint32_t hist[128 * 64];
  __shared__ uint32_t stile[33 * SQ_SW];
  __shared__ double lut[SQ_LUT];
  __shared__ uint4 xbuf_all[2][14 * SQ3_XS / 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t t_idx = blockIdx.x;
  if (t_idx >= total) return;  // (grid = total: never; no barrier skipped)
  const int tile = (int)(t_idx % a.band_tiles) + a.ty0 * a.tiles_x;
  const int img = (int)(t_idx / a.band_tiles);
  const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
  const uint32_t* argb = a.argb + img * a.pitch;
  const int ts = 1 << a.bits, w = a.width, h = a.height;
  const int x0 = tx * ts, y0 = ty * ts;
  const int x1 = min(x0 + ts, w), y1 = min(y0 + ts, h);
  const int ystep = (y1 - y0 > 16) ? 2 : 1;
  const int tw = x1 - x0, rows = (y1 - y0 + ystep - 1) / ystep;
  // (WG_BOUNDS) the rows this launch may read: its band's and the one above
  [[maybe_unused]] const int r_lo = max(a.ty0 * ts - 1, 0), r_hi = min((a.ty0 + a.band_tiles / a.tiles_x) * ts, h);
  [[maybe_unused]] const uint32_t* band_px = argb + (int64_t)r_lo * w;
  [[maybe_unused]] const int64_t band_n = (int64_t)(r_hi - r_lo) * w * 4;
  {
    // staged rows y0 - 1 .. y1 - 1 with estimateEntropy's edge values;
    // i / scols by a multiply (exact: i < 2^16 / scols)
    const int srows = y1 - y0 + 1, scols = x1 - x0 + 2, n = srows * scols;
    const uint32_t inv = (65535u + (uint32_t)scols) / (uint32_t)scols;  // ceil(2^16 / scols)
    constexpr int SN = (33 * SQ_SW + 127) / 128;
    uint32_t v[SN];
    int at[SN];
#pragma unroll
    for (int j = 0; j < SN; j++) {
      const int i = (int)threadIdx.x + 128 * j;
      const int rr = (int)(((uint32_t)i * inv) >> 16), cc = i - rr * scols;
      v[j] = 0;
      at[j] = rr * SQ_SW + cc;
      if (i < n) {
        const int y = y0 - 1 + rr, x = x0 - 1 + cc;
        const uint32_t* p = argb + (int64_t)y * w + min(x, w - 1);
        if (y >= 0 && x >= 0 && WG_CHK(p, 4, band_px, band_n, "k_vp8l_select_q3 argb")) v[j] = *p;
      }
    }
    for (int i = threadIdx.x; i < SQ_LUT; i += 128) lut[i] = a.lut[i];
    for (int i = threadIdx.x; i < 128 * 64 / 4; i += 128) reinterpret_cast<uint4*>(hist)[i] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < SN; j++)
      if ((int)threadIdx.x + 128 * j < n) stile[at[j]] = v[j];
  }
  __syncthreads();
  uint32_t* const xb = reinterpret_cast<uint32_t*>(xbuf_all[wave]);
  const int col_m = lane >> 2, shift = 24 - 8 * (lane & 3);  // column lane: mode, channel (alpha, red, green, blue)
  const bool col = lane < SQ2_COLS;
  const uint32_t* const xrow = xb + (col ? col_m : 0) * SQ3_XS;
  uint32_t* const myh = hist + lane;
  const int half = lane >> 5, sx = lane & 31;
  // wave w: sample rows w, w + 2, ...; a pass takes two of them (lanes 0-31 /
  // 32-63), so pass k covers rows w + 4k and w + 4k + 2
  for (int yy0 = wave; yy0 < rows; yy0 += 4) {
    const int yy = yy0 + 2 * half;
    {
      const int c = min(sx, tw - 1) + 1;                                  // staged column of x
      const uint32_t* srow = stile + (1 + min(yy, rows - 1) * ystep) * SQ_SW;  // staged row y0 + yy * ystep
      const uint32_t* sprev = srow - SQ_SW;
      const uint32_t p = srow[c], l = srow[c - 1], t = sprev[c], tl = sprev[c - 1], tr = sprev[c + 1];
#pragma unroll
      for (int m = 0; m < 14; m++) xb[m * SQ3_XS + lane] = sub_pixels(p, predict(m, l, t, tr, tl));
    }
    // (the LDS unit runs one wave's DS instructions in issue order: the reads
    // below see every lane's writes above with no wait, and the next pass's
    // writes come after these reads; only the compiler must keep the order)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int n0 = min(tw, 32), n1 = yy0 + 2 < rows ? n0 : 0;  // live samples of each row (wave-uniform)
    if (col) {
#pragma unroll
      for (int hh = 0; hh < 2; hh++) {
        const int nv = hh ? n1 : n0;
#pragma unroll
        for (int q = 0; q < 8; q++) {
          if (4 * q >= nv) break;  // (wave-uniform)
          const uint4 r4 = *reinterpret_cast<const uint4*>(xrow + 32 * hh + 4 * q);
          const uint32_t rv[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
          for (int k = 0; k < 4; k++) {
            if (k > 0 && 4 * q + k >= nv) break;
            const uint32_t b7 = __builtin_amdgcn_ubfe(rv[k], shift, 7), hi = __builtin_amdgcn_ubfe(rv[k], shift + 7, 1);
            __hip_atomic_fetch_add(myh + 64 * b7, 1u + 65535u * hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  if (wave != 0) return;  // (no barrier below)
  const uint32_t count = (uint32_t)(tw * rows);
  double ce = 0.0;
  if (col) {
    uint32_t hv[128];
#pragma unroll
    for (int k = 0; k < 128; k++) hv[k] = myh[64 * k];
    ce = lut[count];
#pragma unroll
    for (int hh = 0; hh < 2; hh++) {
#pragma unroll
      for (int k0 = 0; k0 < 128; k0 += 32) {
        double lv[32];
#pragma unroll
        for (int k = 0; k < 32; k++) lv[k] = lut[hh ? hv[k0 + k] >> 16 : hv[k0 + k] & 0xffff];
#pragma unroll
        for (int k = 0; k < 32; k++) ce -= lv[k];
      }
    }
  }
  const double e = (((0.0 + dpp_quad_f64(ce, 0)) + dpp_quad_f64(ce, 1)) + dpp_quad_f64(ce, 2)) + dpp_quad_f64(ce, 3);
  const uint64_t eb = __builtin_bit_cast(uint64_t, e);
  int best = 0;
  double best_cost = 1.7976931348623157e308;
  for (int mm = 0; mm < a.max_mode; mm++) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)eb, 4 * mm);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(eb >> 32), 4 * mm);
    const double cm = __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
    if (cm < best_cost) {
      best_cost = cm;
      best = mm;
    }
  }
  uint32_t* const mp = a.modes + (int64_t)img * a.tiles_x * a.tiles_y + tile;
  if (lane == 0 && WG_CHK(mp, 4, a.modes + (int64_t)img * a.tiles_x * a.tiles_y + a.ty0 * a.tiles_x, 4ll * a.band_tiles,
                          "k_vp8l_select_q3 modes"))
    *mp = ((uint32_t)best << 8) | ARGB_BLACK;
}

struct ResArgs {
  const uint32_t* argb;
  const uint32_t* modes;
  uint32_t* out;
  int64_t pitch;
  int width, height, bits, tiles_x, tiles_y;
  int y0, rows;  // pixel rows [y0, y0 + rows) of each image
};

// copyImageWithPrediction: one thread per pixel, predictions from original
// pixels; at the right edge TR is the current row's first pixel
// (upperRow[width]); row 0 / column 0 use black / left / top.
// Grid (column blocks, rows, images): no index division (a 64-bit divide per
// pixel was most of this kernel's instructions).
__global__ __launch_bounds__(256) void k_vp8l_residual(ResArgs a) {
  const int x = (int)blockIdx.x * 256 + (int)threadIdx.x;
  if (x >= a.width) return;
  const int y = a.y0 + (int)blockIdx.y, img = (int)blockIdx.z;
  const int64_t p = (int64_t)y * a.width + x;
  const uint32_t* cur = a.argb + img * a.pitch + (int64_t)y * a.width;
  // (WG_BOUNDS) reads: the launch's rows and the one above; writes: its rows;
  // modes: its tile rows
  [[maybe_unused]] const int r_lo = max(a.y0 - 1, 0);
  [[maybe_unused]] const uint32_t* rows_px = a.argb + img * a.pitch + (int64_t)r_lo * a.width;
  [[maybe_unused]] const int64_t rows_n = (int64_t)(a.y0 + a.rows - r_lo) * a.width * 4;
  auto px = [&](const uint32_t* q) { return WG_CHK(q, 4, rows_px, rows_n, "k_vp8l_residual argb") ? *q : 0u; };
  uint32_t pred;
  if (y == 0) {
    pred = x == 0 ? ARGB_BLACK : px(cur + x - 1);
  } else if (x == 0) {
    pred = px(cur - a.width);
  } else {
    const uint32_t* up = cur - a.width;
    const uint32_t* mp = a.modes + (int64_t)img * a.tiles_x * a.tiles_y + (y >> a.bits) * a.tiles_x + (x >> a.bits);
    [[maybe_unused]] const uint32_t* mrows = a.modes + (int64_t)img * a.tiles_x * a.tiles_y + (a.y0 >> a.bits) * a.tiles_x;
    const int mode = WG_CHK(mp, 4, mrows, 4ll * a.tiles_x * (((a.y0 + a.rows - 1) >> a.bits) - (a.y0 >> a.bits) + 1),
                            "k_vp8l_residual modes") ? (int)((*mp >> 8) & 0xff) : 0;
    const uint32_t tr = (x < a.width - 1) ? px(up + x + 1) : px(cur);
    pred = predict(mode, px(cur + x - 1), px(up + x), tr, px(up + x - 1));
  }
  uint32_t* const o = a.out + img * a.pitch + p;
  if (WG_CHK(o, 4, a.out + img * a.pitch + (int64_t)a.y0 * a.width, (int64_t)a.rows * a.width * 4, "k_vp8l_residual out"))
    *o = sub_pixels(px(cur + x), pred);
}

struct InvArgs {
  const uint32_t* modes;
  const uint32_t* in;
  uint32_t* out;
  int* ctl;        // [0] band dequeue counter, [1] error flag (wait timeout)
  int* diag;       // wg::diag_words + DIAG_VP8L_INVERSE
  uint64_t* hand;  // [n_img][bands][width] {pixel, tag} granules of each band's last row
  uint64_t* stamps;  // (WG_TIMELINES builds) [band idx][4]: start, end, poll ticks | polls << 32, block
  int64_t pitch;
  int width, height, bits, tiles_x, tiles_y, bands, n_img;
};

constexpr uint64_t SPIN_TICKS = 200000000ull;  // 2 s of s_memrealtime

// predictorInverseTransform.  Rows depend on the row above (T, TL, TR) and on
// their own left neighbour.  A wave takes a band of 32 rows and walks it as a
// diagonal: at step s the lane pair (2k, 2k + 1) reconstructs pixel
// x = s - 2k of row band*32 + k, lane 2k its blue and red channels and lane
// 2k + 1 its green and alpha ones, each as bytes 0 and 2 of a word (bytes 1
// and 3 zero: the "c2" form).  Per channel the predictors are byte averages
// (v_lerp_u8), 16-bit clamps with no unpacking, and a masked add; only
// Select sums over all four channels, one DPP add with the pair's other
// lane.  (A whole pixel per lane took ~130 instructions a step, most of them
// unpacking and repacking the clamped predictors' 16-bit lanes; the walk is
// issue-bound, one wave alone on its SIMD, so halving the band and the work
// per lane nearly halves the step.)  The row above comes from the lane pair
// before's last three outputs (two whole-wave DPP shifts); the first pair's
// row above is the band above's last row.  Bands are dequeued in (band,
// image) order from a counter, so a band only ever waits on a band owned by
// a running wave.
//
// Hand-off between bands: the band's last row writes its pixels as 8-B
// {pixel, tag} granules, two at a time with one 16-B sc1 (write-through)
// store (MI355X_MICROARCH.md, R2 granules: untorn, no flag, no drain); the
// band below loads one granule a step, UPD = 5 steps before it needs it, and
// re-polls one whose tag is not set yet.  The band below then trails by the
// diagonal's 64 steps plus UPD, a step for the pairing and a store's flight.
//
// The walk runs in chunks of 16 steps, and everything but the predictor and
// the row above is done per chunk: each lane's 16 residuals and tile modes
// (loaded a chunk ahead, one pair per step) and the 16 outputs (the even
// lane of each pair stores the whole pixels as one 64-B run).
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x4a4_t __attribute__((ext_vector_type(4), aligned(4)));  // a row's pixels: 4-B aligned
// steps between a row-above granule's load and its use (round 6, C5's
// inverse: 4 -> 3.41 ms, 5 -> 3.33, 6 -> 3.38, 8 -> 3.50)
constexpr int UPD = 5;
constexpr int INV_ROWS = 32;  // rows per band (a lane pair per row)
constexpr uint32_t C2_EVEN = 0x0c020c00u, C2_ODD = 0x0c030c01u;  // v_perm selectors: a pixel's c2 halves

__device__ __forceinline__ uint32_t c2_of(uint32_t p, uint32_t sel) { return __builtin_amdgcn_perm(0u, p, sel); }
__device__ __forceinline__ uint32_t c2_add(uint32_t a, uint32_t b) { return (a + b) & 0x00ff00ffu; }  // mod 256 per channel
__device__ __forceinline__ uint32_t c2_clamp_full(uint32_t a, uint32_t b, uint32_t c) {
  return as_u(clamp255(as_v2(a) + as_v2(b) - as_v2(c)));
}
__device__ __forceinline__ uint32_t c2_clamp_half(uint32_t avg, uint32_t c) { return as_u(half_step(as_v2(avg), as_v2(c))); }
// The kPredCtl predictor on half pixels (c2 form), with the control word's select
// masks m[b] = (bit b set ? ~0 : 0) read from LDS; `black` is this lane's
// half of ARGB_BLACK.  msel is m ? a : b bitwise: one v_bitop3_b32 (gfx950's
// three-input logic op); as an inline-asm v_bfi_b32 the compiler put an
// s_nop on each side of every select (round 6: C5 inverse 3.53 -> 3.47 ms)
__device__ __forceinline__ uint32_t msel(uint32_t m, uint32_t a, uint32_t b) {
  return (m & a) | (~m & b);
}
struct SelMasks {
  uint32_t m[13];
};
__device__ __forceinline__ uint32_t predict_c2(const SelMasks& k, uint32_t l, uint32_t t, uint32_t tr, uint32_t tl,
                                               uint32_t black) {
  const uint32_t* m = k.m;
  const uint32_t pc = msel(m[3], tl, msel(m[2], tr, t));
  const uint32_t r1 = msel(m[4], tl, tr);
  const uint32_t qc = msel(m[7], msel(m[6], avg2(t, tr), tl), msel(m[6], tr, t));
  const int sad_t = (int)__builtin_amdgcn_sad_u8(t, tl, 0u);
  const uint32_t q = msel(m[5], l, qc);
  const uint32_t p = msel(m[0], avg2(l, r1), msel(m[1], l, pc));
  const uint32_t pavg = avg2(p, q);
  // Select: the channel sums of |L - TL| - |T - TL|, this lane's two plus the pair's other two (quad_perm 1,0,3,2)
  const int pa_half = (int)__builtin_amdgcn_sad_u8(l, tl, 0u) - sad_t;
  const int pa = pa_half + __builtin_amdgcn_update_dpp(0, pa_half, 0xb1, 0xf, 0xf, false);
  uint32_t r = msel(m[8], pa <= 0 ? t : l, pavg);
  r = msel(m[9], c2_clamp_full(l, t, tl), r);
  r = msel(m[10], c2_clamp_half(pavg, tl), r);
  return msel(m[11], black, r);
}
// the value of the lane pair before (lane i <- i - 2, two wave_shr:1); the
// first pair gets the band above's c2 halves (lane 0 `even`, lane 1 `odd`)
__device__ __forceinline__ uint32_t from_pair_above(uint32_t v, uint32_t even, uint32_t odd) {
  const uint32_t s1 = (uint32_t)__builtin_amdgcn_update_dpp((int)odd, (int)v, 0x138, 0xf, 0xf, false);
  return (uint32_t)__builtin_amdgcn_update_dpp((int)even, (int)s1, 0x138, 0xf, 0xf, false);
}

// The control words' select masks, 64 B a row: rows 0-15 kPredCtl[mode],
// then the border rules 16 x = 0 (T), 17 x = 0 on row 0 (black), 18 row 0
// (L); rows 19-37 the same with C_EDGE (x = w - 1).  A step reads its row
// with three 16-B reads and one 4-B read, a step ahead, instead of
// extracting 13 bit masks on the VALU.
constexpr int MROWS = 38;
__device__ __forceinline__ void fill_mtab(uint32_t (*mtab)[16], int tid, int nthreads) {
  for (int i = tid; i < MROWS * 16; i += nthreads) {
    const int row = i >> 4, b = i & 15, id = row % 19;
    const uint32_t ctl = (id < 16 ? kPredCtl[id] : (id == 16 ? kPredCtl[2] : (id == 17 ? kPredCtl[0] : kPredCtl[1]))) |
                         (row >= 19 ? (uint32_t)C_EDGE : 0u);
    mtab[row][b] = b < 13 && ((ctl >> b) & 1) ? ~0u : 0u;
  }
}

// One band's walk.  The row above arrives as {pixel, tag} granules from
// `up_row` (global memory written by the wave of the band above; tag 1 set,
// cleared by the launch's memset); the band's last row leaves the same way
// to `hand_mine`.  (Round 5 measured bands grouped four to a workgroup with
// LDS hand-offs inside the group once more: 3.46 -> 3.71 ms at 4096², as in
// round 4 -- co-resident waves slow each other's steps.)
template <bool TILE16>
__device__ __forceinline__ void inv_band(const InvArgs& a, const uint32_t (*mtab)[16], int band, int img, int lane,
                                         const uint64_t* up_row, uint64_t* hand_mine, int64_t stamp_idx) {
  auto ld_masks = [&](uint32_t row) {
    SelMasks k;
    const uint4 a0 = *reinterpret_cast<const uint4*>(&mtab[row][0]), a1 = *reinterpret_cast<const uint4*>(&mtab[row][4]);
    const uint4 a2 = *reinterpret_cast<const uint4*>(&mtab[row][8]);
    k.m[0] = a0.x, k.m[1] = a0.y, k.m[2] = a0.z, k.m[3] = a0.w;
    k.m[4] = a1.x, k.m[5] = a1.y, k.m[6] = a1.z, k.m[7] = a1.w;
    k.m[8] = a2.x, k.m[9] = a2.y, k.m[10] = a2.z, k.m[11] = a2.w;
    k.m[12] = mtab[row][12];
    return k;
  };
  const int w = a.width;
  const int k = lane >> 1;  // the lane pair's row in the band
  const uint32_t sel = (lane & 1) ? C2_ODD : C2_EVEN;
  const uint32_t black = (lane & 1) ? 0x00ff0000u : 0u;  // ARGB_BLACK's channels (alpha 255)
  {
    const int y = band * INV_ROWS + k;
    const bool live = y < a.height;
    const uint32_t* in = a.in + img * a.pitch;
    uint32_t* out = a.out + img * a.pitch;
    const int last_row = min(INV_ROWS - 1, a.height - 1 - band * INV_ROWS);
    const bool hands_off = band + 1 < a.bands && lane == 2 * last_row;  // the last row's even lane
    const uint32_t* mrow =
        a.modes + (int64_t)img * a.tiles_x * a.tiles_y + (int64_t)(min(y, a.height - 1) >> a.bits) * a.tiles_x;
    const uint32_t* inrow = in + (int64_t)min(y, a.height - 1) * w;
    uint32_t* orow = out + (int64_t)min(y, a.height - 1) * w;
    uint32_t o1 = 0, first = 0;  // this lane's output (c2) at x - 1; at x = 0
    // (WG_BOUNDS) the buffers' extents from the entry point's shapes
    [[maybe_unused]] const int64_t px_n = 4ll * a.n_img * a.pitch, modes_n = 4ll * a.n_img * a.tiles_x * a.tiles_y,
                                   hand_n = 8ll * a.n_img * a.bands * ((w + 1) & ~1);
    // (WG_TIMELINES builds) the per-band timeline: s_memrealtime (100 MHz) at
    // the band's start and end, and the ticks spent re-polling the band above
    WG_IF_TIMELINES(const uint64_t t_band = __builtin_amdgcn_s_memrealtime(); uint64_t poll_ticks = 0, polls = 0;)
    const int steps = w + 2 * last_row;
    // the band above's row, one granule a step: column c sits in gr[c & 15],
    // loaded UPD steps before step c - 1 (where it is TR); up_take re-polls it
    // until its tag is set and returns the pixel
    // (unconditional loads at clamped addresses: a load inside a branch makes
    // the compiler drain every load before its use)
    // (band 0: up_row is any valid row, values unused)
    auto up_load = [&](int c) -> uint64_t {
      const uint64_t* g = up_row + min(c, w - 1);
      return WG_CHK(g, 8, a.hand, hand_n, "k_vp8l_inverse hand load")
                 ? __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                 : 0ull;
    };
    // re-poll column c's granule until its tag is set (band > 0, c < w)
    auto up_poll = [&](int c) -> uint64_t {
      uint64_t g = 0;
      const uint64_t t0 = wg::wait_clock();
      for (uint32_t it = 0;; it++) {
        __builtin_amdgcn_s_sleep(1);
        g = up_load(c);
        if (__builtin_amdgcn_readfirstlane((int)__builtin_bit_cast(uint2, g).y) != 0) {
          WG_IF_TIMELINES(poll_ticks += wg::wait_clock() - t0; polls++;)
          break;
        }
        if ((it & 15) == 15 && (wg::wait_clock() - t0 > SPIN_TICKS ||
                                __hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
          if (lane == 0) {
            __hip_atomic_fetch_or(&a.ctl[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            wg::note_timeout(a.diag, c, (int)(wg::wait_clock() - t0), (int)blockIdx.x, 0, 0, 0);
          }
          break;
        }
      }
      return g;
    };
    // (round 6, also measured: the tag tested by a VALU compare and an
    // exec-mask branch, and the check made every other step for two columns:
    // both slower, 3.53 -> 3.57 ms)
    // The tag word alone goes through one v_readfirstlane and a scalar
    // compare: made opaque first, so the compiler does not fold the test into
    // a 64-bit compare of the whole granule (two v_readfirstlane, a 64-bit
    // v_cmp and the VCC branch hazard on every step of a band that follows
    // another: C5 inverse 3.51 -> 3.39 ms, round 6)
    auto up_take = [&](int c, uint64_t g) -> uint32_t {
      uint32_t tag = __builtin_bit_cast(uint2, g).y;
      asm volatile("" : "+v"(tag));
      if (band > 0 && c < w && __builtin_amdgcn_readfirstlane((int)tag) == 0) g = up_poll(c);
      return band > 0 ? (uint32_t)g : 0u;
    };
    // A chunk's inputs: the residuals of pixels x0 .. x0 + 15 of the lane's
    // row -- four 16-B loads where the chunk lies inside the row, else
    // single loads at clamped addresses (the walk's first and last chunks;
    // only pixels inside the row are used) -- and their tiles' modes: with
    // tiles of >= 16 pixels (TILE16) a chunk touches at most two tiles, t0
    // for u < ub and the next one past it.
    auto ld_res = [&](int x0, uint32_t* r) {
      if (x0 >= 0 && x0 + 15 < w && WG_CHK(inrow + x0, 64, a.in, px_n, "k_vp8l_inverse in")) {
        const u32x4a4_t* p = reinterpret_cast<const u32x4a4_t*>(inrow + x0);
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const u32x4a4_t v = p[j];
          r[4 * j] = v.x;
          r[4 * j + 1] = v.y;
          r[4 * j + 2] = v.z;
          r[4 * j + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const uint32_t* q = inrow + min(max(x0 + u, 0), w - 1);
          r[u] = WG_CHK(q, 4, a.in, px_n, "k_vp8l_inverse in") ? *q : 0u;
        }
      }
    };
    struct Modes {
      uint32_t m[TILE16 ? 2 : 16];
      int ub;
    };
    auto ld_modes = [&](int x0, Modes& m) {
      if constexpr (TILE16) {
        const int t0 = min(max(x0, 0), w - 1) >> a.bits;
        const uint32_t *q0 = mrow + t0, *q1 = mrow + min(t0 + 1, a.tiles_x - 1);
        m.m[0] = WG_CHK(q0, 4, a.modes, modes_n, "k_vp8l_inverse modes") ? *q0 : 0u;
        m.m[1] = WG_CHK(q1, 4, a.modes, modes_n, "k_vp8l_inverse modes") ? *q1 : 0u;
        m.ub = ((t0 + 1) << a.bits) - x0;
      } else {
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const uint32_t* q = mrow + (min(max(x0 + u, 0), w - 1) >> a.bits);
          m.m[u] = WG_CHK(q, 4, a.modes, modes_n, "k_vp8l_inverse modes") ? *q : 0u;
        }
        m.ub = 0;
      }
    };
    uint32_t rc[16];
    Modes mc;
    uint64_t gr[16];
    ld_res(-2 * k, rc);
    ld_modes(-2 * k, mc);
#pragma unroll
    for (int c = 0; c <= UPD; c++) gr[c & 15] = up_load(c);
    // the row above at x and x - 1 (T and TL) of the step, as c2 halves: TR
    // and T of the step before
    const uint32_t cT = up_take(0, gr[0]);
    uint32_t t = c2_of(cT, sel), tl = t;
    for (int s0 = 0; s0 < steps; s0 += 16) {
      const int x0 = s0 - 2 * k;  // this chunk's first pixel in the lane's row
      uint32_t rn[16], ov[16], cc[16];  // cc: the pixels' mask rows
      Modes mn;
      // the chunk's control words (the tile modes arrived a chunk ago), with
      // the reference's border rules: row 0 L (black at x = 0), column 0 T,
      // TR past the right edge is this row's first pixel.  Those apply in the
      // walk's first and last chunks only (x0 <= 0 or x0 + 15 >= w - 1 on
      // some lane of the wave).
      if constexpr (TILE16) {
        const uint32_t k0 = y == 0 ? 18u : (mc.m[0] >> 8) & 0xf, k1 = y == 0 ? 18u : (mc.m[1] >> 8) & 0xf;
#pragma unroll
        for (int u = 0; u < 16; u++) cc[u] = u < mc.ub ? k0 : k1;
      } else {
#pragma unroll
        for (int u = 0; u < 16; u++) cc[u] = y == 0 ? 18u : (mc.m[u] >> 8) & 0xf;
      }
      // (a chunk where x = 0 on some lane: the walk's first ones)
      const bool starts = __builtin_amdgcn_readfirstlane(s0 <= 2 * (INV_ROWS - 1));
      if (starts || __builtin_amdgcn_readfirstlane(s0 + 15 >= w - 1)) {
        const uint32_t kx0 = y == 0 ? 17u : 16u;
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const int x = x0 + u;
          cc[u] = (x == 0 ? kx0 : cc[u]) + (x == w - 1 ? 19u : 0u);
        }
      }
      SelMasks km = ld_masks(cc[0]);
      ld_res(x0 + 16, rn);  // the next chunk's inputs
      ld_modes(x0 + 16, mn);
#pragma unroll
      for (int u = 0; u < 16; u++) {
        const int x = x0 + u;  // steps past the end run idle (x >= w on every lane)
        gr[(u + 1 + UPD) & 15] = up_load(s0 + u + 1 + UPD);
        const uint32_t cTR = up_take(s0 + u + 1, gr[(u + 1) & 15]);
        // row above at x + 1: the pair before's output from its previous
        // step; at x and x - 1 the last two steps' TR
        const uint32_t up_x1 = from_pair_above(o1, c2_of(cTR, C2_EVEN), c2_of(cTR, C2_ODD));
        const SelMasks kn = ld_masks(cc[(u + 1) & 15]);  // the next step's (u = 15: unused)
        const uint32_t tr = msel(km.m[12], first, up_x1);
        const uint32_t v = c2_add(c2_of(rc[u], sel), predict_c2(km, o1, t, tr, tl, black));
        km = kn;
        tl = t;
        t = up_x1;
        // the whole pixel on the pair's even lane (quad_perm 1,1,3,3: the odd lane's half)
        const uint32_t vodd = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xf5, 0xf, 0xf, false);
        const uint32_t full = v | vodd << 8;
        // the hand-off: x has the step's parity (2k is even), so odd steps
        // store the pair (x - 1, x); an odd width's last pixel goes alone
        // (the hand-off lane's row is live)
        if (u & 1) {
          if (hands_off && (uint32_t)x < (uint32_t)w &&
              WG_CHK(hand_mine + x - 1, 16, a.hand, hand_n, "k_vp8l_inverse hand store")) {
            const u32x4_t g2 = {ov[u - 1], 1u, full, 1u};
            // (s_nop: the data VGPRs are read after issue -- see st_sc1_128 in decode.hip)
            asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(hand_mine + x - 1), "v"(g2) : "memory");
          }
        } else if (hands_off && x == w - 1 && WG_CHK(hand_mine + x, 8, a.hand, hand_n, "k_vp8l_inverse hand store")) {
          __hip_atomic_store(hand_mine + x, 1ull << 32 | full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (starts) first = x == 0 ? v : first;
        // (outputs at x outside the row are never read: at x = 0 the row
        // above's TL and the left neighbour are unused, and the pair below
        // reads x = w as TR only where C_EDGE takes `first` instead)
        o1 = v;
        ov[u] = full;
      }
      // this chunk's outputs: pixels x0 .. x0 + 15 of the row, from the even lane
      if ((lane & 1) == 0 && live) {
        if (x0 >= 0 && x0 + 15 < w && WG_CHK(orow + x0, 64, a.out, px_n, "k_vp8l_inverse out")) {
          uint64_t* d = reinterpret_cast<uint64_t*>(orow + x0);
#pragma unroll
          for (int j = 0; j < 8; j++) d[j] = (uint64_t)ov[2 * j + 1] << 32 | ov[2 * j];
        } else {
#pragma unroll
          for (int u = 0; u < 16; u++) {
            const int x = x0 + u;
            if (x >= 0 && x < w && WG_CHK(orow + x, 4, a.out, px_n, "k_vp8l_inverse out")) orow[x] = ov[u];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 16; u++) rc[u] = rn[u];
      mc = mn;
    }
    WG_IF_TIMELINES(if (lane == 0) {
      uint64_t* st = a.stamps + 4 * stamp_idx;
      st[0] = t_band;
      st[1] = __builtin_amdgcn_s_memrealtime();
      st[2] = poll_ticks | polls << 32;
      st[3] = blockIdx.x;
    })
  }
}

// One wave a band, bands dequeued in (band, image) order from a counter (a
// band only ever waits on a band owned by a running wave); every hand-off
// through global memory.
template <bool TILE16>
__global__ __launch_bounds__(64) void k_vp8l_inverse(InvArgs a) {
  __shared__ int sh_band;
  __shared__ uint32_t mtab[MROWS][16];
  const int lane = threadIdx.x;
  fill_mtab(mtab, lane, 64);
  __syncthreads();
  const int total = a.bands * a.n_img;
  const int hs = (a.width + 1) & ~1;  // granules per hand-off row (even: 16-B aligned pairs)
  for (;;) {
    if (lane == 0) sh_band = __hip_atomic_fetch_add(&a.ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int idx = __builtin_amdgcn_readfirstlane(sh_band);
    __syncthreads();
    if (idx >= total) break;
    const int band = idx / a.n_img, img = idx % a.n_img;
    uint64_t* hand_mine = a.hand + ((int64_t)img * a.bands + band) * hs;
    const uint64_t* up_row = band > 0 ? hand_mine - hs : hand_mine;
    inv_band<TILE16>(a, mtab, band, img, lane, up_row, hand_mine, idx);
  }
}

__global__ __launch_bounds__(256) void k_vp8l_green(uint32_t* argb, int64_t n, int add) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = argb[i], g = (p >> 8) & 0xff;
  const uint32_t r = (p >> 16) & 0xff, b = p & 0xff;
  const uint32_t r2 = (add ? r + g : r - g) & 0xff, b2 = (add ? b + g : b - g) & 0xff;
  argb[i] = (p & 0xff00ff00u) | (r2 << 16) | b2;
}

int subsample(int size, int bits) { return (size + (1 << bits) - 1) >> bits; }

}  // namespace

namespace wg {
const double* vp8l_slog2_lut_device();  // vp8l_host.cpp
}

extern "C" int wg_vp8l_residual_image_rows(const uint32_t* argb, int32_t width, int32_t height, int64_t image_pitch,
                                           int32_t bits, int32_t quality, int32_t ty_begin, int32_t ty_end,
                                           int32_t n_images, uint32_t* modes, uint32_t* residuals, void* stream) {
  WG_REQUIRE(argb && modes && residuals && width > 0 && height > 0 && n_images > 0);
  WG_REQUIRE(bits >= 2 && bits <= 9 && image_pitch >= (int64_t)width * height);
  const int tiles_x = subsample(width, bits), tiles_y = subsample(height, bits);
  WG_REQUIRE(ty_begin >= 0 && ty_begin < ty_end && ty_end <= tiles_y);
  WG_REQUIRE(height <= 65535 && n_images <= 65535);  // (k_vp8l_residual's grid y / z)
  const double* lut = wg::vp8l_slog2_lut_device();
  if (!lut) return WG_EHIP;
  hipStream_t s = wg::as_stream(stream);
  SelArgs sa;
  sa.argb = argb;
  sa.pitch = image_pitch;
  sa.modes = modes;
  sa.lut = lut;
  sa.width = width;
  sa.height = height;
  sa.bits = bits;
  sa.tiles_x = tiles_x;
  sa.tiles_y = tiles_y;
  sa.max_mode = quality < 25 ? 4 : (quality < 50 ? 8 : 14);
  sa.ty0 = ty_begin;
  sa.band_tiles = tiles_x * (ty_end - ty_begin);
  const int64_t tiles = (int64_t)sa.band_tiles * n_images;
  WG_REQUIRE(tiles < (1ll << 31));
  int rc;
  if (bits <= 5) {  // counts <= 512: all modes in one pass over the samples
    hipLaunchKernelGGL(k_vp8l_select_q3, dim3((unsigned)tiles), dim3(128), 0, s, sa, tiles);
    rc = wg::check_launch("k_vp8l_select_q3");
  } else {
    hipLaunchKernelGGL(k_vp8l_select, dim3((unsigned)tiles), dim3(64 * SEL_WAVES), 0, s, sa);
    rc = wg::check_launch("k_vp8l_select");
  }
  if (rc != WG_OK) return rc;
  ResArgs ra;
  ra.argb = argb;
  ra.modes = modes;
  ra.out = residuals;
  ra.pitch = image_pitch;
  ra.width = width;
  ra.height = height;
  ra.bits = bits;
  ra.tiles_x = tiles_x;
  ra.tiles_y = tiles_y;
  ra.y0 = ty_begin << bits;
  ra.rows = min(ty_end << bits, height) - ra.y0;
  hipLaunchKernelGGL(k_vp8l_residual, dim3((unsigned)((width + 255) / 256), (unsigned)ra.rows, (unsigned)n_images),
                     dim3(256), 0, s, ra);
  return wg::check_launch("k_vp8l_residual");
}

extern "C" int wg_vp8l_residual_image(const uint32_t* argb, int32_t width, int32_t height, int64_t image_pitch,
                                      int32_t bits, int32_t quality, int32_t n_images, uint32_t* modes,
                                      uint32_t* residuals, void* stream) {
  WG_REQUIRE(width > 0 && height > 0 && bits >= 2 && bits <= 9);
  return wg_vp8l_residual_image_rows(argb, width, height, image_pitch, bits, quality, 0, subsample(height, bits),
                                     n_images, modes, residuals, stream);
}

extern "C" size_t wg_vp8l_inverse_work_bytes(int32_t width, int32_t height, int32_t n_images) {
  if (width <= 0 || height <= 0 || n_images <= 0) return 0;
  const size_t bands = (size_t)n_images * ((height + INV_ROWS - 1) / INV_ROWS);
  return 16 + sizeof(uint64_t) * bands * ((width + 1) & ~1) WG_IF_TIMELINES(+32 * bands);  // (+ the timeline records)
}

extern "C" int wg_vp8l_inverse_predictor(const uint32_t* modes, int32_t bits, int32_t width, int32_t height,
                                         int64_t image_pitch, int32_t n_images, const uint32_t* residuals,
                                         uint32_t* out, void* work, void* stream) {
  WG_REQUIRE(modes && residuals && out && work && width > 0 && height > 0 && n_images > 0);
  WG_REQUIRE(bits >= 2 && bits <= 9 && image_pitch >= (int64_t)width * height);
  WG_REQUIRE(reinterpret_cast<uintptr_t>(work) % 16 == 0);
  hipStream_t s = wg::as_stream(stream);
  InvArgs a;
  a.modes = modes;
  a.in = residuals;
  a.out = out;
  a.bands = (height + INV_ROWS - 1) / INV_ROWS;
  a.n_img = n_images;
  a.ctl = static_cast<int*>(work);
  a.diag = wg::diag_words(s);
  if (!a.diag) return WG_EHIP;
  a.diag += wg::DIAG_VP8L_INVERSE;
  a.hand = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(work) + 16);
  a.stamps = a.hand + (size_t)n_images * a.bands * ((width + 1) & ~1);
  a.pitch = image_pitch;
  a.width = width;
  a.height = height;
  a.bits = bits;
  a.tiles_x = subsample(width, bits);
  a.tiles_y = subsample(height, bits);
  // counters and every granule's tag start clear
  if (hipMemsetAsync(work, 0, wg_vp8l_inverse_work_bytes(width, height, n_images), s) != hipSuccess)
    return wg::check_launch("hipMemsetAsync(vp8l work)");
  const int total = a.bands * n_images;
  const int grid = total < 2048 ? total : 2048;
  if (bits >= 4)
    hipLaunchKernelGGL(k_vp8l_inverse<true>, dim3((unsigned)grid), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(k_vp8l_inverse<false>, dim3((unsigned)grid), dim3(64), 0, s, a);
  return wg::check_launch("k_vp8l_inverse");
}

extern "C" int wg_vp8l_inverse_status(const void* work, void* stream) {
  WG_REQUIRE(work);
  return wg::wait_status(static_cast<const int*>(work) + 1, wg::DIAG_VP8L_INVERSE, wg::as_stream(stream),
                         "wg_vp8l_inverse_status: vp8l inverse band", "step, ticks, block, -, -, -");
}

extern "C" int wg_vp8l_green(uint32_t* argb, int64_t n, int32_t add, void* stream) {
  WG_REQUIRE(argb && n >= 0);
  if (n == 0) return WG_OK;
  hipLaunchKernelGGL(k_vp8l_green, dim3(wg::blocks_for(n, 256)), dim3(256), 0, wg::as_stream(stream), argb, n,
                     add ? 1 : 0);
  return wg::check_launch("k_vp8l_green");
}
