// encode_rd.hip -- the encoder's macroblock RD loop on gfx950 (SURVEY.md
// 8(a) A20): Phase A of encodeFrameParallel (internal/lossy/
// encode_parallel.go:168-1495), methods 3-6 (method 3: plain quantisation instead of the trellis), for whole frames.
//
// Schedule: one persistent launch.  A wave dequeues a
// macroblock ROW from an ordered counter -- in the order of the row schedule
// wg_encode_row_order leaves in the work buffer (textured frames' rows up to
// mbh/4 rows early), always after the row above -- and walks it left to right
// as the reference's encodeRow does.  Row y starts MB x once row y-1 has
// finished MB x and waits for MB x+1 only at I4 step 3, the first read of the
// top-right pixels (the reference waits for x+1 up front, :286-295; the
// outputs are the same).  The shared top arrays (topY/U/V, topModes, topNz,
// topNzDC) become one record of 11 {word, tag} granules per MB column, each
// handed down as one 64-bit atomic store and polled by the row below; the left context stays
// in LDS.  Two workgroup shapes:
//   4-wave workgroups, one wave a row, sharing the cost tables in LDS (batch
//   launches with more rows than twice the pair slots); and
//   PAIR workgroups, two waves a row (launches with few rows, e.g. one
//   frame): wave A imports, builds the context and runs the I4 RD; wave B
//   runs the I16 RD, posts its score (A's early exit reads it), the UV RD, the
//   I16 final residuals speculatively and the chroma residuals; one barrier
//   joins them and A exports.
//
// Inside a macroblock the lanes take the reference's independent loops:
//   I16 RD     lane = (mode, block): 4 x 16 blocks predicted, transformed,
//              quantised, costed and reconstructed at once; contexts from the
//              neighbours' nz; one lane per mode runs the DC WHT path;
//              per-mode sums by DPP reductions
//   UV RD      lane = (mode, plane, block): 4 x 8 blocks
//   I4 RD      the 16 blocks as a wavefront of 10 steps (block (bx, by) at
//              step bx + 2 by; the two blocks of a step one per half-wave);
//              per block lanes 0-9 pre-screen the 10 modes, the candidate
//              pick is the reference's first-argmin on 32-bit keys, and the K
//              candidates run in parallel: transform per lane, trellis prep
//              per (candidate, position pair), the 16-step DP on a lane quad
//              per candidate, reconstruction + TDisto one row per quad lane
//   final      I16 AC blocks trellis-quantised speculatively, three rounds
//              of one DP per (block, initial context it can still get), each
//              followed by the reference's raster-order resolution of the
//              actual contexts; DC and chroma in parallel; then
//              reconstruction and export
// All integer; bit-exact with the C restatement (oracle/lossy_rd.c).
#include <cstdlib>
#include <mutex>

#include "vp8_tables.h"
#include "wg_common.h"
#include "wg_dsp.h"
#include "wg_instr.h"

namespace {

using namespace wg;

constexpr int BPS = 32;
constexpr int YOFF = BPS * 1 + 8;
constexpr int UOFF = YOFF + BPS * 16 + BPS;
constexpr int VOFF = UOFF + 16;
constexpr int YUV = BPS * 17 + BPS * 9;
constexpr int REC = 128;  // per MB column hand-off record: REC_WORDS {word, tag} 8-B granules (88 B used)
constexpr int REC_WORDS = 11;

struct SQuant {  // SegmentQuant (encode.go:311-323); layout = wg_squant
  int32_t quant, iquant, bias, zthresh;
  int32_t dc_quant, dc_iquant, dc_bias, dc_zthresh;
  int16_t sharpen[16];
};
struct Segment {  // = wg_segment
  SQuant y1, y2, uv;
  int32_t lambda_i4, lambda_i16, lambda_uv, lambda_mode;
  int32_t tlambda_i4, tlambda_i16, tlambda_uv, tlambda_sd;
};
static_assert(sizeof(SQuant) == 64 && sizeof(Segment) == 224, "segment layout");

struct MbEnc {  // = wg_mb_enc (MBEncInfo subset)
  int16_t coeffs[400];
  uint8_t modes[16];
  uint8_t nz_y[16];
  uint8_t nz_uv[8];
  uint32_t non_zero_y, non_zero_uv;
  uint8_t mb_type, i16_mode, uv_mode, nz_dc;
  uint8_t skip, segment, pad0, pad1;
  uint64_t score;
};
static_assert(sizeof(MbEnc) == 864, "MbEnc layout");

// zigzag scan as a compile-time table: with the coefficient loops unrolled
// every co[zig] / q[zig] index is a constant (no scratch-memory arrays)
constexpr int kZig[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
constexpr int kBand[17] = {0, 1, 2, 3, 6, 4, 5, 6, 6, 6, 6, 6, 6, 6, 6, 7, 0};
// raster index -> zigzag position (kRZig[kZig[n]] == n); immediates, not
// constant-memory loads (those landed in SGPRs and spilled)
constexpr int kRZig[16] = {0, 1, 5, 6, 2, 4, 7, 12, 3, 8, 11, 13, 9, 10, 14, 15};

constexpr uint64_t pack_zig() {
  uint64_t v = 0;
  for (int n = 0; n < 16; n++) v |= (uint64_t)kZig[n] << (4 * n);
  return v;
}
constexpr uint64_t pack_band() {
  uint64_t v = 0;
  for (int n = 0; n < 17; n++) v |= (uint64_t)kBand[n] << (3 * n);
  return v;
}
// lane-varying scan lookups (a position per lane) without a memory access
__device__ __forceinline__ int zig_of(int n) { return (int)((pack_zig() >> (4 * n)) & 15); }
__device__ __forceinline__ int band_of(int n) { return (int)((pack_band() >> (3 * n)) & 7); }

// One trellis position, prepared by a lane of its own (trellis_prep) and
// consumed by the lane quad running the DP (trellis_dp4).
struct alignas(8) TRec {
  // x[row][pc]: the transition from predecessor context pc, as a key
  // (score x16 + idx, idx = 4 pc + the level code: 0 level 0, 1 L0, 2 L0 + 1)
  // to add to that predecessor's state, with the rows routed by the end
  // context they reach:
  //   R1  level 1 or L0 >= 2: (nz token + level cost) * lam16 + distortion,
  //       idx 4pc + 1 for level L0, 4pc + 2 for level L0 + 1 (= 1 when L0 = 0)
  //   R2  level L0 + 1 >= 2 (idx 4pc + 2), all BIG when L0 = 0
  // + BIG when that level is not a candidate.  The level-0 row R0 (end
  // context 0: zero-token cost * lam16 + idx 4pc) depends only on the
  // position and the segment's lambda: one table per macroblock and phase
  // (Shared::r0, trellis_r0), not a row of every record.
  int64_t x[2][3];
};
static_assert(sizeof(TRec) == 48, "TRec layout");

// two int16 lanes of one word (packed 16-bit arithmetic: v_pk_*_i16 / v_dot2)
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int as_int(s16x2 v) { return __builtin_bit_cast(int, v); }
__device__ __forceinline__ s16x2 as_s16x2(int v) { return __builtin_bit_cast(s16x2, v); }
// two int16 values in one word (low = a)
__device__ __forceinline__ uint32_t pack16(int a, int b) { return (uint32_t)(a & 0xffff) | (uint32_t)b << 16; }
// four coefficients (each fits int16) into an 8-B aligned int16 row piece
__device__ __forceinline__ void st_co4(int16_t* d, const int* c) {
  *reinterpret_cast<uint2*>(d) = make_uint2(pack16(c[0], c[1]), pack16(c[2], c[3]));
}

__constant__ uint16_t c_level_codes[134];
__constant__ uint16_t c_fixed_i4[1000];
__constant__ int32_t c_wtrellis[16];

// ------------------------------------------------------------------ LDS state
// token costs of one (type, band) row, per context 0..2: `zero` = not-EOB +
// zero token, `nz` = not-EOB + non-zero token prefix, `eob` = EOB
// (the bit-cost sums TokenCostForCoeffs / TrellisQuantizeBlock take per
// position, encode_quant.go:154-223, encode_trellis.go:150-230)
struct alignas(16) TokRow {
  uint16_t zero[4], nz[4], eob[4], pad[4];
};
// Table-driven 4x4 intra prediction for lane-varying modes.  Every pixel of
// every PredLuma4 mode (predict_lossy.go:185-424) is one entry of a 64-byte
// per-block value table V built from the 13 context pixels:
//   V[0..14]  edge E = L L K J I X A B C D E F G H H (L and H repeated)
//   V[16+i]   avg2(E[i], E[i+1])          V[32+i]  avg3(E[i-1], E[i], E[i+1])
//   V[47]     the DC value                V[48+p]  the TM value of pixel p
// kPred4Code[mode][pixel] is the V index (checked against pred4_row on
// random contexts by tools-side derivation; pinned on the GPU by the
// encoder parity tests).
constexpr uint8_t kPred4Code[10][16] = {
  {47, 47, 47, 47, 47, 47, 47, 47, 47, 47, 47, 47, 47, 47, 47, 47},
  {48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63},
  {38, 39, 40, 41, 38, 39, 40, 41, 38, 39, 40, 41, 38, 39, 40, 41},
  {36, 36, 36, 36, 35, 35, 35, 35, 34, 34, 34, 34, 33, 33, 33, 33},
  {37, 38, 39, 40, 36, 37, 38, 39, 35, 36, 37, 38, 34, 35, 36, 37},
  {21, 22, 23, 24, 37, 38, 39, 40, 36, 21, 22, 23, 35, 37, 38, 39},
  {39, 40, 41, 42, 40, 41, 42, 43, 41, 42, 43, 44, 42, 43, 44, 45},
  {22, 23, 24, 25, 39, 40, 41, 42, 23, 24, 25, 43, 40, 41, 42, 44},
  {20, 37, 38, 39, 19, 36, 20, 37, 18, 35, 19, 36, 17, 34, 18, 35},
  {19, 35, 18, 34, 18, 34, 17, 33, 17, 33, 1, 1, 1, 1, 1, 1}
};

// Tables shared by the workgroup's waves (filled once per launch)
struct Tables {
  uint8_t proba[4 * 8 * 3 * 11];
  uint16_t ecost[256];
  uint16_t lfixed[2048];
  TokRow tok[4 * 8];
  // token cost of a level for every (type, band), level 0..67 and context,
  // but the level's fixed cost (lfixed): level 0 = not-EOB + zero token,
  // level >= 1 = not-EOB + non-zero token + variableLevelCost (levels past
  // 67 share entry 67; encode_quant.go:170-220, 258-273).  The three
  // contexts of one level sit in one 8-byte word: one ds_read_b64 per
  // position, and a position's cost is vcost[.][min(v, 67)] + lfixed[v]
  // (lfixed[0] = 0) with no select on v == 0
  uint64_t vcost[4 * 8][68];
  uint16_t fixed_i4[1000];
  int wtr[16];  // trellis distortion weights (kWeightTrellis)
  alignas(16) uint8_t pcode[10][16];  // kPred4Code
};
// Per-wave state: each wave of the workgroup encodes its own macroblock row
struct Shared {
  uint8_t yin[YUV], yout[YUV], yout2[YUV];
  alignas(16) int16_t coeffs[400];
  uint8_t mbtail[64];  // wg_mb_enc bytes 800..863, staged so the record leaves in one 16-B-per-lane store
  uint8_t modes4[16];
  uint8_t nzy[16], nzuv[8];
  int mode_rate[4], mode_disto[4], uv_rate[4], uv_disto[4];
  alignas(16) int16_t co_buf[16][16];  // transform coefficients handed to the trellis prep lanes (|c| < 2^12)
  // trellis position records: I4 (half, candidate) / final I16 (block of the
  // round).  Slots 17 records apart (WG_ENC_TPAD): at 16 (768 B, a multiple of
  // the 256-B bank row) the six DP quads' reads of one position all hit the
  // same banks.
// (WG_ENC_NLAST) the DP may stop after the last position of the round at
// which any of its blocks has a non-zero level candidate: past it every state
// but context 0's is invalid, so no terminal (EOB from context 1 / 2) can
// still win and the histories only gain zero levels -- the result is the same
// as walking to position 15, as the reference does.  The walk's length is a
// template bucket (positions < 8 or all 16): a run-time exit made the
// compiler re-roll the loop and wait on every position's loads (slower
// than walking all 16).  Measured (round 5, isolated 64 x 1080p launch, A/B):
// the run-time exit 20.2-20.4 -> 21.2-21.3 ms, the buckets 20.3-20.6 ->
// 20.6-20.7 ms (the second DP copy's registers and code): off.
  // (the final I16 trellis, WG_ENC_I16ONE: the 16 blocks' records of one
  // half of the positions at a time, 9 records apart, and all 16 blocks'
  // level records)
  union {
    TRec trec[6][17];
    TRec trec16[16][9];
  };
  int64_t r0[17][6];       // the phase's level-0 trellis row [0..2] and terminal row [3..5] (trellis_r0)
  int64_t eobl[16][2];     // the phase's terminal costs x lam16 (trellis_r0, WG_ENC_EOBT)
  union {
    int16_t l0s[6][16];    // per position: L0 << 3 | negative << 2 | min(L0, 2) (< 2^14)
    int16_t l0s16[16][16];
  };
  alignas(16) int16_t cand_q[6][16];  // I4 candidates' levels for the lane-parallel token cost
  int cand_nz[6], cand_rate[6];
  alignas(16) uint8_t pv[2][64];  // per half-wave: the I4 block's prediction value table
  int word;
  // pair mode (k_encode_rows<., true>): the I4 wave (A) hands the MB's
  // neighbour context to the I16 / chroma wave (B) in ctxw; B posts the I16
  // score for A's early exit (s16v, then s16_flag) and its results (post_*)
  uint32_t ctxw[4];  // top_nz, top_nz_dc, left_nz, left_nz_dc
  int s16_flag, post_best16, post_best_uv, post_nz_dc;
  uint64_t s16v, post_s16;
};
constexpr int WAVES = 4;  // rows per band: the waves of a group (one wave a row)
// Groups (bands in flight) per workgroup.  3 = 12-wave workgroups, one per
// CU, three waves per SIMD (149 VGPRs, 161 KB of LDS): measured slower in the
// bench than two 4-wave workgroups per CU ("Three waves per SIMD"),
// so 1 is the default.
constexpr int GROUPS = 1;

__device__ __forceinline__ int ecost(const Tables& t, int p) { return t.ecost[p]; }
__device__ __forceinline__ int bit_cost(const Tables& t, int bit, int p) { return t.ecost[bit ? 255 - p : p]; }
__device__ __forceinline__ const uint8_t* proba_p(const Tables& t, int type, int band, int ctx) {
  return t.proba + ((type * 8 + band) * 3 + ctx) * 11;
}
__device__ __forceinline__ int pick3(int c, int a0, int a1, int a2) { return c == 0 ? a0 : (c == 1 ? a1 : a2); }
__device__ __forceinline__ int vc_of(uint64_t w, int c) { return (int)((w >> (16 * c)) & 0xffff); }

// QuantizeCoeffs (encode_quant.go:16-80): returns the zigzag nz count
__device__ __forceinline__ int quantize(const int co[16], int16_t q[16], const SQuant& sq, int first) {
  int max_zz = -1;
  // the quantiser as four 16-byte LDS reads (SQuant is 64 B, 16-B aligned)
  const uint4 h0 = *reinterpret_cast<const uint4*>(&sq.quant);     // quant iquant bias zthresh
  const uint4 h1 = *reinterpret_cast<const uint4*>(&sq.dc_quant);  // the DC ones
  const uint4 s0 = *reinterpret_cast<const uint4*>(&sq.sharpen[0]), s1 = *reinterpret_cast<const uint4*>(&sq.sharpen[8]);
  const uint32_t sw[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
  for (int n = 0; n < 16; n++) {
    if (n < first) {
      q[n] = 0;
      continue;
    }
    int v = co[n];
    const int sign = v < 0 ? -1 : 1;
    v = abs(v) + (int)(int16_t)(sw[n >> 1] >> (16 * (n & 1)));
    v = max(v, 0);
    const uint32_t iq = n == 0 ? h1.y : h0.y;
    const uint32_t bias = n == 0 ? h1.z : h0.z;
    // (v < 2^16 and iq <= 2^15: the full-rate 24-bit multiplier is exact)
    const int c = min((int)(((uint32_t)wg::mul_i24(v, (int)iq) + bias) >> 17), 2047);
    q[n] = (int16_t)(sign * c);
    if (c != 0) max_zz = max(max_zz, kRZig[n]);
  }
  return max_zz + 1;
}

// 16 levels packed two per VGPR (int16 arrays otherwise take one VGPR each)
struct Q16 {
  uint32_t w[8];
  __device__ __forceinline__ int get(int i) const { return (int)(int16_t)(w[i >> 1] >> (16 * (i & 1))); }
};
__device__ __forceinline__ int quantize(const int co[16], Q16& q, const SQuant& sq, int first) {
  int16_t t[16];
  const int nz = quantize(co, t, sq, first);
#pragma unroll
  for (int i = 0; i < 8; i++) q.w[i] = (uint32_t)(uint16_t)t[2 * i] | (uint32_t)(uint16_t)t[2 * i + 1] << 16;
  return nz;
}

__device__ __forceinline__ int variable_level_cost(const Tables& t, int level, const uint8_t* p) {
  const int idx = min(level - 1, 66);
  int pattern = c_level_codes[2 * idx], bits = c_level_codes[2 * idx + 1], cost = 0;
  for (int i = 2; pattern != 0; i++) {
    if (pattern & 1) cost += bit_cost(t, bits & 1, p[i]);
    bits >>= 1;
    pattern >>= 1;
  }
  return cost;
}

// TokenCostForCoeffs (encode_quant.go:154-223), branch-free: the context of
// every position follows from the levels alone (min(|q|, 2) of the previous
// one), so all table reads are independent and issue back to back.
__device__ __forceinline__ int lvl_at(const int16_t* q, int i) { return q[i]; }
__device__ __forceinline__ int lvl_at(const Q16& q, int i) { return q.get(i); }
template <typename QT>
__device__ __forceinline__ int token_cost(const Tables& t, const QT& q, int nz_count, int type, int ctx0, int first) {
  int cost = 0, ctx = ctx0, ctx_eob = ctx0;
  const int eob_at = max(nz_count, first);
#pragma unroll
  for (int n = 0; n < 16; n++) {
    if (n < first) continue;
    const int v = abs(lvl_at(q, kZig[n]));
    const int tokc = vc_of(t.vcost[type * 8 + kBand[n]][min(v, 67)], ctx) + t.lfixed[min(v, 2047)];
    cost += n < nz_count ? tokc : 0;
    ctx_eob = n == eob_at ? ctx : ctx_eob;
    ctx = min(v, 2);
  }
  // EOB at position eob_at (none after position 15)
  if (eob_at < 16) cost += t.tok[type * 8 + band_of(eob_at)].eob[ctx_eob];
  return cost;
}

// TrellisQuantizeBlock (encode_trellis.go:23-301), split across lanes.
//
// Scores are kept x16 so the low 4 bits of a 64-bit key can carry the
// candidate's position in the reference's update order; "first strict
// minimum in order" then is a plain min over keys.  Candidates per position
// and end context: level 0 from predecessor pc (key idx = 4pc, end ctx 0),
// level L0 (idx 4pc + 1) and L0 + 1 (idx 4pc + 2), whose end context is
// min(level, 2): idx grows in the reference's update order, and its low two
// bits are the level code the DP's histories keep.  Invalid states carry scores >= 2^58 (valid ones stay below
// 2^51), so they never win against a valid candidate.  The path keeps the
// winning idx per end context (4 bits each, 16 bits per position); levels
// are re-derived from the position records when walking back.
//
// ---- TrellisQuantizeBlock split across lanes ----------------------------
// Everything a trellis position needs that does not depend on the DP state
// (level candidates, distortion deltas, token + level costs per predecessor
// context) is computed by one lane per position into a TRec; the lane that
// runs the serial DP then does only the 3 x 3 transitions per position.
// R0, the level-0 row, is the same for every block of a phase
// (trellis_r0).
//
// The R0 table of a phase: position n, predecessor context pc -> the
// zero-token cost of band(n + 1) * lam16 + idx 4pc; lane 3n + pc writes it.
// (WG_ENC_TWO, needs WG_ENC_EOBT) class-2 positions (L0 >= 2, both non-zero
// levels end in context 2) are folded into the records: R1 = BIG, R2 =
// min(R1, R2) per predecessor (the keys of L0 and L0 + 1 differ in their idx
// bit, so the min is the reference's first strict minimum), and the DP keeps
// no class test: every lane's own minimum is its context's new state

// (WG_ENC_EOBT) lanes 48 + n also write the phase's terminal costs: EOB after
// position n from end context 1 / 2, x lam16 (0 after position 15), plus n
// (the key's position field, see trellis_dp4), which the DP adds to a state
// instead of multiplying the EOB cost per position.
template <int CTX_TYPE>
__device__ __forceinline__ void trellis_r0(const Tables& t, int lane, int lam16, int64_t (*r0)[6],
                                           int64_t (*eobl)[2]) {
  if (lane < 48) {
    const int n = lane / 3, pc = lane - 3 * n;
    r0[n][pc] = (int64_t)vc_of(t.vcost[CTX_TYPE * 8 + band_of(n + 1)][0], pc) * lam16 + 4 * pc;
  }
  else {
    const int n = lane - 48;
    const TokRow& tr = t.tok[CTX_TYPE * 8 + band_of(n + 1)];
    eobl[n][0] = (n < 15 ? (int64_t)tr.eob[1] * lam16 : 0) + n;
    eobl[n][1] = (n < 15 ? (int64_t)tr.eob[2] * lam16 : 0) + n;
    // the terminal lane's row of step n + 1 (trellis_dp4t): {0, EOB after
    // position n from context 1, from context 2}; none before the walk's
    // first position (FIRST: 0 for the I4 blocks, 1 for the I16 AC blocks)
    constexpr int64_t BIG = 1ll << 59;
    constexpr int FIRST = CTX_TYPE == 0 ? 1 : 0;
    const bool none = n + 1 == FIRST;
    r0[n + 1][3] = 0;
    r0[n + 1][4] = none ? BIG : (n < 15 ? (int64_t)tr.eob[1] * lam16 : 0);
    r0[n + 1][5] = none ? BIG : (n < 15 ? (int64_t)tr.eob[2] * lam16 : 0);
    if (n == 0) {
      r0[0][3] = 0;
      r0[0][4] = BIG;
      r0[0][5] = BIG;
    }
  }
}

// The level candidates, distortion deltas and token + level costs of two
// positions of one block at once (returns whether either has a non-zero
// level under the neutral bias: the reference's all-zero pre-scan), with the table reads
// in two rounds: everything that depends on the position only (the
// coefficient, sharpening, quantiser, distortion weight),
// then the level costs of L0 and L0 + 1.  The scheduling barriers keep each
// round's reads issued together (left to itself the compiler waited on each
// read before issuing the next: eight LDS round trips per lane instead of two).
// Positions below FIRST (the I16 AC blocks' DC) take a zero coefficient and
// report no level.
template <int CTX_TYPE, int FIRST>
__device__ __forceinline__ bool trellis_prep2(const Tables& t, const int16_t* co, int n0, const SQuant& sq, int lam16,
                                              TRec out[2], int l0s[2]) {
  constexpr int64_t BIG = 1ll << 59;
  int co_z[2], sh[2], quant[2], iquant[2], w4096[2];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const int n = n0 + j, zig = zig_of(n);
    co_z[j] = n >= FIRST ? co[zig] : 0;
    sh[j] = sq.sharpen[zig];
    quant[j] = n == 0 ? sq.dc_quant : sq.quant;
    iquant[j] = n == 0 ? sq.dc_iquant : sq.iquant;
    w4096[j] = t.wtr[zig];
  }
  __builtin_amdgcn_sched_barrier(0);
  int c0[2], L0raw[2], L0[2], thresh[2], lf0[2], lf1[2];
  uint64_t v0[2], v1[2];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    c0[j] = max(abs(co_z[j]) + sh[j], 0);
    // (c0 < 2^13, iquant <= 2^15: exact on the full-rate 24-bit multiplier)
    L0raw[j] = (int)((uint32_t)wg::mul_i24(c0[j], iquant[j]) >> 17);
    L0[j] = min(L0raw[j], 2047);
    thresh[j] = min((int)(((uint32_t)wg::mul_i24(c0[j], iquant[j]) + 65536u) >> 17), 2047);
    const int band = band_of(n0 + j + 1);
    lf0[j] = t.lfixed[L0[j]];
    lf1[j] = t.lfixed[min(L0[j] + 1, 2047)];
    v0[j] = t.vcost[CTX_TYPE * 8 + band][min(L0[j], 67)];
    v1[j] = t.vcost[CTX_TYPE * 8 + band][min(L0[j] + 1, 67)];
  }
  __builtin_amdgcn_sched_barrier(0);
  bool pnz = false;
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const bool has0 = L0[j] > 0 && L0[j] <= thresh[j];
    const bool has1 = L0[j] + 1 <= 2047 && L0[j] + 1 <= thresh[j];
    const int w = w4096[j] * 4096;
    const int e0 = c0[j] - wg::mul_i24(L0[j], quant[j]), e1 = e0 - quant[j];
    const int c2 = wg::mul_i24(c0[j], c0[j]);
    const int64_t A0 = (int64_t)lf0[j] * lam16 + (int64_t)w * (wg::mul_i24(e0, e0) - c2) + (has0 ? 0 : BIG);
    const int64_t A1 = (int64_t)lf1[j] * lam16 + (int64_t)w * (wg::mul_i24(e1, e1) - c2) + (has1 ? 0 : BIG);
    const bool z = L0[j] == 0;
    const bool two = L0[j] >= 2;
#pragma unroll
    for (int pc = 0; pc < 3; pc++) {
      const int64_t r1 = (int64_t)vc_of(v0[j], pc) * lam16 + A0 + 4 * pc + 1;
      const int64_t r2 = (int64_t)vc_of(v1[j], pc) * lam16 + A1 + 4 * pc + 2;
      out[j].x[0][pc] = z ? r2 : (two ? BIG : r1);
      out[j].x[1][pc] = z ? BIG : (two && r1 < r2 ? r1 : r2);
    }
    l0s[j] = L0[j] << 3 | (co_z[j] < 0 ? 4 : 0) | min(L0[j], 2);
    pnz |= L0raw[j] > 0 && n0 + j >= FIRST;
  }
  return pnz;
}

// 64-bit value of lane j of this lane's quad (DPP quad_perm broadcast)
template <int J>
__device__ __forceinline__ int64_t quad_bcast(int64_t v) {
  constexpr int perm = J | J << 2 | J << 4 | J << 6;
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, perm, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)((uint64_t)v >> 32), perm, 0xf, 0xf, false);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// 4 x 4 transpose across a lane quad: lane r holds row r (v[c] = M[r][c])
// and gets column r (v[k] = M[k][r]): two exchange stages, with the lane
// r ^ 1 then r ^ 2, of the elements whose index differs from r in that bit
template <int X>
__device__ __forceinline__ void quad_xstage(int v[4]) {
  constexpr int perm = X == 1 ? 0xB1 : 0x4E;  // quad_perm [1,0,3,2] / [2,3,0,1]
  const int r = __lane_id() & 3;
  int t[4];
#pragma unroll
  for (int c = 0; c < 4; c++) t[c] = __builtin_amdgcn_mov_dpp(v[c ^ X], perm, 0xf, 0xf, false);
#pragma unroll
  for (int c = 0; c < 4; c++) v[c] = ((c ^ r) & X) ? t[c] : v[c];
}
__device__ __forceinline__ void quad_transpose(int v[4]) {
  quad_xstage<1>(v);
  quad_xstage<2>(v);
}
// sum over the 4 lanes of a quad, in every lane of it
__device__ __forceinline__ int quad_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  return v;
}
template <int J>
__device__ __forceinline__ int quad_bcast32(int v) {
  return __builtin_amdgcn_mov_dpp(v, J | J << 2 | J << 4 | J << 6, 0xf, 0xf, false);
}

// (WG_ENC_DPPADD) c_j = (lane j of this lane's quad's s) + x_j, j = 0, 1, 2,
// 64-bit: the quad broadcasts fused into the adds' DPP source operand (two
// VOP2 DPP adds each, instead of two v_mov_dpp and two adds).  NOP: the
// wait states before the first DPP read of s (2 after a VALU write of it,
// 5 after an EXEC write: the walks' first position takes 5).
// (T3: lane 3 adds its OWN value to x0 -- quad_perm [0,0,0,3] -- the
// terminal lane of trellis_dp4t)
template <int NOP, bool T3 = false>
__device__ __forceinline__ void quad_bcast_add3(int64_t s, int64_t x0, int64_t x1, int64_t x2, int64_t& c0,
                                                int64_t& c1, int64_t& c2) {
  static_assert(NOP == 1 || NOP == 4, "s_nop count");
  uint32_t a0, b0, a1, b1, a2, b2;
  if constexpr (T3)
    asm volatile(
        "s_nop %c14\n\t"
        "v_add_co_u32_dpp %0, vcc, %6, %8 quad_perm:[0,0,0,3] row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32_dpp %1, vcc, %7, %9, vcc quad_perm:[0,0,0,3] row_mask:0xf bank_mask:0xf\n\t"
        "v_add_co_u32_dpp %2, vcc, %6, %10 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32_dpp %3, vcc, %7, %11, vcc quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_add_co_u32_dpp %4, vcc, %6, %12 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32_dpp %5, vcc, %7, %13, vcc quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf"
        : "=&v"(a0), "=&v"(b0), "=&v"(a1), "=&v"(b1), "=&v"(a2), "=&v"(b2)
        : "v"((uint32_t)s), "v"((uint32_t)((uint64_t)s >> 32)), "v"((uint32_t)x0), "v"((uint32_t)((uint64_t)x0 >> 32)),
          "v"((uint32_t)x1), "v"((uint32_t)((uint64_t)x1 >> 32)), "v"((uint32_t)x2), "v"((uint32_t)((uint64_t)x2 >> 32)),
          "i"(NOP)
        : "vcc");
  else
  asm volatile(
      "s_nop %c14\n\t"
      "v_add_co_u32_dpp %0, vcc, %6, %8 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t"
      "v_addc_co_u32_dpp %1, vcc, %7, %9, vcc quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t"
      "v_add_co_u32_dpp %2, vcc, %6, %10 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t"
      "v_addc_co_u32_dpp %3, vcc, %7, %11, vcc quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t"
      "v_add_co_u32_dpp %4, vcc, %6, %12 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_addc_co_u32_dpp %5, vcc, %7, %13, vcc quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf"
      : "=&v"(a0), "=&v"(b0), "=&v"(a1), "=&v"(b1), "=&v"(a2), "=&v"(b2)
      : "v"((uint32_t)s), "v"((uint32_t)((uint64_t)s >> 32)), "v"((uint32_t)x0), "v"((uint32_t)((uint64_t)x0 >> 32)),
        "v"((uint32_t)x1), "v"((uint32_t)((uint64_t)x1 >> 32)), "v"((uint32_t)x2), "v"((uint32_t)((uint64_t)x2 >> 32)),
        "i"(NOP)
      : "vcc");
  c0 = (int64_t)((uint64_t)b0 << 32 | a0);
  c1 = (int64_t)((uint64_t)b1 << 32 | a1);
  c2 = (int64_t)((uint64_t)b2 << 32 | a2);
}

// The trellis DP on a quad of lanes.  trellis_prep routes the transitions
// by the end context they reach (TRec rows R0 / R1 / R2), so lane k of the
// quad (e = min(k, 2); lane 3 shadows lane 2) takes the minimum of the three
// predecessor states plus its row: keys are score x16 + the candidate's index
// in the reference's update order, so the first strict minimum of
// encode_trellis.go:215-245 is a plain min and the keys of one end context
// never tie.  The three minima reach every lane by DPP broadcasts; where L0 >= 2
// both non-zero levels end in context 2, which then takes min(R1, R2) and
// context 1 is empty.
//
// Instead of a path table walked back from the best terminal, every state
// carries its own history: 2 bits per position (0 = level 0, 1 = L0,
// 2 = L0 + 1), copied from the winning predecessor.  The best terminal
// (EOB after position n from context 1 or 2, :257-270) keeps the history it
// ended, and the levels then follow position by position with no serial
// chain: the quad's lane r writes positions 4r..4r+3 (raster) to q, and lane
// 0 writes the zigzag nz count to *nz.
template <int CTX_TYPE>
__device__ __forceinline__ void trellis_levels(const Tables& t, uint32_t hist, int k, uint2 l0w, int l0prev, int init_ctx,
                                               int16_t* q, int* nz, int* rate);
// Lane 3 of the quad is the best terminal (rather than a shadow of lane 2
// with every lane keeping a best-terminal key and its history, a 64-bit add,
// compare and three selects a position): at step n it takes the
// same three-way minimum as the context lanes, over its own previous value
// (DPP quad_perm [0,0,0,3]: lane 3 reads itself) and the context-1 / -2
// states after position n - 1 plus their EOB costs, its row {0, EOB1, EOB2}
// of step n in the phase's R0 table (columns 3..5, trellis_r0), so the
// terminal costs no instruction of its own; one step past the last position
// takes the EOB after it.  The keys of its row carry no position bits: ties
// keep the earlier terminal (strict compares, the previous value first) and
// context 1 before context 2 at one position (c1 before c2), the
// reference's first strict minimum; its low bits stay 0, so its "level
// code" is 0 and its history is the winner's as is.
template <int FIRST, int CTX_TYPE>
__device__ __forceinline__ void trellis_dp4t(const Tables& t, const TRec* rec, const int64_t (*r0)[6],
                                             const int16_t* l0s, int init_ctx, int lam16, int k, int16_t* q, int* nz,
                                             int* rate = nullptr) {
  constexpr int64_t BIG = 1ll << 59;
  init_ctx = min(init_ctx, 2);
  const TokRow& t_init = t.tok[CTX_TYPE * 8 + FIRST];  // kBand[0] = 0, kBand[1] = 1
  // lanes 0..2: context k's state; lane 3: the best terminal (the all-zero block to start)
  int64_t st = k == 3 ? (int64_t)pick3(init_ctx, t_init.eob[0], t_init.eob[1], t_init.eob[2]) * lam16
                      : (k == init_ctx ? 0 : BIG);
  uint32_t h0 = 0, h1 = 0, h2 = 0, hm = 0;
  const int64_t* mine = k == 3 ? &r0[0][3] : (k == 0 ? &r0[0][0] : &rec[0].x[k - 1][0]);
  constexpr int STRIDE = (int)(sizeof(TRec) / sizeof(int64_t));
  const uint2 l0w = *reinterpret_cast<const uint2*>(l0s + 4 * k);
  const int l0prev = l0s[max(4 * k - 1, 0)];
  int64_t x0 = mine[FIRST * STRIDE], x1 = mine[FIRST * STRIDE + 1], x2 = mine[FIRST * STRIDE + 2];
#pragma unroll
  for (int n = FIRST; n <= 16; n++) {  // (step 16: the terminal lane only)
    int64_t nx0 = 0, nx1 = 0, nx2 = 0;
    if (n + 1 <= 16) {
      nx0 = mine[(n + 1) * STRIDE];
      nx1 = mine[(n + 1) * STRIDE + 1];
      nx2 = mine[(n + 1) * STRIDE + 2];
    }
    asm volatile("" : "+v"(st)::"memory");
    int64_t c0, c1, c2;
    if (n == FIRST) quad_bcast_add3<4, true>(st, x0, x1, x2, c0, c1, c2);
    else quad_bcast_add3<1, true>(st, x0, x1, x2, c0, c1, c2);
    x0 = nx0;
    x1 = nx1;
    x2 = nx2;
    const bool lt1 = c1 < c0;
    const int64_t m01 = lt1 ? c1 : c0;
    const bool lt2 = c2 < m01;
    const int64_t m = lt2 ? c2 : m01;
    const uint32_t hsel = lt2 ? h2 : (lt1 ? h1 : h0);
    hm = n < 16 ? hsel | ((uint32_t)m & 3) << (2 * (n & 15)) : hsel;
    st = m & ~15ll;
    h0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)hm, 0xC0, 0xf, 0xf, false);  // quad_perm [0,0,0,3]
    h1 = quad_bcast32<1>(hm);
    h2 = quad_bcast32<2>(hm);
  }
  trellis_levels<CTX_TYPE>(t, quad_bcast32<3>(hm), k, l0w, l0prev, init_ctx, q, nz, rate);
}

// The chosen levels from the winning history (2 bits a position): the quad's
// lane r writes positions 4r..4r+3 (raster) to q, every lane gets the zigzag
// nz count in *nz and, with `rate`, the block's token cost (FIRST 0 only).
template <int CTX_TYPE>
__device__ __forceinline__ void trellis_levels(const Tables& t, uint32_t hist, int k, uint2 l0w, int l0prev, int init_ctx,
                                               int16_t* q, int* nz, int* rate) {
  // lane r: positions 4r .. 4r + 3
  const int r = k;
  const uint32_t nzb = (hist | hist >> 1) & 0x55555555u;
  const int nzc = nzb == 0 ? 0 : ((31 - __builtin_clz(nzb)) >> 1) + 1;
  int mags[5];
  {  // (the level before position 4r: the context of 4r's token)
    const int n = max(4 * r - 1, 0);
    const int code = r == 0 ? 0 : (int)((hist >> (2 * n)) & 3);
    mags[0] = code == 0 ? 0 : (l0prev >> 3) + code - 1;
  }
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int n = 4 * r + j;
    const int code = (int)((hist >> (2 * n)) & 3);
    const int ls = (int)(((j < 2 ? l0w.x : l0w.y) >> (16 * (j & 1))) & 0xffff);  // (l0s values are < 2^14)
    const int mag = code == 0 ? 0 : (ls >> 3) + code - 1;
    mags[j + 1] = mag;
    q[zig_of(n)] = (int16_t)((ls & 4) ? -mag : mag);
  }
  *nz = nzc;  // (every lane of the quad: the callers pass registers)
  if (rate) {
    // TokenCostForCoeffs (encode_quant.go:154-223) of the chosen levels, lane r
    // taking positions 4r .. 4r + 3 (FIRST 0 only: the I4 blocks), summed over
    // the quad: the candidate's rate with no LDS round trip for its levels
    int part = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int n = 4 * r + j, v = mags[j + 1];
      const int ctx = n == 0 ? init_ctx : min(mags[j], 2);
      const int band = band_of(n);
      const int tokc = vc_of(t.vcost[CTX_TYPE * 8 + band][min(v, 67)], ctx) + t.lfixed[min(v, 2047)];
      const int eobc = t.tok[CTX_TYPE * 8 + band].eob[ctx];
      part += n < nzc ? tokc : (n == nzc ? eobc : 0);
    }
    part = quad_sum(part);
    *rate = part;  // (the quad's sum, in every lane)
  }
}

// The I16 AC blocks' trellis for all three start contexts at once
// (WG_ENC_I16ONE).  A block's start context enters the DP only as its initial
// state, so the three DPs of trellis_dp4 share every record and terminal
// load: the quad carries three independent state sets (start s: context
// states ps[s][], histories h[s][], best terminal bt[s] / bh[s]), each
// updated exactly as trellis_dp4 updates its one (same keys, same compares,
// WG_ENC_TWO / EOBT records), so start s's result is trellis_dp4's for
// init_ctx s.  Walked in two halves (positions [NB, NE)), the records of
// the half at `mine` (`mine[n * STRIDE]` = this lane's row at position n).
// (WG_ENC_TLANE: lane 3 of the quad is each start's best terminal, as in
// trellis_dp4t: its row is the phase table's columns 3..5, one step past the
// last position takes the EOB after it)
struct DP3 {
  int64_t st[3];     // [start]: lanes 0..2 context k's state, lane 3 the best terminal
  uint32_t h[3][3];  // [start][j]: lane j's history (lane 3 reads its own as j = 0)
};
__device__ __forceinline__ void dp3_init(DP3& S, const Tables& t, int lam16, int k) {
  constexpr int64_t BIG = 1ll << 59;
  const TokRow& t_init = t.tok[1];  // type 0, kBand[1] = 1
#pragma unroll
  for (int s = 0; s < 3; s++) {
    S.st[s] = k == 3 ? (int64_t)t_init.eob[s] * lam16 : (k == s ? 0 : BIG);
#pragma unroll
    for (int c = 0; c < 3; c++) S.h[s][c] = 0;
  }
}
template <int NB, int NE>
__device__ __forceinline__ void dp3_walk(DP3& S, const int64_t* mine, const int64_t*) {
  constexpr int STRIDE = (int)(sizeof(TRec) / sizeof(int64_t));
  int64_t x0 = mine[NB * STRIDE], x1 = mine[NB * STRIDE + 1], x2 = mine[NB * STRIDE + 2];
#pragma unroll
  for (int n = NB; n < NE; n++) {  // (step 16: the terminal lane only)
    int64_t nx0 = 0, nx1 = 0, nx2 = 0;
    if (n + 1 < NE) {
      nx0 = mine[(n + 1) * STRIDE];
      nx1 = mine[(n + 1) * STRIDE + 1];
      nx2 = mine[(n + 1) * STRIDE + 2];
    }
    asm volatile("" : "+v"(S.st[0]), "+v"(S.st[1]), "+v"(S.st[2])::"memory");
#pragma unroll
    for (int s = 0; s < 3; s++) {
      int64_t c0, c1, c2;
      if (n == NB && s == 0) quad_bcast_add3<4, true>(S.st[s], x0, x1, x2, c0, c1, c2);
      else quad_bcast_add3<1, true>(S.st[s], x0, x1, x2, c0, c1, c2);
      const bool lt1 = c1 < c0;
      const int64_t m01 = lt1 ? c1 : c0;
      const bool lt2 = c2 < m01;
      const int64_t m = lt2 ? c2 : m01;
      const uint32_t hv0 = S.h[s][0], hv1 = S.h[s][1], hv2 = S.h[s][2];  // (values: see below)
      const uint32_t hsel = lt2 ? hv2 : (lt1 ? hv1 : hv0);
      const uint32_t hm = n < 16 ? hsel | ((uint32_t)m & 3) << (2 * (n & 15)) : hsel;
      S.st[s] = m & ~15ll;
      S.h[s][0] = (uint32_t)__builtin_amdgcn_mov_dpp((int)hm, 0xC0, 0xf, 0xf, false);  // quad_perm [0,0,0,3]
      S.h[s][1] = quad_bcast32<1>(hm);
      S.h[s][2] = quad_bcast32<2>(hm);
    }
    x0 = nx0;
    x1 = nx1;
    x2 = nx2;
  }
}
// start s's chosen history: the terminal lane's
__device__ __forceinline__ uint32_t dp3_hist(const DP3& S, int s) {
  const uint32_t g0 = S.h[0][0], g1 = S.h[1][0], g2 = S.h[2][0];
  return quad_bcast32<3>(s == 0 ? g0 : (s == 1 ? g1 : g2));
}
__device__ __forceinline__ int hist_nz(uint32_t hist) {
  const uint32_t nzb = (hist | hist >> 1) & 0x55555555u;
  return nzb == 0 ? 0 : ((31 - __builtin_clz(nzb)) >> 1) + 1;
}

// TokenCostForCoeffs's term for position n alone (lane-parallel form of
// token_cost(); the caller sums over n).  q: raster levels in LDS.
template <int TYPE>
__device__ __forceinline__ int token_cost_pos(const Tables& t, const int16_t* q, int n, int nz_count, int ctx0, int first) {
  if (n < first) return 0;
  const int band = band_of(n);
  const int v = abs((int)q[zig_of(n)]);
  const int ctx = n == first ? ctx0 : min(abs((int)q[zig_of(max(n - 1, 0))]), 2);
  if (n < nz_count) return vc_of(t.vcost[TYPE * 8 + band][min(v, 67)], ctx) + t.lfixed[min(v, 2047)];
  return n == max(nz_count, first) ? t.tok[TYPE * 8 + band].eob[ctx] : 0;
}

template <int WIDTH>
__device__ __forceinline__ int group_sum_first(int v);
// ---- the I16 DC path (Walsh-Hadamard, quantise, cost, dequantise, inverse)
// lane-parallel over a 16-lane DPP row: lane b holds coefficient b (raster)
// of one 4x4 DC block.  Every WHT pass is four butterflies whose outputs are
// +-sums of four inputs; kWhtSign[p] gives the signs (bit k: input k
// negative) of output pattern p for the row and column passes of both
// transforms (transforms.go:500-531 forward, :232-252 inverse).
constexpr uint32_t kWhtSign[4] = {0x0, 0xC, 0x6, 0xA};
__device__ __forceinline__ int sum4_signed(const int v[4], uint32_t m) {
  return (m & 1 ? -v[0] : v[0]) + (m & 2 ? -v[1] : v[1]) + (m & 4 ? -v[2] : v[2]) + (m & 8 ? -v[3] : v[3]);
}
// the lane's quad (lanes 4r..4r+3 of the row): q[m] = value of lane 4r + m
__device__ __forceinline__ void quad4(int v, int q[4]) {
  q[0] = quad_bcast32<0>(v);
  q[1] = quad_bcast32<1>(v);
  q[2] = quad_bcast32<2>(v);
  q[3] = quad_bcast32<3>(v);
}
// the lane's column (lanes c, 4 + c, 8 + c, 12 + c), rotated: v4[d] = value of
// lane (b + 4d) & 15, i.e. of row (r + d) & 3
__device__ __forceinline__ void col4(int v, int v4[4]) {
  v4[0] = v;
  v4[1] = __builtin_amdgcn_update_dpp(0, v, 0x12C, 0xf, 0xf, false);  // row_ror:12: lane b <- b + 4
  v4[2] = __builtin_amdgcn_update_dpp(0, v, 0x128, 0xf, 0xf, false);  // row_ror:8
  v4[3] = __builtin_amdgcn_update_dpp(0, v, 0x124, 0xf, 0xf, false);  // row_ror:4:  lane b <- b + 12
}
// sign mask of absolute inputs re-indexed for col4's rotation by `own`
__device__ __forceinline__ uint32_t rot_sign(uint32_t m, int own) { return ((m | m << 4) >> own) & 15; }
// FTransformWHT output b of the row's 16 DC inputs (int16 like the reference)
__device__ __forceinline__ int fwht_lane(int in, int b) {
  const int r = b >> 2, c = b & 3;
  int q[4], v4[4];
  quad4(in, q);
  col4(sum4_signed(q, kWhtSign[c]), v4);  // row pass: tmp[4r + c]
  return (int16_t)(sum4_signed(v4, rot_sign(kWhtSign[r], r)) >> 1);
}
// TransformWHT (inverse) output b of the row's 16 dequantised inputs
__device__ __forceinline__ int iwht_lane(int in, int b) {
  const int k = b >> 2, i = b & 3;
  int v4[4], q[4];
  col4(in, v4);
  quad4(sum4_signed(v4, rot_sign(kWhtSign[k], k)), q);  // column pass: tmp[4k + i]
  return (int16_t)((sum4_signed(q, kWhtSign[i]) + 3) >> 3);
}
// QuantizeCoeffs of coefficient b alone (encode_quant.go:16-75)
__device__ __forceinline__ int quantize_one(int v, int b, const SQuant& sq) {
  const int4 h = b == 0 ? *reinterpret_cast<const int4*>(&sq.dc_quant) : *reinterpret_cast<const int4*>(&sq.quant);
  const int sign = v < 0 ? -1 : 1;
  const int a = max(abs(v) + sq.sharpen[b], 0);
  const int c = min((int)(((uint32_t)wg::mul_i24(a, h.y) + (uint32_t)h.z) >> 17), 2047);
  return sign * c;
}
// max over the 16 lanes of a DPP row, in every lane of the row
__device__ __forceinline__ int row_max(int v) {
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false));  // row_half_mirror
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xf, 0xf, false));  // row_mirror
  return v;
}
constexpr uint64_t pack_rzig() {
  uint64_t v = 0;
  for (int i = 0; i < 16; i++) v |= (uint64_t)kRZig[i] << (4 * i);
  return v;
}
__device__ __forceinline__ int rzig_of(int n) { return (int)((pack_rzig() >> (4 * n)) & 15); }
// The Y2 (DC) block of an I16 macroblock, lane-parallel (pickBestI16ModeRD
// :640-660 and encodeResiduals's DC part): lane b of a 16-lane row passes
// its 4x4 block's DC coefficient and gets back the block's reconstructed DC
// (the inverse WHT of the dequantised levels).  *q = level b; *nz = the
// block's zigzag nz count and *cost = its TokenCostForCoeffs (type 1) --
// *nz in every lane of the row, *cost in the row's first lane.
__device__ __forceinline__ int dc_block_lane(const Tables& t, int dc_in, int lane, const SQuant& y2, int ctx0, int* q,
                                             int* nz, int* cost) {
  const int b = lane & 15, base = lane & ~15;
  const int lv = quantize_one(fwht_lane(dc_in, b), b, y2);
  const int nzc = row_max(lv != 0 ? rzig_of(b) + 1 : 0);
  // lane b = zigzag position b of the token cost
  const int v = abs(__shfl(lv, base + zig_of(b), 64));
  const int prev = abs(__shfl(lv, base + zig_of(max(b - 1, 0)), 64));
  const int ctx = b == 0 ? ctx0 : min(prev, 2);
  const int band = band_of(b);
  int tc = 0;
  if (b < nzc) tc = vc_of(t.vcost[8 + band][min(v, 67)], ctx) + t.lfixed[min(v, 2047)];
  else if (b == nzc) tc = t.tok[8 + band].eob[ctx];
  *q = lv;
  *nz = nzc;
  *cost = group_sum_first<16>(tc);
  const int2 qq = make_int2(y2.quant, y2.dc_quant);
  return iwht_lane((int16_t)(lv * (b == 0 ? qq.y : qq.x)), b);
}

// lane L of each 16-lane DPP row, broadcast to the row (row_newbcast, gfx90a+)
template <int L>
__device__ __forceinline__ uint64_t row_bcast64(uint64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x150 + L, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x150 + L, 0xf, 0xf, false);
  return (uint64_t)(uint32_t)hi << 32 | (uint32_t)lo;
}
// min over the 16 lanes of a DPP row, result in every lane of the row
__device__ __forceinline__ uint32_t row_min_u32(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false));  // row_half_mirror
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false));  // row_mirror
  return v;
}

// The reference's candidate pick for one I4 block (tryI4ModesRDParallel
// :869-886): compact the eligible modes, then K rounds of first-argmin +
// swap.  Lane m (< 10) of a 16-lane row holds mode m's key
// sse << 8 | compacted position << 4 | m (sse <= 16 * 255^2 < 2^21), so the
// first minimum is a row min; the swap moves the element at position i to
// the winner's position.  Returns candidate i's mode in cm[i], uniform over
// the row.  `eligible`: bit m set when mode m is allowed for this block.
__device__ __forceinline__ void select_i4_modes(int sse, int m, uint32_t eligible, int K, int cm[3]) {
  const bool ok = m < 10 && ((eligible >> m) & 1);
  uint32_t key = ok ? ((uint32_t)sse << 8 | (uint32_t)__builtin_popcount(eligible & ((1u << m) - 1)) << 4 | (uint32_t)m) : ~0u;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const uint32_t kmin = row_min_u32(key);
    cm[i] = (int)(kmin & 15);
    if (i + 1 < 3) {
      const uint32_t wpos = (kmin >> 4) & 15;
      const bool at_i = ((key >> 4) & 15) == (uint32_t)i;
      key = key == kmin ? ~0u : (at_i && key != ~0u ? ((key & ~0xf0u) | wpos << 4) : key);
    }
  }
  (void)K;
}

// residual + reconstruction of one 4x4 block: rec = clip(pred + IDCT(dq))
template <typename QT>
__device__ __forceinline__ void dequant(const QT& q, int dq[16], const SQuant& sq) {
  const int2 qq = make_int2(sq.quant, sq.dc_quant);
  // |level| <= 2047, quantisers < 2^10: full-rate 24-bit products
  dq[0] = (int16_t)wg::mul_i24(lvl_at(q, 0), qq.y);
#pragma unroll
  for (int i = 1; i < 16; i++) dq[i] = (int16_t)wg::mul_i24(lvl_at(q, i), qq.x);
}
__device__ __forceinline__ void recon4(const int pred[16], const int dq[16], int rec[16]) {
#pragma unroll
  for (int r = 0; r < 4; r++) {
    int res[4];
    idct_row(dq, r, res);
#pragma unroll
    for (int c = 0; c < 4; c++) rec[4 * r + c] = clip8(pred[4 * r + c] + res[c]);
  }
}
__device__ __forceinline__ int sse16(const int a[16], const int b[16]) {
  int s = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) s += (a[i] - b[i]) * (a[i] - b[i]);
  return s;
}
__device__ __forceinline__ int ttrans(const int px[16]) {  // tTransform (ssim.go:266-304)
  const int kw[16] = {38, 32, 20, 9, 32, 28, 17, 7, 20, 17, 10, 4, 9, 7, 4, 2};
  int tmp[16];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int* r = px + 4 * i;
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
__device__ __forceinline__ void fdct(const int src[16], const int pred[16], int co[16]) {
  wg::s16x2_t d01[4], d32[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    d01[k] = (wg::s16x2_t){(short)(src[k] - pred[k]), (short)(src[4 + k] - pred[4 + k])};
    d32[k] = (wg::s16x2_t){(short)(src[12 + k] - pred[12 + k]), (short)(src[8 + k] - pred[8 + k])};
  }
  wg::fdct4x4_pk(d01, d32, co);
}
__device__ __forceinline__ void store4x4(uint8_t* p, const int v[16]) {
#pragma unroll
  for (int r = 0; r < 4; r++)
    *reinterpret_cast<uint32_t*>(p + r * BPS) = pack4(v[4 * r], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
}
__device__ __forceinline__ void unpack_rows(uint32_t w, int* d) {
#pragma unroll
  for (int c = 0; c < 4; c++) d[c] = byte_of(w, c);
}
__device__ __forceinline__ void load4x4(const uint8_t* p, int v[16]) {  // p 4-byte aligned (all block origins are)
#pragma unroll
  for (int r = 0; r < 4; r++) unpack_rows(*reinterpret_cast<const uint32_t*>(p + r * BPS), v + 4 * r);
}
// A 4x4 pixel block as four packed row words (4 VGPRs instead of 16):
// blocks stay packed across the RD phases and are unpacked a row at a time.
struct P4 {
  uint32_t r[4];
};
__device__ __forceinline__ P4 ld4(const uint8_t* p) {  // p 4-byte aligned
  P4 b;
#pragma unroll
  for (int r = 0; r < 4; r++) b.r[r] = *reinterpret_cast<const uint32_t*>(p + r * BPS);
  return b;
}
__device__ __forceinline__ void st4(uint8_t* p, const P4& b) {
#pragma unroll
  for (int r = 0; r < 4; r++) *reinterpret_cast<uint32_t*>(p + r * BPS) = b.r[r];
}
// sum of squared byte differences: a.a + b.b - 2 a.b with v_dot4_u32_u8
__device__ __forceinline__ int sse_p(const P4& a, const P4& b) {
  uint32_t aa = 0, bb = 0, ab = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    aa = __builtin_amdgcn_udot4(a.r[r], a.r[r], aa, false);
    bb = __builtin_amdgcn_udot4(b.r[r], b.r[r], bb, false);
    ab = __builtin_amdgcn_udot4(a.r[r], b.r[r], ab, false);
  }
  return (int)(aa + bb - 2 * ab);
}
// FTransform of (src - pred), rows unpacked one at a time
__device__ __forceinline__ void fdct_p(const P4& s, const P4& p, int co[16]) {
  // (byte k of rows a and b as the int16 halves of a word: one v_perm each)
  wg::s16x2_t d01[4], d32[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t sel = 0x0c000c00u | (uint32_t)(4 + k) << 16 | (uint32_t)k;
    d01[k] = __builtin_bit_cast(wg::s16x2_t, __builtin_amdgcn_perm(s.r[1], s.r[0], sel)) -
             __builtin_bit_cast(wg::s16x2_t, __builtin_amdgcn_perm(p.r[1], p.r[0], sel));
    d32[k] = __builtin_bit_cast(wg::s16x2_t, __builtin_amdgcn_perm(s.r[2], s.r[3], sel)) -
             __builtin_bit_cast(wg::s16x2_t, __builtin_amdgcn_perm(p.r[2], p.r[3], sel));
  }
  wg::fdct4x4_pk(d01, d32, co);
  return;
  int tmp[16];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int d0 = byte_of(s.r[r], 0) - byte_of(p.r[r], 0), d1 = byte_of(s.r[r], 1) - byte_of(p.r[r], 1);
    const int d2 = byte_of(s.r[r], 2) - byte_of(p.r[r], 2), d3 = byte_of(s.r[r], 3) - byte_of(p.r[r], 3);
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
    co[c] = (int16_t)((a0 + a1 + 7) >> 4);
    co[4 + c] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0));
    co[8 + c] = (int16_t)((a0 - a1 + 7) >> 4);
    co[12 + c] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
  }
}
// rec = clip(pred + IDCT(dq)), a row at a time
__device__ __forceinline__ P4 recon_p(const P4& pred, const int dq[16]) {
  P4 o;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    int res[4];
    idct_row(dq, r, res);
    o.r[r] = pack4(clip8(byte_of(pred.r[r], 0) + res[0]), clip8(byte_of(pred.r[r], 1) + res[1]),
                   clip8(byte_of(pred.r[r], 2) + res[2]), clip8(byte_of(pred.r[r], 3) + res[3]));
  }
  return o;
}
// tTransform (ssim.go:266-304) of a packed block
__device__ __forceinline__ int ttrans_p(const P4& b) {
  const int kw[16] = {38, 32, 20, 9, 32, 28, 17, 7, 20, 17, 10, 4, 9, 7, 4, 2};
  int tmp[16];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int r0 = byte_of(b.r[i], 0), r1 = byte_of(b.r[i], 1), r2 = byte_of(b.r[i], 2), r3 = byte_of(b.r[i], 3);
    const int a0 = r0 + r2, a1 = r1 + r3, a2 = r1 - r3, a3 = r0 - r2;
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
// ttrans_p(b) - ttrans_p(a) in one pass: each pixel pair (b, a) as the two
// int16 halves of a word (v_perm), the transform's butterflies packed
// (|values| <= 4080), and sum_j w_j (|Tb_j| - |Ta_j|) as signed dot products
// with (w_j, -w_j): the same integer as the two sums' difference
__device__ __forceinline__ int ttrans_diff_p(const P4& a, const P4& b) {
  const short kw[16] = {38, 32, 20, 9, 32, 28, 17, 7, 20, 17, 10, 4, 9, 7, 4, 2};
  s16x2 tmp[16];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    s16x2 p[4];
#pragma unroll
    for (int k = 0; k < 4; k++)  // {b byte k, a byte k} as int16 halves
      p[k] = as_s16x2((int)__builtin_amdgcn_perm(a.r[i], b.r[i], 0x0c000c00u | (uint32_t)(4 + k) << 16 | (uint32_t)k));
    const s16x2 a0 = p[0] + p[2], a1 = p[1] + p[3], a2 = p[1] - p[3], a3 = p[0] - p[2];
    tmp[4 * i] = a0 + a1;
    tmp[4 * i + 1] = a3 + a2;
    tmp[4 * i + 2] = a3 - a2;
    tmp[4 * i + 3] = a0 - a1;
  }
  int sum = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const s16x2 a0 = tmp[i] + tmp[8 + i], a1 = tmp[4 + i] + tmp[12 + i];
    const s16x2 a2 = tmp[4 + i] - tmp[12 + i], a3 = tmp[i] - tmp[8 + i];
    const s16x2 o[4] = {a0 + a1, a3 + a2, a3 - a2, a0 - a1};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const short w = kw[4 * j + i];
      sum = __builtin_amdgcn_sdot2(__builtin_elementwise_max(o[j], -o[j]), (s16x2){w, (short)-w}, sum, false);
    }
  }
  return sum;
}
__device__ __forceinline__ int tdisto_p(const P4& a, const P4& b) { return abs(ttrans_diff_p(a, b)) >> 5; }
__device__ __forceinline__ P4 predsq_p(int mode, const uint8_t* base, int size, int px, int py) {
  const int dc = predsq_dc(mode, base, size);
  P4 o;
#pragma unroll
  for (int r = 0; r < 4; r++) o.r[r] = predsq_row4(mode, base, px, py + r, dc);
  return o;
}
// 16x16 / 8x8 square prediction of the 4x4 block at (px, py) of `base`
__device__ __forceinline__ void predsq_block(int mode, const uint8_t* base, int size, int px, int py, int pred[16]) {
  const int dc = predsq_dc(mode, base, size);
#pragma unroll
  for (int r = 0; r < 4; r++) unpack_rows(predsq_row4(mode, base, px, py + r, dc), pred + 4 * r);
}
// Build the block's value table V (see kPred4Code) from the context around
// buf + off in one pass of the caller's half-wave (lane i < 32): lanes 0..14
// load the edge E[i] and take their neighbours' by DPP row shifts for the
// pair / triple averages, lane 15 the DC, lanes 16..31 the TM values.  The
// caller syncs once after it.
__device__ __forceinline__ void pred4_values(const uint8_t* buf, int off, int i, uint8_t* v) {
  const uint8_t* d = buf + off;
  int e = 0;
  if (i < 15) {  // E: L L K J I X A..H H
    const int src = i <= 1 ? -1 + 3 * BPS : (i <= 4 ? -1 + (4 - i) * BPS : (i == 5 ? -1 - BPS : -BPS + min(i - 6, 7)));
    e = d[src];
  }
  // E[i + 1] and E[i - 1] (lanes 0..15 are one DPP row of the half-wave)
  const int en = __builtin_amdgcn_update_dpp(0, e, 0x101, 0xf, 0xf, false);  // row_shl:1: lane i <- i + 1
  const int ep = __builtin_amdgcn_update_dpp(0, e, 0x111, 0xf, 0xf, false);  // row_shr:1: lane i <- i - 1
  if (i < 15) {
    v[i] = (uint8_t)e;
    if (i < 14) v[16 + i] = (uint8_t)avg2(e, en);
    if (i >= 1 && i <= 13) v[32 + i] = (uint8_t)avg3(ep, e, en);
  } else if (i == 15) {
    int sum = 4;
#pragma unroll
    for (int k = 0; k < 4; k++) sum += d[k - BPS] + d[-1 + k * BPS];
    v[47] = (uint8_t)(sum >> 3);
  } else {  // TM of pixel p = i - 16
    const int p = i - 16, x = p & 3, y = p >> 2;
    v[48 + p] = (uint8_t)clip8(d[-1 + y * BPS] + d[x - BPS] - d[-1 - BPS]);
  }
}
__device__ __forceinline__ void pred4_lut(const uint4 c, const uint8_t* v, int pred[16]) {
  const uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
  for (int p = 0; p < 16; p++) pred[p] = v[(w[p >> 2] >> (8 * (p & 3))) & 0xff];
}
__device__ __forceinline__ void pred4_lut(const uint8_t* code, const uint8_t* v, int pred[16]) {
  pred4_lut(*reinterpret_cast<const uint4*>(code), v, pred);
}
__device__ __forceinline__ int check_mode(int mbx, int mby, int mode) {
  const int edge = (mbx == 0) ? ((mby == 0) ? 6 : 5) : ((mby == 0) ? 4 : 0);
  return mode == 0 ? edge : mode;
}
__device__ __forceinline__ uint64_t rd_score(int disto, int rate, int lambda) {
  return (uint64_t)(int64_t)rate * (uint64_t)(int64_t)lambda + 256ull * (uint64_t)(int64_t)disto;
}
// Sum over an aligned group of 8 / 16 lanes, valid in the group's FIRST lane
// only, by DPP (quad_perm swaps, then row_ror): the __shfl_xor form went
// through ds_bpermute, an LDS round trip per level.
template <int WIDTH>
__device__ __forceinline__ int group_sum_first(int v) {
  static_assert(WIDTH == 8 || WIDTH == 16, "group width");
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0, v, 0x12C, 0xf, 0xf, false);  // row_ror:12 (lane i <- i + 4 mod 16)
  if (WIDTH == 16) v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xf, 0xf, false);  // row_ror:8
  return v;
}
template <typename T>
__device__ __forceinline__ T group_sum(T v, int width) {  // sum over aligned groups of `width` lanes
  for (int o = width >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Each wave works on its own macroblock row, so the cross-lane hand-offs
// through LDS need a wave-level order only: the LDS unit executes one wave's
// DS instructions in issue order, so a read issued after a write of the
// same wave returns the written bytes without draining the queue first
// (s_waitcnt lgkmcnt(0) before every hand-off cost 1.3% of the launch:
// noise frame 15.73 -> 15.52 ms, 64 x 1080p 23.16 -> 22.86 ms); only the
// compiler must not move accesses across.  Waits on the data an LDS read
// returns stay the compiler's.  WG_ENC_DRAIN restores the drains (A/B).
// Cross-wave exchanges (the pair schedule's join, the I16 score flag) keep
// their barriers and explicit waits.
__device__ __forceinline__ void lds_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// An opaque copy of the LDS base (still typed as LDS, so accesses stay
// ds_read/ds_write).  Re-taken at the top of a loop body it stops the
// compiler from hoisting loop-invariant table reads (token-cost rows,
// segment fields) out of the loop and pinning them in registers for the
// whole loop -- which is what drove this kernel past 256 VGPRs.
// threadIdx.x through an opaque move: lane-derived values (addresses,
// block coordinates) are then re-derived where used instead of being
// hoisted out of the row loop and pinned in registers for the whole kernel
__device__ __forceinline__ int opaque_lane() {
  int l;
  asm volatile("v_mov_b32 %0, %1" : "=v"(l) : "v"((int)threadIdx.x & 63));
  return l;
}
// a wave-uniform 64-bit value into SGPRs (the builtin takes 32 bits)
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32;
}
template <typename T>
__device__ __forceinline__ T& launder(T& s) {
  typedef __attribute__((address_space(3))) T LdsT;
  LdsT* p = (LdsT*)&s;
  asm volatile("" : "+s"(p));
  return *(T*)p;
}

// The row hand-off: a record of REC_WORDS words per MB column (the Y bottom
// row's pixels 0-3, U 4-5, V 6-7, top nz 8, top modes 9, top DC nz 10), each
// word in an 8-B granule {word, tag} that is written and read as ONE 64-bit
// atomic (single-copy atomic in the AMDGPU memory model), tag = the writing
// row + 1.  The row below polls the granules themselves -- no progress
// counter, no store drain before a flag, and the record arrives with the poll
// that finds it -- and no granule can pass the poll with a word other than
// the one stored beside its tag.  Every launch clears the records first (with
// its control words, wg_encode_mbs), so a granule holds 0 until its row of
// THIS launch writes it: no record of an earlier launch on the buffer passes.
__device__ __forceinline__ uint64_t ld_granule(const uint8_t* p) {
  return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_granule(uint8_t* p, uint32_t word, uint32_t tag) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), (uint64_t)tag << 32 | word, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

struct EncArgs {
  const uint8_t* y;  // source planes (stride 16*mbw / 8*mbw), pitch per image
  const uint8_t* u;
  const uint8_t* v;
  uint8_t* ry;  // reconstruction (may alias the source)
  uint8_t* ru;
  uint8_t* rv;
  const uint8_t* segments;  // per MB segment id, n_img * mbw * mbh
  const Segment* segs;      // 4 per image, segs_pitch bytes apart (0: one table for all)
  int64_t segs_pitch;
  const uint8_t* proba;     // 1056
  MbEnc* out;
  uint8_t* top;   // [n_img][mbw][REC]
  int* ctl;       // [0] dequeue, [1] error
  int* diag;      // wg::diag_words + DIAG_ENCODE
  const int* order;  // the work buffer's row schedule (wg_encode_row_order): dequeue index -> row * n_img + image
  const int* border; // the same schedule over bands of WAVES rows: dequeue index -> band * n_img + image
  const int* order_tag;  // {ORDER_TAG ^ n_img, ~(ORDER_TAG ^ mbh)} when the schedule was built for this batch shape, else (row, image) order
  int64_t y_pitch, uv_pitch;
  int width, height, mbw, mbh, n_img, quality;
};

constexpr uint64_t SPIN_TICKS = 200000000ull;

constexpr int ORDER_TAG = 0x5e0d0000;  // marks a row schedule in the work buffer (xor the batch shape)

// (WG_STAMPS builds, wg_instr.h) cycles per phase summed over macroblocks
WG_IF_STAMPS(__device__ unsigned long long g_enc_phase[16];)

// (WG_ROWTIMES builds) per dequeued row, {ro, start, end, block} in
// s_memrealtime ticks (100 MHz) -- the launch's row timeline
WG_IF_ROWTIMES(__device__ unsigned long long g_row_times[16384][4];)


// (WG_EXP_REP_<P> builds: WG_REP_BEGIN(P) / WG_REP_END around a phase, wg_instr.h)

// An image's four segment tables (4 x 224 B = 56 x 16 B) into LDS
__device__ __forceinline__ void load_segments(const EncArgs& a, int img, Segment* dst, int lane) {
  const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(a.segs) + img * a.segs_pitch);
  if (lane < 56 && WG_CHK(src + lane, 16, a.segs, a.segs_pitch ? a.n_img * a.segs_pitch : 4 * (int64_t)sizeof(Segment),
                          "k_encode_rows segs"))
    reinterpret_cast<uint4*>(dst)[lane] = src[lane];
}

// The barrier of one group of WAVES waves inside a larger workgroup: each
// wave's lane 0 counts itself in at *cnt (release) and waits until the whole
// group has (acquire).  *gen is the wave's running target; every wave of the
// group passes the same barriers.
__device__ __forceinline__ void group_barrier(int* cnt, int& gen, int lane) {
  gen += WAVES;
  if (lane == 0) {
    __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < gen) __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_wave_barrier();
}
// TRELLIS: method >= 4 (trellis quantisation in the I4 RD and the final I16
// residuals, encode_parallel.go:793, :1202); method 3 quantises plainly
// (pickBestI4ModeRDParallel :842-929, QuantizeCoeffs at :1215).
//
// PAIR: a row is walked by a pair of waves (a 2-wave workgroup).  The luma
// and chroma chains of a macroblock are independent up to the export (the
// I4 / I16 choice reads luma only, the chroma mode chroma only), so wave A
// (wave 0) runs import, context and the I4 RD while wave B (wave 1) runs the
// I16 RD, the UV RD, the final residuals of I16 (speculatively) and chroma
// and their reconstruction; A joins the two and exports.  A's early exit
// takes B's I16 score once B has posted it; until then it runs on (an I4
// pass the reference would have cut short loses to I16 all the same).  This
// roughly halves a macroblock's latency for launches whose rows fit the
// wave slots twice over (one frame, C2); a full batch keeps one wave a row.
template <bool TRELLIS, bool PAIR>
__global__ __launch_bounds__(64 * (PAIR ? 2 : WAVES * GROUPS), PAIR ? 2 : 2) void k_encode_rows(EncArgs a) {
  constexpr int NW = PAIR ? 2 : WAVES * GROUPS;
  __shared__ Tables t_lds;
  __shared__ Shared s_waves[NW];
  __shared__ int s_gbar[GROUPS];  // the groups' barrier counters (group_barrier)
  // the quantisers of the image a group's band (PAIR: the pair's row) belongs to
  // (one group: two tables, by band sequence parity -- the group's waves
  // move on to their next band one by one, see the dequeue below)
  constexpr bool LOOSE = !PAIR && GROUPS == 1;
  __shared__ Segment s_seg[PAIR ? 1 : (LOOSE ? 2 : GROUPS)][4];
  // LOOSE: the band of each sequence parity, its publication (sequence + 1)
  // and the count of waves done with it (monotonic over the parity's uses)
  __shared__ int s_band[2], s_ready[2], s_done[2];
  static_assert(PAIR || sizeof(Tables) + NW * sizeof(Shared) + sizeof(s_gbar) + sizeof(s_seg) <= 160 * 1024,
                "the workgroup's LDS must fit one CU");
  Tables& t = t_lds;
  const int tid = threadIdx.x;
  constexpr int NT = 64 * NW;
  for (int i = tid; i < 1056; i += NT) t.proba[i] = a.proba[i];
  for (int i = tid; i < 256; i += NT) t.ecost[i] = vp8_entropy_cost[i];
  for (int i = tid; i < 2048; i += NT) t.lfixed[i] = vp8_level_fixed_costs[i];
  for (int i = tid; i < 1000; i += NT) t.fixed_i4[i] = c_fixed_i4[i];
  if (tid < 16) t.wtr[tid] = c_wtrellis[tid];
  if (tid < GROUPS) s_gbar[tid] = 0;
  if (tid < 2) s_ready[tid] = s_done[tid] = 0;
  for (int i = tid; i < 160; i += NT) t.pcode[i >> 4][i & 15] = kPred4Code[i >> 4][i & 15];
  __syncthreads();
  for (int i = tid; i < 4 * 8 * 68; i += NT) {
    const int tb = i / 68, level = i % 68;
    uint64_t w = 0;
    for (int c = 0; c < 3; c++) {
      const uint8_t* p = t.proba + (tb * 3 + c) * 11;
      // the whole token cost of a level at this (type, band, context) but
      // its fixed part: zero token for level 0, else the non-zero prefix +
      // variableLevelCost (encode_quant.go:170-220, 258-273)
      const int cost = level == 0 ? ecost(t, 255 - p[0]) + ecost(t, p[1])
                                  : ecost(t, 255 - p[0]) + ecost(t, 255 - p[1]) + variable_level_cost(t, level, p);
      w |= (uint64_t)cost << (16 * c);
    }
    t.vcost[tb][level] = w;
  }
  if (tid < 4 * 8) {
    TokRow r = {};
    for (int c = 0; c < 3; c++) {
      const uint8_t* p = t.proba + (tid * 3 + c) * 11;
      r.zero[c] = (uint16_t)(ecost(t, 255 - p[0]) + ecost(t, p[1]));
      r.nz[c] = (uint16_t)(ecost(t, 255 - p[0]) + ecost(t, 255 - p[1]));
      r.eob[c] = (uint16_t)ecost(t, p[0]);
    }
    t.tok[tid] = r;
  }
  __syncthreads();  // the tables are read-only from here; the waves run independently
  __builtin_amdgcn_s_setprio(1);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  // roles (wave-uniform): one wave a row does both; in PAIR wave 0 is A, wave 1 is B
  const bool isA = !PAIR || wave == 0, isB = !PAIR || wave == 1;
  Shared& s = s_waves[wave];
  const int mbw = a.mbw, mbh = a.mbh;
  const int ys = 16 * mbw, uvs = 8 * mbw;
  const int max_modes = a.quality < 50 ? 2 : 3;
  const int total_rows = a.n_img * mbh;
  ESTAMP_DECL;

  const bool use_order = a.order_tag[0] == (ORDER_TAG ^ a.n_img) && a.order_tag[1] == ~(ORDER_TAG ^ mbh);
  const int n_bands = (mbh + WAVES - 1) / WAVES;
  // (not PAIR) this wave's group and its place in it
  const int grp = wave / WAVES, gw = wave - WAVES * grp;
  int gen = 0;
  int q = 0;  // LOOSE: this wave's band sequence number in the workgroup
  // LOOSE: bounded LDS spin of the whole wave until *p >= need (acquire)
  auto wait_lds = [&](const int* p, int need) {
    const uint64_t t0 = wg::wait_clock();
    for (uint32_t it = 0;; it++) {
      if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) >= need)
        return;
      if ((it & 63) == 63 && wg::wait_clock() - t0 > SPIN_TICKS) {
        if (lane == 0) {
          __hip_atomic_fetch_or(&a.ctl[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          wg::note_timeout(a.diag, -1, q, need, 0, (int)(wg::wait_clock() - t0), (int)blockIdx.x);
        }
        return;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  };
  for (;;) {
    // PAIR: the workgroup's wave pair dequeues a row; otherwise each group
    // of WAVES waves dequeues a BAND of WAVES consecutive rows of one image
    // and its wave w walks row WAVES * band + w.  The band's rows start
    // staggered (each trails the one above by about two macroblocks) and
    // finish together, so the group takes its next band as soon as this one
    // is done, and the workgroup leaves when its groups find no band left:
    // with one row per wave dequeued independently, a workgroup with one row
    // left held all its wave slots and its LDS through the launch's tail, and
    // the next batch's launch could not start there (tools/enc_timeline.py).
    // A group barrier after the dequeue (the next write of word is after the
    // band's closing barrier).
    int row, mby, img, ro;
    if constexpr (PAIR) {  // the pair dequeues together (the next write of word is two barriers on)
      if (tid == 0) s_waves[0].word = __hip_atomic_fetch_add(&a.ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      row = __builtin_amdgcn_readfirstlane(s_waves[0].word);
      if (row >= total_rows) break;
      ro = use_order ? __builtin_amdgcn_readfirstlane(a.order[row]) : row;
      mby = ro / a.n_img;
      img = ro % a.n_img;
    } else if constexpr (LOOSE) {
      // The group's waves do not meet between bands: a band's rows start
      // staggered (each trails the row above by a little more than one
      // macroblock) and end staggered the same way, so a barrier there held
      // the leading waves idle for the trailing rows' lag twice a band
      // (~14 macroblock times of four waves in 480).  Wave 0 dequeues band
      // sequence q as soon as it finishes q - 1 (and every wave has finished
      // q - 2, whose table slot it reuses); each wave picks it up when it is
      // done with its own row of q - 1.  Every wait is still on a row
      // dequeued earlier.
      const int p = q & 1;
      if (gw == 0) {
        if (q >= 2) wait_lds(&s_done[p], WAVES * (q / 2));
        int b = 0;
        if (lane == 0) b = __hip_atomic_fetch_add(&a.ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        b = __shfl(b, 0, 64);
        if (b < a.n_img * n_bands) {
          const int bo = use_order ? __builtin_amdgcn_readfirstlane(a.border[b]) : b;
          load_segments(a, bo % a.n_img, s_seg[p], lane);
        }
        if (lane == 0) {
          s_band[p] = b;
          __hip_atomic_store(&s_ready[p], q + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      wait_lds(&s_ready[p], q + 1);
      const int band = __builtin_amdgcn_readfirstlane(s_band[p]);
      if (band >= a.n_img * n_bands) break;
      const int bo = use_order ? __builtin_amdgcn_readfirstlane(a.border[band]) : band;  // band y * n_img + image
      img = bo % a.n_img;
      mby = WAVES * (bo / a.n_img) + gw;
      ro = mby * a.n_img + img;
      row = WAVES * band + gw;
    } else {
      int& word = s_waves[WAVES * grp].word;
      if (gw == 0) {  // the group's leader dequeues and fetches the band's image's segments
        if (lane == 0) word = __hip_atomic_fetch_add(&a.ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lds_sync();
        const int band = __builtin_amdgcn_readfirstlane(word);
        if (band < a.n_img * n_bands) {
          const int bo = use_order ? __builtin_amdgcn_readfirstlane(a.border[band]) : band;
          load_segments(a, bo % a.n_img, s_seg[grp], lane);
        }
      }
      if constexpr (GROUPS == 1) __syncthreads();
      else group_barrier(&s_gbar[grp], gen, lane);
      const int band = __builtin_amdgcn_readfirstlane(word);
      if (band >= a.n_img * n_bands) break;
      const int bo = use_order ? __builtin_amdgcn_readfirstlane(a.border[band]) : band;  // band y * n_img + image
      img = bo % a.n_img;
      mby = WAVES * (bo / a.n_img) + gw;
      ro = mby * a.n_img + img;
      row = WAVES * band + gw;
    }
    const bool live = mby < mbh;  // (the last band of an image may have fewer rows)
    WG_IF_ROWTIMES(const unsigned long long row_t0 = wg::wait_clock();)
    const uint8_t* Y = a.y + img * a.y_pitch;
    const uint8_t* U = a.u + img * a.uv_pitch;
    const uint8_t* V = a.v + img * a.uv_pitch;
    uint8_t* RY = a.ry + img * a.y_pitch;
    uint8_t* RU = a.ru + img * a.uv_pitch;
    uint8_t* RV = a.rv + img * a.uv_pitch;
    uint8_t* top = a.top + (int64_t)img * mbw * REC;
    // (WG_BOUNDS) the buffers' extents from wg_encode_mbs' shapes
    [[maybe_unused]] const int64_t y_n = a.n_img * a.y_pitch, uv_n = a.n_img * a.uv_pitch,
                                   top_n = (int64_t)a.n_img * mbw * REC, mb_n = (int64_t)a.n_img * mbw * mbh;
    if (PAIR && isA) load_segments(a, img, s_seg[0], lane);  // (B reads them after the MB's first join barrier)
    // left context (encodeRow :257-282)
    if (lane < 16) s.yout[YOFF - 1 + lane * BPS] = 129;
    else if (lane < 24) s.yout[UOFF - 1 + (lane - 16) * BPS] = 129;
    else if (lane < 32) s.yout[VOFF - 1 + (lane - 24) * BPS] = 129;
    uint32_t left_nz = 0;
    int left_nz_dc = 0;
    uint32_t left_modes = 0;  // 4 x 8 bits, B_DC_PRED = 0
    int tl_y = 127, tl_u = 127, tl_v = 127;
    // source rows loaded ahead for the next MBs of the pair / quad (import),
    // reconstruction rows held back for a whole-sector store (export)
    uint4 stg0 = make_uint4(0, 0, 0, 0), stg1 = stg0, rst0 = stg0;
    uint2 rst1 = make_uint2(0, 0);

    for (int mbx = 0; live && mbx < mbw; mbx++) {
      Shared& s = launder(s_waves[wave]);
      Shared& c = launder(s_waves[PAIR ? 0 : wave]);  // the MB's pixels and context (A's)
      Tables& t = launder(t_lds);
      const int lane = opaque_lane();
      const int64_t mbi = ((int64_t)img * mbh + mby) * mbw + mbx;
      ESTAMP(0);
      // ---- wait for the row above ----
      // The reference starts MB x of row y once row y-1 has finished MB x+1
      // (encode_parallel.go:286-295); only the I4 blocks on the right edge
      // (3, 7, 11, 15) read MB x+1 of the row above (its first 4 bottom
      // pixels, the top-right context), and the first of them runs at I4
      // step 3.  So the MB starts once MB x of the row above is done, and
      // waits for MB x+1 only there (the top-right poll): the outputs are
      // the reference's, the rows just trail each other by less.
      // the record of column x of the row above (lane i < n: word i), polled
      // until every granule carries the row's tag
      auto poll_rec = [&](const uint8_t* rec, int n) -> uint32_t {
        uint32_t w = 0;
        if (mby > 0) {
          const uint32_t want = (uint32_t)mby;  // row mby - 1's tag
          const uint64_t t0 = wg::wait_clock();
          for (uint32_t it = 0;; it++) {
            const uint64_t g =
                lane < n && WG_CHK(rec + 8 * lane, 8, a.top, top_n, "k_encode_rows record load") ? ld_granule(rec + 8 * lane) : 0;
            w = (uint32_t)g;
            if (__ballot(lane < n && (uint32_t)(g >> 32) != want) == 0) break;
            if ((it & 63) == 63 && (wg::wait_clock() - t0 > SPIN_TICKS ||
                                    __hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
              if (lane == 0) {
                __hip_atomic_fetch_or(&a.ctl[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                wg::note_timeout(a.diag, mby, img, mbx, n, (int)(wg::wait_clock() - t0), (int)blockIdx.x);
              }
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
        }
        return w;
      };
      uint32_t above = 0;
      if (isA) above = poll_rec(top + mbx * REC, REC_WORDS);
      ESTAMP(1);
      const int segid =
          a.segments && WG_CHK(a.segments + mbi, 1, a.segments, mb_n, "k_encode_rows segment ids") ? (a.segments[mbi] & 3) : 0;
      const Segment& sg = s_seg[PAIR ? 0 : (LOOSE ? (q & 1) : grp)][segid];
      uint32_t top_nz = 0, top_modes = 0;
      int top_nz_dc = 0;
      if (isA) {
      // ---- import (importBlockParallel :433-452) with edge replication ----
      // A lane loads one source row.  Where whole 32-B sectors lie inside the
      // image, a Y lane loads the rows of MB pairs (x even, x + 1) and a U / V
      // lane those of MB quads in one go and keeps the rest in registers
      // (stg0 / stg1), so every sector is fetched once: a 16-B (Y) or 8-B
      // (U / V) load per MB fetched the whole sector again for the next MB.
      {
        const int x = 16 * mbx, y = 16 * mby;
        const int ww = min(a.width - x, 16), hh = min(a.height - y, 16);
        if (lane < 16) {
          const int r = min(lane, hh - 1);
          const uint8_t* src = Y + (int64_t)(y + r) * ys + x;
          if (16 * ((mbx & ~1) + 2) <= a.width) {  // the pair is whole
            if ((mbx & 1) == 0 && WG_CHK(src, 32, a.y, y_n, "k_encode_rows Y")) {
              stg0 = *reinterpret_cast<const uint4*>(src);
              stg1 = *reinterpret_cast<const uint4*>(src + 16);
            }
            const uint4 v = (mbx & 1) ? stg1 : stg0;
            *reinterpret_cast<uint2*>(s.yin + YOFF + lane * BPS) = make_uint2(v.x, v.y);
            *reinterpret_cast<uint2*>(s.yin + YOFF + lane * BPS + 8) = make_uint2(v.z, v.w);
          } else {
            for (int c = 0; c < 16; c++)
              s.yin[YOFF + lane * BPS + c] = WG_CHK(src + min(c, ww - 1), 1, a.y, y_n, "k_encode_rows Y") ? src[min(c, ww - 1)] : 0;
          }
        } else if (lane < 32) {
          const int k = lane - 16, pl = k >> 3, j = k & 7;
          const int uvw = (ww + 1) >> 1, uvh = (hh + 1) >> 1;
          const int r = min(j, uvh - 1);
          const uint8_t* P = (pl ? V : U) + (int64_t)(8 * mby + r) * uvs + 8 * mbx;
          if (16 * ((mbx & ~3) + 4) <= a.width) {  // the quad is whole (rows 8-B aligned: 8-B loads)
            if ((mbx & 3) == 0 && WG_CHK(P, 32, pl ? a.v : a.u, uv_n, "k_encode_rows UV")) {
              const uint2 p0 = reinterpret_cast<const uint2*>(P)[0], p1 = reinterpret_cast<const uint2*>(P)[1];
              const uint2 p2 = reinterpret_cast<const uint2*>(P)[2], p3 = reinterpret_cast<const uint2*>(P)[3];
              stg0 = make_uint4(p0.x, p0.y, p1.x, p1.y);
              stg1 = make_uint4(p2.x, p2.y, p3.x, p3.y);
            }
            const uint4 h = (mbx & 2) ? stg1 : stg0;
            *reinterpret_cast<uint2*>(s.yin + (pl ? VOFF : UOFF) + j * BPS) =
                (mbx & 1) ? make_uint2(h.z, h.w) : make_uint2(h.x, h.y);
          } else {
            for (int c = 0; c < 8; c++)
              s.yin[(pl ? VOFF : UOFF) + j * BPS + c] =
                  WG_CHK(P + min(c, uvw - 1), 1, pl ? a.v : a.u, uv_n, "k_encode_rows UV") ? P[min(c, uvw - 1)] : 0;
          }
        }
      }
      // ---- prediction context (fillPredContextParallel :455-562) ----
      {
        if (mby > 0) {
          // lane i holds word i (Y16 U8 V8 of the row above: words 0-7)
          if (lane < 8) {
            const int o = lane < 4 ? YOFF - BPS + 4 * lane : (lane < 6 ? UOFF - BPS + 4 * (lane - 4) : VOFF - BPS + 4 * (lane - 6));
            *reinterpret_cast<uint32_t*>(s.yout + o) = above;
          }
          top_nz = (uint32_t)__builtin_amdgcn_readlane((int)above, 8);
          top_modes = (uint32_t)__builtin_amdgcn_readlane((int)above, 9);
          top_nz_dc = __builtin_amdgcn_readlane((int)above, 10);
        } else {
          if (lane < 21) s.yout[YOFF - BPS + lane] = 127;  // cols 0..20 (top-right incl.)
          else if (lane < 29) s.yout[UOFF - BPS + lane - 21] = 127;
          else if (lane < 37) s.yout[VOFF - BPS + lane - 29] = 127;
        }
        if (lane == 37) s.yout[YOFF - BPS - 1] = (mbx > 0 && mby > 0) ? tl_y : (mby > 0 ? 129 : 127);
        if (lane == 38) s.yout[UOFF - BPS - 1] = (mbx > 0 && mby > 0) ? tl_u : (mby > 0 ? 129 : 127);
        if (lane == 39) s.yout[VOFF - BPS - 1] = (mbx > 0 && mby > 0) ? tl_v : (mby > 0 ? 129 : 127);
      }
      lds_sync();
      // scalar copies of the neighbour context
      top_nz = __builtin_amdgcn_readfirstlane(top_nz);
      top_modes = __builtin_amdgcn_readfirstlane(top_modes);
      top_nz_dc = __builtin_amdgcn_readfirstlane(top_nz_dc);
      if constexpr (PAIR) {  // B's inputs; A's working copy of the context for I4 (B writes yout from here on)
        if (lane == 0) {
          s.ctxw[0] = top_nz;
          s.ctxw[1] = (uint32_t)top_nz_dc;
          s.ctxw[2] = left_nz;
          s.ctxw[3] = (uint32_t)left_nz_dc;
          s.s16_flag = 0;
        }
#pragma unroll
        for (int k = 0; k < (YUV / 4 + 63) / 64; k++) {
          const int i = lane + 64 * k;
          if (i < YUV / 4) reinterpret_cast<uint32_t*>(s.yout2)[i] = reinterpret_cast<const uint32_t*>(s.yout)[i];
        }
      }
      }  // isA
      if constexpr (PAIR) {
        __syncthreads();
        if (isB) {
          top_nz = __builtin_amdgcn_readfirstlane(c.ctxw[0]);
          top_nz_dc = __builtin_amdgcn_readfirstlane((int)c.ctxw[1]);
          left_nz = __builtin_amdgcn_readfirstlane(c.ctxw[2]);
          left_nz_dc = __builtin_amdgcn_readfirstlane((int)c.ctxw[3]);
        }
      }

      ESTAMP(2);
      const int b = lane & 15, bx = b & 3, by = b >> 2;  // I16 lane = (mode, block)
      int best16 = 0, best_uv = 0;
      uint64_t s16 = ~0ull;
      if (isB) {
      // ================= I16 RD (pickBestI16ModeRDParallel :624-737) =================
      // then UV RD (pickBestUVModeRDParallel :1030-1114)
      WG_REP_BEGIN(RD)
      bool src_flat;
      {
        // isFlatSource16 (encode_analysis.go:358)
        const uint8_t v0 = c.yin[YOFF];
        bool mine = true;
#pragma unroll
        for (int k = 0; k < 4; k++) {  // fixed trip count (lane is opaque to the compiler)
          const int i = lane + 64 * k;
          mine &= c.yin[YOFF + (i >> 4) * BPS + (i & 15)] == v0;
        }
        src_flat = __all(mine);
      }
      const int m = lane >> 4;
      const bool mvalid = !((m == 2 && mby == 0) || (m == 3 && mbx == 0) || (m == 1 && (mbx == 0 || mby == 0)));
      P4 src16, pred16;
      Q16 q16;
      int nz16 = 0, dc_in = 0;
      {
        const int off = YOFF + 4 * by * BPS + 4 * bx;
        src16 = ld4(c.yin + off);
        pred16 = predsq_p(check_mode(mbx, mby, m), c.yout + YOFF, 16, 4 * bx, 4 * by);
        int co[16];
        fdct_p(src16, pred16, co);
        dc_in = co[0];
        co[0] = 0;
        nz16 = quantize(co, q16, sg.y1, 1);
      }
      // contexts from the neighbours' nz within the same mode
      // left / top neighbour within the mode's 16-lane row (only read when bx / by > 0): DPP row shifts
      {
        const int nz_left = __builtin_amdgcn_update_dpp(0, nz16, 0x111, 0xf, 0xf, false);  // row_shr:1
        const int nz_top = __builtin_amdgcn_update_dpp(0, nz16, 0x114, 0xf, 0xf, false);   // row_shr:4
        const int l = bx > 0 ? (nz_left > 0) : (int)((left_nz >> by) & 1);
        const int tp = by > 0 ? (nz_top > 0) : (int)((top_nz >> bx) & 1);
        const int ctx = min(l + tp, 2);
        int rate = token_cost(t, q16, nz16, 0, ctx, 1);
        rate = mvalid ? rate : 0;
        bool acnz = false;
#pragma unroll
        for (int i = 1; i < 16; i++) acnz |= q16.get(i) != 0;
        // the mode's DC block (WHT path), lane-parallel over its 16 lanes
        int dcq = 0, dcnz = 0, dccost = 0;
        const int dcrec = dc_block_lane(t, dc_in, lane, sg.y2, min(top_nz_dc + left_nz_dc, 2), &dcq, &dcnz, &dccost);
        int dq[16];
        dequant(q16, dq, sg.y1);
        dq[0] = dcrec;
        const P4 rec16 = recon_p(pred16, dq);
        const int sse = sse_p(src16, rec16);
        const int td = sg.tlambda_sd > 0 ? tdisto_p(src16, rec16) : 0;
        const int rsum = group_sum_first<16>(rate), ssum = group_sum_first<16>(sse), tsum = group_sum_first<16>(td);  // used by lane b == 0
        const unsigned long long acmask = __ballot(acnz);
        if (b == 0 && mvalid) {
          const int total_rate = vp8_mode_fixed_cost16[m] + dccost + rsum;
          int disto = ssum;
          if (sg.tlambda_sd > 0) disto += (sg.tlambda_sd * tsum + 128) >> 8;
          if (src_flat && ((acmask >> (16 * m)) & 0xffffull) == 0) disto *= 2;
          s.mode_rate[m] = total_rate;
          s.mode_disto[m] = disto;
        }
      }
      // The UV RD after the I16 one, not interleaved with it: as one stream
      // the two held 184 VGPRs at once (the kernel's peak), apart they fit the
      // budget of three waves per SIMD.
      __builtin_amdgcn_sched_barrier(0);
      {
        // UV lane = (mode, plane, block) over lanes 0..31; lanes 32..63 repeat
        // them (discarded) so that no branch splits the stream
        const int ul = lane & 31, um = ul >> 3, uk = ul & 7, upl = uk >> 2, uub = uk & 3, uubx = uub & 1, uuby = uub >> 1;
        const int base = upl ? VOFF : UOFF;
        const P4 usrc = ld4(c.yin + base + 4 * uuby * BPS + 4 * uubx);
        const P4 upred = predsq_p(check_mode(mbx, mby, um), c.yout + base, 8, 4 * uubx, 4 * uuby);
        Q16 uq;
        int unz;
        {
          int co[16];
          fdct_p(usrc, upred, co);
          unz = quantize(co, uq, sg.uv, 0);
        }
        // left / top block of the same plane (only read when ubx / uby > 0): DPP row shifts
        const int unzl = __builtin_amdgcn_update_dpp(0, unz, 0x111, 0xf, 0xf, false);  // row_shr:1
        const int unzt = __builtin_amdgcn_update_dpp(0, unz, 0x112, 0xf, 0xf, false);  // row_shr:2
        const int ul_ = uubx > 0 ? (unzl > 0) : (int)((left_nz >> (4 + 2 * upl + uuby)) & 1);
        const int ut_ = uuby > 0 ? (unzt > 0) : (int)((top_nz >> (4 + 2 * upl + uubx)) & 1);
        const int urate = token_cost(t, uq, unz, 2, min(ul_ + ut_, 2), 0);
        int dq[16];
        dequant(uq, dq, sg.uv);
        const int usse = sse_p(usrc, recon_p(upred, dq));
        int uacn = 0;
#pragma unroll
        for (int i = 1; i < 16; i++) uacn += uq.get(i) != 0;
        const int ursum = group_sum_first<8>(urate), ussum = group_sum_first<8>(usse), uasum = group_sum_first<8>(uacn);  // lane uk == 0
        if (lane < 32 && uk == 0) {
          int total = vp8_mode_fixed_cost_uv[um] + ursum;
          if (um > 0 && uasum <= 2) total += 140 * 8;
          s.uv_rate[um] = total;
          s.uv_disto[um] = ussum;
        }
      }
      lds_sync();
      {
        uint64_t best = ~0ull;
        for (int mm = 0; mm < 4; mm++) {
          if ((mm == 2 && mby == 0) || (mm == 3 && mbx == 0) || (mm == 1 && (mbx == 0 || mby == 0))) continue;
          const uint64_t sc = rd_score(s.uv_disto[mm], s.uv_rate[mm], sg.lambda_uv);
          if (sc < best) {
            best = sc;
            best_uv = mm;
          }
        }
      }
      int rate16 = 0, disto16 = 0;
      {
        uint64_t best = ~0ull;
        for (int mm = 0; mm < 4; mm++) {
          if ((mm == 2 && mby == 0) || (mm == 3 && mbx == 0) || (mm == 1 && (mbx == 0 || mby == 0))) continue;
          const uint64_t sc = rd_score(s.mode_disto[mm], s.mode_rate[mm], sg.lambda_i16);
          if (sc < best) {
            best = sc;
            best16 = mm;
            rate16 = s.mode_rate[mm];
            disto16 = s.mode_disto[mm];
          }
        }
      }
      s16 = rd_score(disto16, rate16, sg.lambda_mode);
      WG_REP_END
      if constexpr (PAIR) {  // for A's early exit: the score, then the flag
        if (lane == 0) {
          *reinterpret_cast<volatile uint64_t*>(&c.s16v) = s16;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          *reinterpret_cast<volatile int*>(&c.s16_flag) = 1;
        }
      }
      }  // isB

      ESTAMP(3);
      uint64_t s4 = ~0ull;
      if (isA) {
      __builtin_amdgcn_s_setprio(2);
      // ================= I4 RD (tryI4ModesRDParallel :739-846) =================
      // The 16 blocks run as a wavefront, step st = bx + 2 by: a block's left,
      // top and top-right neighbours (the LD/VL context) all finish in earlier
      // steps, so the (up to) two blocks of a step run at once, one per
      // half-wave.  The reference's raster-order early exit (:820-833) is
      // applied afterwards from the per-block results: a block reads only
      // reconstructions of raster-earlier blocks, so every block evaluated
      // before the exit point sees exactly the reference's inputs.
      if constexpr (!PAIR) {  // (PAIR: copied before the pair's barrier)
#pragma unroll
        for (int k = 0; k < (YUV / 4 + 63) / 64; k++) {
          const int i = lane + 64 * k;
          if (i < YUV / 4) reinterpret_cast<uint32_t*>(s.yout2)[i] = reinterpret_cast<const uint32_t*>(s.yout)[i];
        }
      }
      WG_REP_BEGIN(I4)
      if constexpr (TRELLIS) trellis_r0<3>(t, lane, sg.tlambda_i4 * 16, s.r0, s.eobl);
      lds_sync();
      {
        // running totals over the finished blocks: rate, distortion and header
        // bits only grow, so once the finished blocks alone reach the exit
        // condition the reference exits too (at some block) and I4 loses
        int run_rate = 0, run_disto = 0, run_header = 0;
        bool early = false;
        for (int st = 0; st < 10 && !early; st++) {
          Shared& s = launder(s_waves[wave]);
          Tables& t = launder(t_lds);
          const int lane = opaque_lane();
          if (st == 3) {
            // the top-right context of block 3 (MB x+1 of the row above, or
            // its last top pixel repeated at the right edge; 127 on the first
            // row from the context fill) and its copies beside rows 3, 7, 11
            // for blocks 7, 11, 15 (fillPredContextParallel :455-562)
            if (mby > 0) {
              // (granule 0 of column x + 1: word 0, the Y bottom row's pixels 0-3)
              const uint32_t trn = mbx < mbw - 1 ? (uint32_t)__builtin_amdgcn_readfirstlane(
                                                       (int)poll_rec(top + (mbx + 1) * REC, 1))
                                                 : 0u;
              if (lane == 0) {
                const uint32_t tr = mbx < mbw - 1 ? trn : 0x01010101u * s.yout2[YOFF - BPS + 15];
                *reinterpret_cast<uint32_t*>(s.yout2 + YOFF - BPS + 16) = tr;
              }
              lds_sync();
            }
            if (lane < 12) {
              const int r = 4 * (lane / 4 + 1) - 1, i = lane & 3;
              s.yout2[YOFF - BPS + 16 + (r + 1) * BPS + i] = s.yout2[YOFF - BPS + 16 + i];
            }
            lds_sync();
          }
          const int half = lane >> 5, hl = lane & 31;
          const int wy = (st <= 3 ? 0 : (st - 2) >> 1) + half, wx = st - 2 * wy;
          const bool bvalid = wy <= 3 && wx >= 0 && wx <= 3;
          const int by4 = bvalid ? wy : 0, bx4 = bvalid ? wx : 0;  // an idle half works on block 0 (discarded)
          const int blk = by4 * 4 + bx4;
          const int top_mode = by4 == 0 ? (int)((top_modes >> (8 * bx4)) & 0xff) : s.modes4[max(blk - 4, 0)];
          const int left_mode = bx4 == 0 ? (int)((left_modes >> (8 * by4)) & 0xff) : s.modes4[max(blk - 1, 0)];
          const int off = YOFF + 4 * by4 * BPS + 4 * bx4;
          const bool has_top = mby > 0 || by4 > 0, has_left = mbx > 0 || bx4 > 0;
          const int l = bx4 > 0 ? (s.nzy[max(blk - 1, 0)] > 0) : (int)((left_nz >> by4) & 1);
          const int tp = by4 > 0 ? (s.nzy[max(blk - 4, 0)] > 0) : (int)((top_nz >> bx4) & 1);
          const int nz_ctx = min(l + tp, 2);
          int src[16];
          load4x4(s.yin + off, src);
          SSTAMP(-1);
          // pre-screen all eligible modes by prediction SSE (lanes 0-9 of each half)
          int sse_lane = 0;
          // (FUSE) every pre-screen lane also transforms its mode's residual:
          // the candidates are among these lanes, so their coefficients come
          // without a second prediction pass (its 17 LDS reads) after the pick
          constexpr bool FUSE = TRELLIS;
          int pco[FUSE ? 16 : 1];
      WG_REP_BEGIN(PRE)
          // two lanes a mode (round 6): lane m (the half's first DPP row)
          // takes rows 0-1 of mode m's residual, lane m + 16 rows 3-2; each
          // makes the SSE of its rows and the row pass of its pair, the pairs
          // trade halves with one v_permlane16_swap (rows of 16 lanes), and
          // each lane finishes two columns of the FTransform (columns 2 part,
          // 2 part + 1).  Half the LDS reads and transform work on the step's
          // chain: 156.5k -> 151.2k cycles a macroblock (stamped build), the
          // isolated 64 x 1080p launch 20.1-20.3 -> 19.7-19.8 ms
          const int pm_mode = hl & 15, part = hl >> 4;
          const uint2 pcw2 = *reinterpret_cast<const uint2*>(&t.pcode[min(pm_mode, 9)][8 * part]);
          pred4_values(s.yout2, off, hl, s.pv[half]);
          lds_sync();
          if (bvalid && pm_mode < 10) {
            // this lane's two rows: part 0 rows 0, 1; part 1 rows 3, 2 (the
            // packed FTransform's (3, 2) pair order)
            const uint32_t ca = part ? pcw2.y : pcw2.x, cb = part ? pcw2.x : pcw2.y;
            const int ra = part ? 3 : 0, rb = part ? 2 : 1;
            wg::s16x2_t d[4];
            int sse = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
              const int pa = s.pv[half][(ca >> (8 * k)) & 0xff], pb = s.pv[half][(cb >> (8 * k)) & 0xff];
              const int da = src[4 * ra + k] - pa, db = src[4 * rb + k] - pb;
              sse += da * da + db * db;
              d[k] = (wg::s16x2_t){(short)da, (short)db};
            }
            wg::s16x2_t T[4];
            wg::fdct4x4_rowpair(d, T);  // part 0: P = rows (0, 1); part 1: Q = rows (3, 2)
            // the partner's SSE and the two row-pass pairs of this lane's columns
            auto other = [&](uint32_t v) {
              const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
              return part ? r[0] : r[1];
            };
            sse_lane = sse + (int)other((uint32_t)sse);
            const uint32_t x0 = __builtin_bit_cast(uint32_t, part ? T[0] : T[2]);
            const uint32_t x1 = __builtin_bit_cast(uint32_t, part ? T[1] : T[3]);
            const wg::s16x2_t R0 = __builtin_bit_cast(wg::s16x2_t, other(x0));
            const wg::s16x2_t R1 = __builtin_bit_cast(wg::s16x2_t, other(x1));
            const wg::s16x2_t one = {1, 1}, pmv = {1, -1}, k4 = {5352, 2217}, k12 = {2217, -5352};
#pragma unroll
            for (int j = 0; j < 2; j++) {
              const wg::s16x2_t Pc = part ? (j ? R1 : R0) : T[j];
              const wg::s16x2_t Qc = part ? T[2 + j] : (j ? R1 : R0);
              const wg::s16x2_t S = Pc + Qc, D = Pc - Qc;  // (a0, a1), (a3, a2)
              pco[j] = (int16_t)(wg::sdot2_acc(S, one, 7) >> 4);                                // row 0
              pco[4 + j] = (int16_t)((wg::sdot2_acc(D, k4, 12000) >> 16) + (D.x != 0));          // row 1
              pco[8 + j] = (int16_t)(wg::sdot2_acc(S, pmv, 7) >> 4);                             // row 2
              pco[12 + j] = (int16_t)(wg::sdot2_acc(D, k12, 51000) >> 16);                        // row 3
            }
          }
      WG_REP_END
          SSTAMP(0);
          // eligible modes (no top / no left context rules out some), candidates
          uint32_t eligible = 0x3ff;
          if (!has_top) eligible &= ~0x1f6u;  // TM VE RD VR LD VL HD need the top row
          if (!has_left) eligible &= ~0x31au;  // TM HE RD HD HU need the left column
          const int K = bvalid ? min(max_modes, __builtin_popcount(eligible)) : 0;
          int cm[3];
          // (both DPP rows of the half hold every mode's total SSE, at lane
          // mode and mode + 16: each row's minimum search gives the same cm[])
          select_i4_modes(sse_lane, hl & 15, eligible, K, cm);
          const bool cand = bvalid && hl < K;
          const int mode = pick3(hl, cm[0], cm[1], cm[2]);
          const int slot = half * 3 + min(hl, 2);  // candidate slot in the trellis / level buffers
          // (HOIST) the reconstruction quad's prediction and source rows (lane
          // 4c + r: row r of candidate c), read now: the reads overlap the
          // trellis instead of sitting on the chain after it
          const int qc = min(hl >> 2, 2), qr = hl & 3, qsl = half * 3 + qc;
          const int qmode = min(pick3(qc, cm[0], cm[1], cm[2]) & 15, 9);
          uint32_t pred_row = 0, src_row = 0;
          const int hdr_h = t.fixed_i4[(top_mode * 10 + left_mode) * 10 + qmode];  // the mode's header bits
          {
            const uint32_t cw = reinterpret_cast<const uint32_t*>(t.pcode[qmode])[qr];
            int pr[4];
#pragma unroll
            for (int k = 0; k < 4; k++) pr[k] = s.pv[half][(cw >> (8 * k)) & 0xff];
            pred_row = pack4(pr[0], pr[1], pr[2], pr[3]);
            src_row = *reinterpret_cast<const uint32_t*>(s.yin + off + qr * BPS);
          }
          SSTAMP(1);
          CSTAMP(-1);
          // candidates: prediction + transform (lane hl = candidate hl)
      WG_REP_BEGIN(CAND)
          if constexpr (FUSE) {  // the lane of mode cm[c] stores candidate c's coefficients
            // (both lanes of the mode: columns 2 part, 2 part + 1 of each row)
            const int pm = hl & 15, pp = hl >> 4;
            const int c = (K > 0 && cm[0] == pm) ? 0 : ((K > 1 && cm[1] == pm) ? 1 : ((K > 2 && cm[2] == pm) ? 2 : 3));
            if (bvalid && pm < 10 && c < 3) {
#pragma unroll
              for (int i = 0; i < 4; i++)
                *reinterpret_cast<uint32_t*>(&s.co_buf[half * 3 + c][4 * i + 2 * pp]) = pack16(pco[4 * i], pco[4 * i + 1]);
            }
          } else if (cand) {
            int pred[16], co[16];
            pred4_lut(t.pcode[mode], s.pv[half], pred);
            fdct(src, pred, co);
            if constexpr (TRELLIS) {
#pragma unroll
              for (int i = 0; i < 4; i++) st_co4(&s.co_buf[slot][4 * i], co + 4 * i);
            } else {  // method 3: QuantizeCoeffs (pickBestI4ModeRDParallel :890)
              int16_t q[16];
              s.cand_nz[slot] = quantize(co, q, sg.y1, 0);
#pragma unroll
              for (int i = 0; i < 16; i++) s.cand_q[slot][i] = q[i];
            }
          }
      WG_REP_END
          lds_sync();
          CSTAMP(0);
          // (TRELLIS + TAIL) the candidate's nz count and rate, straight from
          // the DP into the reconstruction quad's registers (the same lanes)
          int dp_nz = 0, dp_rate = 0;
          if constexpr (TRELLIS) {
          // trellis positions: lane (candidate c, pair pp) prepares positions 2pp, 2pp + 1
          const int lam16 = sg.tlambda_i4 * 16;
          bool pnz = false;
      WG_REP_BEGIN(PREP)
          if (bvalid && hl < 8 * K) {
            const int c = hl >> 3, n0 = 2 * (hl & 7), sl = half * 3 + c;
            // both positions into registers first, then stored: their table
            // reads issue together instead of waiting behind the first one's stores
            TRec rr[2];
            int l0[2];
            pnz = trellis_prep2<3, 0>(t, s.co_buf[sl], n0, sg.y1, lam16, rr, l0);
#pragma unroll
            for (int j = 0; j < 2; j++) {
              s.trec[sl][n0 + j] = rr[j];
              s.l0s[sl][n0 + j] = l0[j];
            }
          }
      WG_REP_END
          const uint64_t pnz_mask = __ballot(pnz);
          lds_sync();
          CSTAMP(1);
          DSTAMP(-1);
          // the trellis DP: one lane quad per candidate (lane 4c + k owns end context k)
          if (bvalid && hl < 4 * K) {
            const int c = hl >> 2, sl = half * 3 + c;
            if ((pnz_mask >> (32 * half + 8 * c)) & 0xff) {
              // the DP is the step's serial chain: let it win issue arbitration
              // against the SIMD's other wave while it runs
              __builtin_amdgcn_s_setprio(3);
      WG_REP_BEGIN(DP)
              trellis_dp4t<0, 3>(t, s.trec[sl], s.r0, s.l0s[sl], nz_ctx, lam16, hl & 3, s.cand_q[sl], &dp_nz,
                                 &dp_rate);
      WG_REP_END
              __builtin_amdgcn_s_setprio(2);
            } else {
              dp_nz = 0;
              dp_rate = t.tok[3 * 8].eob[nz_ctx];  // EOB at position 0
              if ((hl & 3) == 0) {
#pragma unroll
                for (int i = 0; i < 16; i++) s.cand_q[sl][i] = 0;
                s.cand_nz[sl] = 0;
              }
            }
          }
          lds_sync();
          DSTAMP(0);
          }  // TRELLIS
          // candidates: reconstruction + distortion on the candidate's lane quad
          // (lane 4c + r owns row r; the TDisto column pass reads the row pass
          // results back from LDS; sums are quad reductions)
          const bool qact = bvalid && hl < 4 * K;
          // (qc, qr, qsl, qmode above: unconditional, so that the
          // reconstruction, TDisto and token-cost streams interleave: lanes past
          // the candidates repeat candidate 2's work, or work on an unused
          // slot, and nothing reads their results)
          // (TAIL) the trellis DP leaves each candidate's rate in dp_rate, and
          // the inverse DCT's vertical pass runs one column a quad lane,
          // transposed across the quad by DPP: 4 levels and 4 products a lane
          // instead of 16 and 16
          constexpr bool TAIL = TRELLIS;
          int16_t qv[TAIL ? 1 : 16];
          int tcol[4];  // (TAIL) column qr of the row pass: reconstruction | source << 16
          int qnz = 0, sse_r = 0, cnt = 0;
          uint32_t rec_row = 0;
          int part = 0;  // token cost, lane-parallel over positions: lane 8c + p takes positions 2p, 2p + 1
          if constexpr (!TAIL) {
            const int c = min(hl >> 3, 2), n0 = 2 * (hl & 7), sl = half * 3 + c;
            const int nzc = s.cand_nz[sl];
            part = token_cost_pos<3>(t, s.cand_q[sl], n0, nzc, nz_ctx, 0) + token_cost_pos<3>(t, s.cand_q[sl], n0 + 1, nzc, nz_ctx, 0);
          }
          {
            int res[4], pr[4], sr[4], rr[4];
            qnz = TRELLIS ? dp_nz : s.cand_nz[qsl];
            if constexpr (TAIL) {
              // column qr: levels qr, 4 + qr, 8 + qr, 12 + qr (raster)
              const int16_t* cq = s.cand_q[qsl];
              int col[4];
#pragma unroll
              for (int j = 0; j < 4; j++) col[j] = cq[4 * j + qr];
              const int2 qq = make_int2(sg.y1.quant, sg.y1.dc_quant);
              int dc[4];
#pragma unroll
              for (int j = 0; j < 4; j++) dc[j] = (int16_t)wg::mul_i24(col[j], (j == 0 && qr == 0) ? qq.y : qq.x);
              cnt = (col[0] != 0 && qr != 0) + (col[1] != 0) + (col[2] != 0) + (col[3] != 0);
              cnt = quad_sum(cnt);  // levels 1..15 that are nonzero
              // the vertical pass of transforms.go:37-136 for column qr: rows 0..3
              int tv[4];
              {
                const int a = dc[0] + dc[2], b = dc[0] - dc[2];
                const int cc = mul2_16(dc[1]) - mul1_16(dc[3]);
                const int d = mul1_16(dc[1]) + mul2_16(dc[3]);
                tv[0] = a + d;
                tv[1] = b + cc;
                tv[2] = b - cc;
                tv[3] = a - d;
              }
              quad_transpose(tv);  // lane qr: row qr's four column outputs
              const int d0 = tv[0] + 4;
              const int a = d0 + tv[2], b = d0 - tv[2];
              const int cc = mul2_24(tv[1]) - mul1_24(tv[3]);
              const int d = mul1_24(tv[1]) + mul2_24(tv[3]);
              res[0] = (a + d) >> 3;
              res[1] = (b + cc) >> 3;
              res[2] = (b - cc) >> 3;
              res[3] = (a - d) >> 3;
            } else {
              int dq[16];
#pragma unroll
              for (int i = 0; i < 16; i++) qv[i] = s.cand_q[qsl][i];
              dequant(qv, dq, sg.y1);
              idct_row(dq, qr, res);
            }
#pragma unroll
            for (int k = 0; k < 4; k++) pr[k] = (pred_row >> (8 * k)) & 0xff;
#pragma unroll
            for (int k = 0; k < 4; k++) {
              sr[k] = (src_row >> (8 * k)) & 0xff;
              rr[k] = clip8(pr[k] + res[k]);
              sse_r += (sr[k] - rr[k]) * (sr[k] - rr[k]);
            }
            rec_row = pack4(rr[0], rr[1], rr[2], rr[3]);
            // tTransform row pass (ssim.go:266-304) of the reconstruction and the source
            int16_t* th = &s.co_buf[2 * qsl][0] + 8 * qr;  // co_buf is free again after the trellis prep
            int4 tr = make_int4(0, 0, 0, 0), ts = tr;
            if constexpr (TAIL) {
              // reconstruction and source as the two int16 halves of one word
              // through both passes (|values| <= 4080): the row pass, then the
              // column pass's inputs by a quad transpose
              const s16x2 p0 = {(short)rr[0], (short)sr[0]}, p1 = {(short)rr[1], (short)sr[1]};
              const s16x2 p2 = {(short)rr[2], (short)sr[2]}, p3 = {(short)rr[3], (short)sr[3]};
              const s16x2 a0 = p0 + p2, a1 = p1 + p3, a2 = p1 - p3, a3 = p0 - p2;
              int pk[4] = {as_int(a0 + a1), as_int(a3 + a2), as_int(a3 - a2), as_int(a0 - a1)};
              quad_transpose(pk);
#pragma unroll
              for (int j = 0; j < 4; j++) tcol[j] = pk[j];
            } else {
              {
                const int a0 = rr[0] + rr[2], a1 = rr[1] + rr[3], a2 = rr[1] - rr[3], a3 = rr[0] - rr[2];
                tr = make_int4(a0 + a1, a3 + a2, a3 - a2, a0 - a1);
              }
              {
                const int a0 = sr[0] + sr[2], a1 = sr[1] + sr[3], a2 = sr[1] - sr[3], a3 = sr[0] - sr[2];
                ts = make_int4(a0 + a1, a3 + a2, a3 - a2, a0 - a1);
              }
            }
            if (!TAIL && qact) {
              reinterpret_cast<uint2*>(th)[0] = make_uint2(pack16(tr.x, tr.y), pack16(tr.z, tr.w));  // |values| <= 1020
              reinterpret_cast<uint2*>(th)[1] = make_uint2(pack16(ts.x, ts.y), pack16(ts.z, ts.w));
            }
            if constexpr (!TAIL) {
#pragma unroll
              for (int i = 1; i < 16; i++) cnt += qv[i] != 0;
            }
          }
          if constexpr (!TAIL) lds_sync();
          int wrec = 0, wsrc = 0;  // weighted column sums of column qr
          if constexpr (TAIL) {
            // the column pass on the packed pairs, then sum_j w_j (|rec_j| - |src_j|)
            // as one signed dot product a coefficient with (w_j, -w_j): the
            // TDisto difference of the quad's sums is the sum of these
            const s16x2 c0 = as_s16x2(tcol[0]), c1 = as_s16x2(tcol[1]), c2 = as_s16x2(tcol[2]), c3 = as_s16x2(tcol[3]);
            const s16x2 a0 = c0 + c2, a1 = c1 + c3, a2 = c1 - c3, a3 = c0 - c2;
            const s16x2 o[4] = {a0 + a1, a3 + a2, a3 - a2, a0 - a1};
            // kWeightY (ssim.go:257) column qr, one byte per row
            const uint32_t wcol = qr == 0 ? 0x09142026u : (qr == 1 ? 0x07111c20u : (qr == 2 ? 0x040a1114u : 0x02040709u));
#pragma unroll
            for (int j = 0; j < 4; j++) {
              const short w = (short)((wcol >> (8 * j)) & 0xff);
              const s16x2 m = __builtin_elementwise_max(o[j], -o[j]);
              wrec = __builtin_amdgcn_sdot2(m, (s16x2){w, (short)-w}, wrec, false);
            }
          } else {
            int cr[4], cs[4];
            {
              const int16_t* tx = &s.co_buf[2 * qsl][0];
#pragma unroll
              for (int j = 0; j < 4; j++) {
                cr[j] = tx[8 * j + qr];
                cs[j] = tx[8 * j + 4 + qr];
              }
            }
            // kWeightY (ssim.go:257) column qr, one byte per row
            const uint32_t wcol = qr == 0 ? 0x09142026u : (qr == 1 ? 0x07111c20u : (qr == 2 ? 0x040a1114u : 0x02040709u));
            const int w0 = wcol & 0xff, w1 = (wcol >> 8) & 0xff, w2 = (wcol >> 16) & 0xff, w3 = wcol >> 24;
            {
              const int a0 = cr[0] + cr[2], a1 = cr[1] + cr[3], a2 = cr[1] - cr[3], a3 = cr[0] - cr[2];
              wrec = w0 * abs(a0 + a1) + w1 * abs(a3 + a2) + w2 * abs(a3 - a2) + w3 * abs(a0 - a1);
            }
            {
              const int a0 = cs[0] + cs[2], a1 = cs[1] + cs[3], a2 = cs[1] - cs[3], a3 = cs[0] - cs[2];
              wsrc = w0 * abs(a0 + a1) + w1 * abs(a3 + a2) + w2 * abs(a3 - a2) + w3 * abs(a0 - a1);
            }
          }
          const int sse_q = quad_sum(sse_r), wrec_q = quad_sum(wrec), wsrc_q = TAIL ? 0 : quad_sum(wsrc);
          int disto = sse_q;
          if (sg.tlambda_sd > 0) disto += (sg.tlambda_sd * (abs(wrec_q - wsrc_q) >> 5) + 128) >> 8;
          CSTAMP(2);
          // the token cost summed over each candidate's 8 lanes: candidate c's
          // rate sits in lane 32 * half + 8c; read the six with
          // v_readlane (wave-uniform lanes) instead of LDS permutes
          int tok_rate;
          if constexpr (TAIL) {
            tok_rate = dp_rate;
          } else {
            part = group_sum_first<8>(part);
            const int r00 = __builtin_amdgcn_readlane(part, 0), r01 = __builtin_amdgcn_readlane(part, 8);
            const int r02 = __builtin_amdgcn_readlane(part, 16), r10 = __builtin_amdgcn_readlane(part, 32);
            const int r11 = __builtin_amdgcn_readlane(part, 40), r12 = __builtin_amdgcn_readlane(part, 48);
            tok_rate = half ? pick3(qc, r10, r11, r12) : pick3(qc, r00, r01, r02);
          }
          uint64_t score = ~0ull;
          int rate = 0, hdr = 0;
          if (qact) {
            hdr = hdr_h;
            rate = (qmode > 0 && cnt <= 3) ? 140 : 0;
            rate += tok_rate + hdr;
            score = rd_score(disto, rate, sg.lambda_i4);
          }
          CSTAMP(3);
          SSTAMP(2);
          // first minimum over this half's candidates (strict '<' in candidate
          // order): candidate c's score sits in lane 32 * half + 4c, i.e. lane
          // 4c of the half's first DPP row, broadcast to the row
          int win = 0;
          {
            const uint64_t sc0 = row_bcast64<0>(score), sc1 = row_bcast64<4>(score), sc2 = row_bcast64<8>(score);
            uint64_t wsc = sc0;
            if (1 < K && sc1 < wsc) {
              wsc = sc1;
              win = 1;
            }
            if (2 < K && sc2 < wsc) win = 2;
          }
          if (qact && qc == win) {  // the winning quad: row qr of the reconstruction, 4 levels each
            *reinterpret_cast<uint32_t*>(s.yout2 + off + qr * BPS) = rec_row;
            // levels 4qr..4qr+3 straight from the candidate's LDS row (a
            // lane-varying index into qv[] would be a 16-way select)
            *reinterpret_cast<uint2*>(s.coeffs + blk * 16 + 4 * qr) = *reinterpret_cast<const uint2*>(&s.cand_q[qsl][4 * qr]);
            if (qr == 0) {
              s.modes4[blk] = (uint8_t)qmode;
              s.nzy[blk] = (uint8_t)qnz;
            }
          }
          {
            // the winners' rate, distortion and header bits, read from their
            // lanes (the half's winner index is uniform over the half)
            const int w0 = 4 * __builtin_amdgcn_readfirstlane(win);
            run_rate += __builtin_amdgcn_readlane(rate, w0);
            run_disto += __builtin_amdgcn_readlane(disto, w0);
            run_header += __builtin_amdgcn_readlane(hdr, w0);
            if (st >= 2 && st <= 7) {  // half 1 holds a block
              const int w1 = 32 + 4 * __builtin_amdgcn_readlane(win, 32);
              run_rate += __builtin_amdgcn_readlane(rate, w1);
              run_disto += __builtin_amdgcn_readlane(disto, w1);
              run_header += __builtin_amdgcn_readlane(hdr, w1);
            }
            uint64_t s16_now = s16;
            if constexpr (PAIR) {  // B's I16 score once posted (no exit before)
              s16_now = ~0ull;
              if (*reinterpret_cast<volatile int*>(&s.s16_flag)) s16_now = *reinterpret_cast<volatile uint64_t*>(&s.s16v);
              s16_now = uniform64(s16_now);
            }
            early = rd_score(run_disto, run_rate + 211, sg.lambda_mode) >= s16_now || run_header > 15000;
          }
          lds_sync();
          SSTAMP(3);
        }
        s4 = early ? ~0ull : rd_score(run_disto, run_rate + 211, sg.lambda_mode);
      }
      WG_REP_END
      __builtin_amdgcn_s_setprio(1);
      }  // isA
      bool is_i4 = s4 < s16;  // (PAIR: decided at the join)

      ESTAMP(4);
      // ================= predictions into yout (pickBestModeParallel :586-604) =================
      // (the square predictors read only the borders, so lanes write their blocks directly)
      // PAIR: B runs the I16 residuals (and reconstruction) whatever A's I4 RD
      // decides; A keeps them at the join if I16 wins
      const bool run16 = PAIR || !is_i4;
      uint32_t nzy_mask = 0, nzuv_mask = 0;
      int nz_dc = 0, dc_rec = 0;  // dc_rec: lane b's reconstructed DC (I16)
      if (isB) {
      if (!PAIR && is_i4) {  // I4 reconstruction from the RD pass (I4Cached)
        if (lane < 16)
          *reinterpret_cast<uint4*>(c.yout + YOFF + lane * BPS) = *reinterpret_cast<const uint4*>(s.yout2 + YOFF + lane * BPS);
        else if (lane < 32)
          s.coeffs[384 + lane - 16] = 0;  // no WHT block for I4
      } else if (run16 && lane < 16) {
        int p[16];
        predsq_block(check_mode(mbx, mby, best16), c.yout + YOFF, 16, 4 * bx, 4 * by, p);
        store4x4(c.yout + YOFF + 4 * by * BPS + 4 * bx, p);
      }
      if (lane >= 32 && lane < 40) {
        const int k = lane - 32, pl = k >> 2, ub = k & 3;
        int p[16];
        predsq_block(check_mode(mbx, mby, best_uv), c.yout + (pl ? VOFF : UOFF), 8, 4 * (ub & 1), 4 * (ub >> 1), p);
        store4x4(c.yout + (pl ? VOFF : UOFF) + 4 * (ub >> 1) * BPS + 4 * (ub & 1), p);
      }
      lds_sync();

      ESTAMP(5);
      // ================= final residuals (encodeResidualsParallel :1166-1356) =================
      WG_REP_BEGIN(FIN)
      if (run16) {
        int dc_nz = 0;
        if (lane < 16) {
          const int off = YOFF + 4 * by * BPS + 4 * bx;
          int src[16], pred[16], co[16];
          load4x4(c.yin + off, src);
          load4x4(c.yout + off, pred);
          fdct(src, pred, co);
          if constexpr (TRELLIS) {
#pragma unroll
            for (int i = 0; i < 4; i++) st_co4(&s.co_buf[lane][4 * i], co + 4 * i);  // ([0], the DC, is not read)
          } else {  // method 3: the AC levels by QuantizeCoeffs (encodeI16ResidualsParallel :1215)
            int16_t q[16];
            s.nzy[lane] = (uint8_t)quantize(co, q, sg.y1, 1);
#pragma unroll
            for (int i = 0; i < 16; i++) s.coeffs[lane * 16 + i] = q[i];
          }
          // the Y2 block, lane-parallel over lanes 0..15
          int dcq = 0, dccost = 0;
          dc_rec = dc_block_lane(t, co[0], lane, sg.y2, 0, &dcq, &dc_nz, &dccost);
          s.coeffs[384 + lane] = (int16_t)dcq;
        }
        nz_dc = __builtin_amdgcn_readfirstlane(dc_nz);
        lds_sync();
        if constexpr (TRELLIS) {
        // Trellis of the 16 AC blocks.  A block's DP depends on its left / top
        // neighbours' nz only through its initial context min(l + t, 2), so
        // it is run speculatively for every context the block can still get
        // (1 for block 0, 2 along the MB's top row / left column, 3 inside):
        // three rounds of up to six blocks (their position records fit the
        // six trellis slots) and up to 16 DPs, one per lane quad, each
        // followed by the reference's raster-order resolution of the actual
        // contexts.  (Walking the 7 block diagonals took 7 prep + DP rounds.)
        const int lam16 = sg.tlambda_i16 * 16;
        trellis_r0<0>(t, lane, lam16, s.r0, s.eobl);  // (read after the first round's lds_sync)
        // One round (WG_ENC_I16ONE): quad q runs block q's DP for all three
        // start contexts at once (dp3_walk), over the records of positions
        // 0..7, then (the same LDS, rewritten) 8..15; lane 4q + r preps
        // positions 2r, 2r + 1 of each half.  Then the raster-order
        // resolution on scalars, and each quad writes its block's levels for
        // the context it resolved to.  Measured against the three rounds of
        // up to 16 speculative DPs below: see DESIGN.md (round 5).
        //
        // Positions with no non-zero level candidate (thresh < 1: the
        // prep's `cap`) contribute only level-0 transitions into context
        // 0, so no terminal past them can win and the histories stay zero
        // there: a half with none in any block needs no walk, and an MB
        // with none at all is zero (the all-zero pre-scan says the same).
        // A pre-scan of the 16 blocks' caps decides both, wave-uniformly.
        {
          const int q = lane >> 2, r = lane & 3, e = min(r, 2);
          bool capl = false;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int n = 4 * r + j, zig = zig_of(n);
            const int c0 = max(abs((int)s.co_buf[q][zig]) + (int)sg.y1.sharpen[zig], 0);
            capl |= n >= 1 && wg::mul_i24(c0, sg.y1.iquant) >= 65536;
          }
          const uint64_t capm = __ballot(capl);
          const bool cap_hi = (capm & 0xCCCCCCCCCCCCCCCCull) != 0;  // lanes r = 2, 3: positions 8..15
          // (WG_ENC_QSKIP) by quarter: lanes r = 1 (positions 4..7), r = 3 (12..15)
          [[maybe_unused]] const bool cap_q1 = (capm & 0x2222222222222222ull) != 0,
                                      cap_q3 = (capm & 0x8888888888888888ull) != 0;
          uint64_t pnz_mask = 0;
          DP3 S;
          dp3_init(S, t, lam16, r);
          const int64_t* eobq = &s.eobl[0][(e == 2 ? 2 : 1) - 1];
#pragma unroll
          for (int half = 0; half < 2; half++) {
            if (capm == 0) break;  // (wave-uniform)
            // this lane's row at position n: R0 from the phase's table, R1 / R2
            // from the half's records (position n at record n - 8 half); the
            // terminal lane's (WG_ENC_TLANE) from the phase table's columns 3..5
            const int64_t* mine =
                (r == 3) ? &s.r0[0][3]
                : e == 0 ? &s.r0[0][0]
                         : reinterpret_cast<const int64_t*>(reinterpret_cast<const char*>(&s.trec16[q][0].x[e - 1][0]) -
                                                            8 * half * (int)sizeof(TRec));
            if (half == 1 && !cap_hi) {
              // (no candidates past position 7: one step more for the terminal
              // lane, the EOB after position 7; the context lanes' rows are stale)
              dp3_walk<8, 9>(S, mine, eobq);
              break;
            }
            {
              TRec rr[2];
              int l0[2];
              const int n0 = 8 * half + 2 * r;
              const bool pnz = trellis_prep2<0, 1>(t, s.co_buf[q], n0, sg.y1, lam16, rr, l0);
              pnz_mask |= __ballot(pnz);
#pragma unroll
              for (int k = 0; k < 2; k++) {
                if (n0 + k >= 1) s.trec16[q][2 * r + k] = rr[k];
                s.l0s16[q][n0 + k] = (int16_t)l0[k];
              }
            }
            lds_sync();
            if (half == 0) {
              dp3_walk<1, 8>(S, mine, eobq);
            } else {
                dp3_walk<8, 17>(S, mine, eobq);
            }
            lds_sync();  // (the second half's records overwrite the first's)
          }
          const uint32_t hs0 = dp3_hist(S, 0), hs1 = dp3_hist(S, 1), hs2 = dp3_hist(S, 2);
          // bit 4 q: block q's levels from start context s are non-zero (the
          // all-zero pre-scan: a block with no level at any position is zero)
          const bool bnz = ((pnz_mask >> (4 * q)) & 15) != 0;
          const uint64_t nzm0 = __ballot(r == 0 && bnz && hs0 != 0);
          const uint64_t nzm1 = __ballot(r == 0 && bnz && hs1 != 0);
          const uint64_t nzm2 = __ballot(r == 0 && bnz && hs2 != 0);
          // the reference's raster order, on scalars: block qb's context from
          // its left / top neighbours' resolved nz
          uint32_t nzbits = 0, ctxs = 0;
          for (int qb = 0; qb < 16; qb++) {
            const int qbx = qb & 3, qby = qb >> 2;
            const int l = qbx > 0 ? (int)((nzbits >> (qb - 1)) & 1) : (int)((left_nz >> qby) & 1);
            const int tp = qby > 0 ? (int)((nzbits >> (qb - 4)) & 1) : (int)((top_nz >> qbx) & 1);
            const int cx = min(l + tp, 2);
            const uint64_t nzm = cx == 0 ? nzm0 : (cx == 1 ? nzm1 : nzm2);
            nzbits |= (uint32_t)((nzm >> (4 * qb)) & 1) << qb;
            ctxs |= (uint32_t)cx << (2 * qb);
          }
          const int cq = (int)(ctxs >> (2 * q)) & 3;
          const uint32_t hist = !bnz ? 0u : (cq == 0 ? hs0 : (cq == 1 ? hs1 : hs2));
          const uint2 l0w = *reinterpret_cast<const uint2*>(&s.l0s16[q][4 * r]);
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int n = 4 * r + j;
            const int code = (int)((hist >> (2 * n)) & 3);
            const int ls = (int)(((j < 2 ? l0w.x : l0w.y) >> (16 * (j & 1))) & 0xffff);
            const int mag = code == 0 ? 0 : (ls >> 3) + code - 1;
            s.coeffs[q * 16 + zig_of(n)] = (int16_t)((ls & 4) ? -mag : mag);
          }
          if (r == 0) s.nzy[q] = (uint8_t)hist_nz(hist);
          lds_sync();
        }
        }  // TRELLIS
      }
      if (lane < 8) {  // chroma
        const int pl = lane >> 2, ub = lane & 3;
        const int off = (pl ? VOFF : UOFF) + 4 * (ub >> 1) * BPS + 4 * (ub & 1);
        int src[16], pred[16], co[16];
        int16_t q[16];
        load4x4(c.yin + off, src);
        load4x4(c.yout + off, pred);
        fdct(src, pred, co);
        const int nz = quantize(co, q, sg.uv, 0);
        s.nzuv[lane] = (uint8_t)nz;
#pragma unroll
        for (int i = 0; i < 16; i++) s.coeffs[(16 + lane) * 16 + i] = q[i];
      }
      lds_sync();
      WG_REP_END

      ESTAMP(6);
      // ================= reconstruction (reconstructMBParallel :1358-1410) =================
      if (run16) {
        if (lane < 16) {
          const int off = YOFF + 4 * by * BPS + 4 * bx;
          int16_t q[16];
          int dq[16], pred[16], rec[16];
#pragma unroll
          for (int i = 0; i < 16; i++) q[i] = s.coeffs[lane * 16 + i];
          dequant(q, dq, sg.y1);
          dq[0] = dc_rec;
          load4x4(c.yout + off, pred);
          recon4(pred, dq, rec);
          store4x4(c.yout + off, rec);
        }
      }
      if (lane >= 16 && lane < 24) {
        const int k = lane - 16, pl = k >> 2, ub = k & 3;
        const int off = (pl ? VOFF : UOFF) + 4 * (ub >> 1) * BPS + 4 * (ub & 1);
        int16_t q[16];
        int dq[16], pred[16], rec[16];
#pragma unroll
        for (int i = 0; i < 16; i++) q[i] = s.coeffs[(16 + k) * 16 + i];
        dequant(q, dq, sg.uv);
        load4x4(c.yout + off, pred);
        recon4(pred, dq, rec);
        store4x4(c.yout + off, rec);
      }
      lds_sync();
      if constexpr (PAIR) {
        if (lane == 0) {
          s.post_best16 = best16;
          s.post_best_uv = best_uv;
          s.post_nz_dc = nz_dc;
          s.post_s16 = s16;
        }
      }
      }  // isB
      if constexpr (PAIR) {
        // ---- the join: A keeps B's I16 residuals and reconstruction or its own I4 ones ----
        __syncthreads();
        if (isA) {
          const Shared& sb = launder(s_waves[1]);
          best16 = __builtin_amdgcn_readfirstlane(sb.post_best16);
          best_uv = __builtin_amdgcn_readfirstlane(sb.post_best_uv);
          s16 = uniform64(sb.post_s16);
          is_i4 = s4 < s16;
          nz_dc = is_i4 ? 0 : __builtin_amdgcn_readfirstlane(sb.post_nz_dc);
          const uint4* bq = reinterpret_cast<const uint4*>(sb.coeffs);  // 50 x 16 B
          uint4* cq = reinterpret_cast<uint4*>(s.coeffs);
          if (is_i4) {
            if (lane < 16)  // the I4 reconstruction (I4Cached)
              *reinterpret_cast<uint4*>(s.yout + YOFF + lane * BPS) = *reinterpret_cast<const uint4*>(s.yout2 + YOFF + lane * BPS);
            else if (lane < 32)  // chroma levels (coeffs[256..383] = 16-B pieces 32..47)
              cq[lane + 16] = bq[lane + 16];
            else if (lane < 48)
              s.coeffs[384 + lane - 32] = 0;  // no WHT block for I4
          } else {
            if (lane < 50) cq[lane] = bq[lane];  // luma, chroma and WHT levels
            else if (lane < 54) reinterpret_cast<uint32_t*>(s.nzy)[lane - 50] = reinterpret_cast<const uint32_t*>(sb.nzy)[lane - 50];
          }
          if (lane >= 56 && lane < 58) reinterpret_cast<uint32_t*>(s.nzuv)[lane - 56] = reinterpret_cast<const uint32_t*>(sb.nzuv)[lane - 56];
          lds_sync();
        }
      }
      if (isA) {
      // The hand-off record and the progress flag go first: the row below
      // waits on them (at its MB start and its I4 step 3), while the MBEncInfo
      // record and the reconstruction rows are outputs only and leave after.
      // NZ context update (updateNZContextParallel :343-430)
      uint32_t out_t, out_l;
      // (one LDS read a lane and three ballots: bit b of ym = luma block b's
      // levels past `first`, of uvm = chroma block b's; the reference's
      // shift-register walk then reduces to the blocks of the last row /
      // column: out_t = row 3's luma and row 1's U, V blocks, out_l = column
      // 3's / column 1's)
      {
        const int first = is_i4 ? 0 : 1;
        const int nzl = lane < 16 ? (int)s.nzy[lane] : (lane < 24 ? (int)s.nzuv[lane - 16] : 0);
        const uint32_t any = (uint32_t)__ballot(nzl > 0);
        const uint32_t ym = (uint32_t)__ballot(lane < 16 && nzl > first) & 0xffffu;
        nzy_mask = any & 0xffffu;
        nzuv_mask = (any >> 16) & 0xffu;
        const uint32_t uvm = nzuv_mask;
        out_t = (ym >> 12) | ((uvm >> 2) & 3u) << 4 | ((uvm >> 6) & 3u) << 6;
        out_l = ((ym >> 3) & 1u) | ((ym >> 6) & 2u) | ((ym >> 9) & 4u) | ((ym >> 12) & 8u) |
                (((uvm >> 1) & 1u) | ((uvm >> 2) & 2u)) << 4 | (((uvm >> 5) & 1u) | ((uvm >> 6) & 2u)) << 6;
      }
      if (!is_i4 && nz_dc > 0) nzy_mask |= 1u << 24;
      int new_top_dc = top_nz_dc;
      if (!is_i4) {
        new_top_dc = nz_dc > 0;
        left_nz_dc = nz_dc > 0;
      }
      uint32_t new_top_modes;
      if (is_i4) {
        new_top_modes = (uint32_t)s.modes4[12] | ((uint32_t)s.modes4[13] << 8) | ((uint32_t)s.modes4[14] << 16) |
                        ((uint32_t)s.modes4[15] << 24);
        left_modes = (uint32_t)s.modes4[3] | ((uint32_t)s.modes4[7] << 8) | ((uint32_t)s.modes4[11] << 16) |
                     ((uint32_t)s.modes4[15] << 24);
      } else {
        new_top_modes = 0;
        left_modes = 0;
      }
      left_nz = out_l;
      // hand-off record for the row below: lane i publishes word i with the
      // row's tag in one 64-bit store (no drain, no flag)
      if (mby < mbh - 1 && lane < REC_WORDS &&
          WG_CHK(top + mbx * REC + 8 * lane, 8, a.top, top_n, "k_encode_rows record store")) {
        uint32_t v;
        if (lane < 8) {
          const int so = lane < 4 ? YOFF + 15 * BPS + 4 * lane
                                  : (lane < 6 ? UOFF + 7 * BPS + 4 * (lane - 4) : VOFF + 7 * BPS + 4 * (lane - 6));
          v = *reinterpret_cast<const uint32_t*>(s.yout + so);
        } else {
          v = lane == 8 ? out_t : (lane == 9 ? new_top_modes : (uint32_t)new_top_dc);
        }
        st_granule(top + mbx * REC + 8 * lane, v, (uint32_t)mby + 1);
      }
      // ================= outputs, export, contexts (exportParallel :1412-1495) =================
      MbEnc* o = a.out + mbi;
      {  // the record's tail (bytes 800..863) staged next to the levels in LDS
        MbEnc* so = reinterpret_cast<MbEnc*>(s.coeffs);
        if (lane < 16) {
          so->modes[lane] = is_i4 ? s.modes4[lane] : 0;
          so->nz_y[lane] = s.nzy[lane];
        } else if (lane < 24) {
          so->nz_uv[lane - 16] = s.nzuv[lane - 16];
        } else if (lane == 24) {
          so->non_zero_y = nzy_mask;
          so->non_zero_uv = nzuv_mask;
          so->mb_type = is_i4 ? 1 : 0;
          so->i16_mode = is_i4 ? 0 : (uint8_t)best16;
          so->uv_mode = (uint8_t)best_uv;
          so->nz_dc = (uint8_t)nz_dc;
          so->skip = (nzy_mask == 0 && nzuv_mask == 0) ? 1 : 0;
          so->segment = (uint8_t)segid;
          so->pad0 = so->pad1 = 0;
          so->score = is_i4 ? s4 : s16;
        }
        lds_sync();
        // the whole 864-B record: 54 lanes x 16 B, one store instruction
        uint4* dst = reinterpret_cast<uint4*>(o);
        const uint4* srcv = reinterpret_cast<const uint4*>(s.coeffs);
        if (lane < 54 && WG_CHK(dst + lane, 16, a.out, mb_n * (int64_t)sizeof(MbEnc), "k_encode_rows MBEncInfo"))
          dst[lane] = srcv[lane];
      }
      {
        const int x = 16 * mbx, y = 16 * mby;
        const int wy = min(a.width - x, 16), hy = min(a.height - y, 16);
        // Rows leave in whole 32-B sectors where the MB pair (Y) / quad (U, V)
        // is whole: the earlier MBs' rows wait in registers (rst0 / rst1) and
        // go out back to back with the last one's, so L2 never writes a
        // partial sector back (a 16-B / 8-B piece per MB was written back
        // before the next MB's piece arrived).
        if (lane < hy && WG_CHK(RY + (int64_t)(y + lane) * ys + x - (wy == 16 && 16 * ((mbx & ~1) + 2) <= a.width ? 16 * (mbx & 1) : 0),
                                wy == 16 && 16 * ((mbx & ~1) + 2) <= a.width && (mbx & 1) ? 32 : 16, a.ry, y_n,
                                "k_encode_rows recon Y")) {
          const uint8_t* srow = s.yout + YOFF + lane * BPS;  // 8-B aligned in LDS
          uint8_t* drow = RY + (int64_t)(y + lane) * ys + x;
          if (wy == 16) {  // one 16-B store per row
            const uint2 lo = *reinterpret_cast<const uint2*>(srow), hi = *reinterpret_cast<const uint2*>(srow + 8);
            const uint4 v = make_uint4(lo.x, lo.y, hi.x, hi.y);
            if (16 * ((mbx & ~1) + 2) <= a.width) {
              if ((mbx & 1) == 0) {
                rst0 = v;
              } else {
                reinterpret_cast<uint4*>(drow)[-1] = rst0;
                *reinterpret_cast<uint4*>(drow) = v;
              }
            } else {
              *reinterpret_cast<uint4*>(drow) = v;
            }
          } else {
            for (int c = 0; c < wy; c++) drow[c] = srow[c];
          }
        }
        if (lane >= 16 && lane < 32 &&
            WG_CHK(((lane - 16) >> 3 ? RV : RU) + (int64_t)(8 * mby + ((lane - 16) & 7)) * uvs + 8 * (mbx & ~3), 8,
                   (lane - 16) >> 3 ? a.rv : a.ru, uv_n, "k_encode_rows recon UV") &&
            WG_CHK(((lane - 16) >> 3 ? RV : RU) + (int64_t)(8 * mby + ((lane - 16) & 7)) * uvs + 8 * mbx, 8,
                   (lane - 16) >> 3 ? a.rv : a.ru, uv_n, "k_encode_rows recon UV")) {  // U / V rows: 8 B each
          const int k = lane - 16, pl = k >> 3, j = k & 7;
          uint2* drow = reinterpret_cast<uint2*>((pl ? RV : RU) + (int64_t)(8 * mby + j) * uvs + 8 * mbx);
          const uint2 v = *reinterpret_cast<const uint2*>(s.yout + (pl ? VOFF : UOFF) + j * BPS);
          if (16 * ((mbx & ~3) + 4) <= a.width) {
            const int q = mbx & 3;
            if (q == 0) {
              rst0.x = v.x;
              rst0.y = v.y;
            } else if (q == 1) {
              rst0.z = v.x;
              rst0.w = v.y;
            } else if (q == 2) {
              rst1 = v;
            } else {
              drow[-3] = make_uint2(rst0.x, rst0.y);
              drow[-2] = make_uint2(rst0.z, rst0.w);
              drow[-1] = rst1;
              drow[0] = v;
            }
          } else {
            *drow = v;
          }
        }
      }
      // new top-left: the row above's bottom-right of this column (before we overwrite it)
      tl_y = s.yout[YOFF - BPS + 15];
      tl_u = s.yout[UOFF - BPS + 7];
      tl_v = s.yout[VOFF - BPS + 7];
      // rotate the left context: column 15 / 7 becomes column -1
      lds_sync();
      if (lane < 16) s.yout[YOFF - 1 + lane * BPS] = s.yout[YOFF + 15 + lane * BPS];
      else if (lane < 24) s.yout[UOFF - 1 + (lane - 16) * BPS] = s.yout[UOFF + 7 + (lane - 16) * BPS];
      else if (lane < 32) s.yout[VOFF - 1 + (lane - 24) * BPS] = s.yout[VOFF + 7 + (lane - 24) * BPS];
      if (lane < 16) s.nzy[lane] = 0;
      lds_sync();
      }  // isA
      ESTAMP(7);
    }
    WG_IF_ROWTIMES(
    if (live && (tid == 0 || (!PAIR && lane == 0))) {
      if (row < 16384) {
        g_row_times[row][0] = (unsigned long long)ro;
        g_row_times[row][1] = row_t0;
        g_row_times[row][2] = __builtin_amdgcn_s_memrealtime();
        g_row_times[row][3] = (unsigned long long)blockIdx.x << 8 | (unsigned long long)wave;
      }
    })
    // the band is done: LOOSE, count this wave out of it; else the group
    // dequeues the next one together
    if constexpr (LOOSE) {
      if (lane == 0) __hip_atomic_fetch_add(&s_done[q & 1], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      q++;
    } else if constexpr (!PAIR) {
      group_barrier(&s_gbar[grp], gen, lane);
    }
  }
  ESTAMP_FLUSH();
}

// Devices whose constant tables are uploaded: one bit per device, set under
// the mutex so host threads driving different devices do not race.
std::mutex g_tables_mu;
uint64_t g_tables_ready_mask = 0;

// VP8FixedCostsI4[top][left][mode] (computeFixedCostsI4,
// internal/lossy/encode_analysis.go:1498-1520): the mode tree walked with the
// VP8 bmode probabilities (i4ModeCost :1511).
void build_fixed_costs_i4(uint16_t* fixed) {
  for (int t = 0; t < 10; t++)
    for (int l = 0; l < 10; l++) {
      const uint8_t* prob = vp8_bmodes_proba + (t * 10 + l) * 9;
      for (int m = 0; m < 10; m++) {
        auto contains = [](int node, int mode, auto&& self) -> bool {
          if (node <= 0) return -node == mode;
          return self(vp8_ymodes_intra4[2 * node], mode, self) || self(vp8_ymodes_intra4[2 * node + 1], mode, self);
        };
        int cost = 0, bit = contains(vp8_ymodes_intra4[0], m, contains) ? 0 : 1;
        cost += bit ? vp8_entropy_cost[255 - prob[0]] : vp8_entropy_cost[prob[0]];
        int i = vp8_ymodes_intra4[bit];
        while (i > 0) {
          bit = contains(vp8_ymodes_intra4[2 * i], m, contains) ? 0 : 1;
          cost += bit ? vp8_entropy_cost[255 - prob[i]] : vp8_entropy_cost[prob[i]];
          i = vp8_ymodes_intra4[2 * i + bit];
        }
        fixed[(t * 10 + l) * 10 + m] = (uint16_t)cost;
      }
    }
}

}  // namespace

/* The VP8FixedCostsI4 table wg_encode_mbs uploads (host copy, 1000 entries). */
extern "C" int wg_fixed_costs_i4_host(uint16_t* out) {
  WG_REQUIRE(out);
  build_fixed_costs_i4(out);
  return WG_OK;
}

WG_IF_STAMPS(extern "C" int wg_debug_enc_phases(unsigned long long* host, int n) {
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_enc_phase), sizeof(unsigned long long) * n);
  unsigned long long z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_enc_phase), z, sizeof(z)) == hipSuccess ? 0 : -2;
})

WG_IF_ROWTIMES(extern "C" int wg_debug_enc_rows(unsigned long long* host, int n_rows) {
  if (n_rows > 16384) n_rows = 16384;
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_row_times), sizeof(unsigned long long) * 4 * n_rows);
  return 0;
})

// work: hand-off records [n][mbw][REC] | ctl[4] (both cleared by every
// wg_encode_mbs) | tag[4] | row schedule order[n*mbh] | slack[n] |
// band schedule border[n*ceil(mbh/4)] (wg_encode_row_order; kept across calls)
extern "C" size_t wg_encode_work_bytes(int32_t mbw, int32_t mbh, int32_t n_images) {
  if (mbw <= 0 || mbh <= 0 || n_images <= 0) return 0;
  const size_t bands = (size_t)n_images * ((mbh + WAVES - 1) / WAVES);
  return (size_t)n_images * mbw * REC + sizeof(int) * 4 +
         sizeof(int) * (4 + (size_t)n_images * mbh + (size_t)n_images + bands);
}

namespace {
// ---- the row schedule (wg_encode_row_order) ----
// A launch over many frames ends on the critical path of its slowest frame:
// mbw + ~2 (mbh - 1) macroblock times of the frame whose macroblocks take
// longest (textured content, where the I4 RD dominates).  Its rows are
// therefore dequeued up to 2 mbh / 5 rows ahead of the others: frame i's row
// y takes the key (y - slack_i, y, i), slack_i = (2 mbh / 5) (1 - (m_i /
// 242)^4), m_i = min(mean alpha_i, 242) (computeAlphas' alpha is low for
// textured macroblocks), in integers.  The slack is proportional to the
// frame's expected macroblock time above the smoothest content's: per MB,
// 44 / 62 / 69 us for the bench's gradient / photo / noise frames (mean
// alpha 240 / 187 / 1.4; tools/enc_timeline.py), which (m / 242)^4 fits; the
// round-5 linear form (mbh / 4) (255 - mean) / 255 gave the photo frames 4
// rows and they finished last.  Keys grow with y within a frame, so a row is
// always dequeued after the row above (the kernel's waits stay on running
// waves); the outputs do not depend on the order.  64 mixed 1080p frames:
// 25.4 -> 23.3 ms (round 3); the bench's G / N / P batch 20.30 -> 19.96 ms
// (round 6, profiles/r06_enc_timeline*.json).
__global__ __launch_bounds__(256) void k_row_slack(const int32_t* alphas, int n_mb, int mbh, int* tag, int* slack) {
  __shared__ long long part[256];
  long long sum = 0;
  const int32_t* al = alphas + (int64_t)blockIdx.x * n_mb;
  for (int i = threadIdx.x; i < n_mb; i += 256) sum += min(max(al[i], 0), 255);
  part[threadIdx.x] = sum;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int mean = (int)(part[0] / n_mb);
    const long long m = min(mean, 242), m4 = m * m * m * m, f4 = 242ll * 242 * 242 * 242;
    slack[blockIdx.x] = (int)((long long)(2 * mbh / 5) * (f4 - m4) / f4);
    if (blockIdx.x == 0) {  // the encoder reads it after k_row_order (same stream)
      tag[0] = ORDER_TAG ^ (int)gridDim.x;
      tag[1] = ~(ORDER_TAG ^ mbh);
    }
  }
}
__global__ __launch_bounds__(256) void k_row_order(const int* slack, int n_img, int mbh, int* order) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n_img * mbh) return;
  const int y = k / n_img, i = k % n_img, di = slack[i], r = y - di;
  int pos = 0;  // rows with a smaller key (r', y', i')
  for (int j = 0; j < n_img; j++) {
    const int dj = slack[j], yj = r + dj;  // frame j's row with the same r
    pos += min(max(yj, 0), mbh) + ((yj >= 0 && yj < mbh && (dj < di || (dj == di && j < i))) ? 1 : 0);
  }
  order[pos] = k;
}
// The same schedule over bands of WAVES rows (the 4-wave launches dequeue a
// band per workgroup): band b of frame i takes the key of its first row,
// (WAVES b - slack_i, b, i), and is placed among the bands by it.  Keys grow
// with b within a frame, so a band is dequeued after the band above.
__global__ __launch_bounds__(256) void k_band_order(const int* slack, int n_img, int mbh, int* border) {
  const int nb = (mbh + WAVES - 1) / WAVES;
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n_img * nb) return;
  const int b = k / n_img, i = k % n_img, di = slack[i], r = WAVES * b - di;
  int pos = 0;  // bands with a smaller key (WAVES b' - d_j, b', j)
  for (int j = 0; j < n_img; j++) {
    const int dj = slack[j], v = r + dj;  // band b' of frame j precedes when WAVES b' < v (ties below)
    const int lt = v <= 0 ? 0 : min((v + WAVES - 1) / WAVES, nb);
    const bool tie = v >= 0 && v % WAVES == 0 && v / WAVES < nb && (dj < di || (dj == di && j < i));
    pos += lt + (tie ? 1 : 0);
  }
  border[pos] = b * n_img + i;
}

}  // namespace

extern "C" int wg_encode_row_order(const int32_t* alphas, int32_t mbw, int32_t mbh, int32_t n_images, void* work,
                                   void* stream) {
  WG_REQUIRE(alphas && work && mbw > 0 && mbh > 0 && n_images > 0);
  WG_REQUIRE((reinterpret_cast<uintptr_t>(work) & 15) == 0);
  const int rows = n_images * mbh;
  int* tag = reinterpret_cast<int*>(static_cast<uint8_t*>(work) + (size_t)n_images * mbw * REC) + 4;
  int* order = tag + 4;
  int* slack = order + rows;
  int* border = slack + n_images;
  const int bands = n_images * ((mbh + WAVES - 1) / WAVES);
  hipStream_t s = wg::as_stream(stream);
  hipLaunchKernelGGL(k_row_slack, dim3((unsigned)n_images), dim3(256), 0, s, alphas, mbw * mbh, mbh, tag, slack);
  hipLaunchKernelGGL(k_row_order, dim3(wg::blocks_for(rows, 256)), dim3(256), 0, s, slack, n_images, mbh, order);
  hipLaunchKernelGGL(k_band_order, dim3(wg::blocks_for(bands, 256)), dim3(256), 0, s, slack, n_images, mbh, border);
  return wg::check_launch("k_row_order");
}


extern "C" int wg_encode_mbs(const uint8_t* y, const uint8_t* u, const uint8_t* v, int64_t y_pitch, int64_t uv_pitch,
                             int32_t width, int32_t height, int32_t n_images, const uint8_t* segments,
                             const void* segs, int64_t segs_pitch, const uint8_t* proba, int32_t method, int32_t quality, void* out,
                             uint8_t* ry, uint8_t* ru, uint8_t* rv, void* work, void* stream) {
  WG_REQUIRE(y && u && v && segs && proba && out && ry && ru && rv && work);
  WG_REQUIRE(width > 0 && height > 0 && n_images > 0);
  // methods 0-2 take the serial encodeFrame with non-RD mode choice (encode.go:1356)
  if (method < 3 || method > 6) return wg::invalid("wg_encode_mbs implements methods 3-6 (encode.go:1356 runs 0-2 serially)");
  const int mbw = (width + 15) >> 4, mbh = (height + 15) >> 4;
  // EncodeFrame (internal/lossy/encode.go:1356) runs the row-parallel Phase A
  // only for mbH >= 4; smaller frames take the serial encodeFrame (chroma DC
  // error diffusion, mid-frame proba refresh), which this kernel is not.
  if (mbh < 4) return wg::invalid("wg_encode_mbs needs mbh >= 4 (height > 48): encode.go:1356 encodes smaller frames serially");
  WG_REQUIRE(mbh < 0x4000);  // (the hand-off tags hold the row in 14 bits)
  WG_REQUIRE(((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(work)) & 15) == 0);
  // Y rows move as 16-B pieces, U / V rows as 8-B pieces (k_encode_rows import / export)
  WG_REQUIRE(((reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(ry)) & 15) == 0 &&
             ((reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(ru) |
               reinterpret_cast<uintptr_t>(rv)) & 7) == 0);
  WG_REQUIRE((reinterpret_cast<uintptr_t>(segs) & 15) == 0 && (segs_pitch == 0 || segs_pitch >= (int64_t)(4 * sizeof(Segment))) &&
             (segs_pitch & 15) == 0);
  WG_REQUIRE(y_pitch >= (int64_t)256 * mbw * mbh && uv_pitch >= (int64_t)64 * mbw * mbh && (y_pitch & 15) == 0 &&
             (uv_pitch & 7) == 0);
  hipStream_t s = wg::as_stream(stream);
  int dev = 0, sdev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return wg::check_launch("hipGetDevice");
  if (wg::stream_device(s, &sdev) != WG_OK) return WG_EHIP;
  WG_REQUIRE(dev >= 0 && dev < 64);
  // the constant tables are uploaded to, and the occupancy read from, the
  // current device: the stream must be on it (webpgpu.h conventions)
  if (sdev != dev) return wg::invalid("wg_encode_mbs: the stream's device is not the current device");
  {
    std::lock_guard<std::mutex> lock(g_tables_mu);
    if (!(g_tables_ready_mask >> dev & 1)) {  // constant tables: level codes, fixed I4 mode costs, scan orders
      uint16_t fixed[1000];
      build_fixed_costs_i4(fixed);
      if (hipMemcpyToSymbol(HIP_SYMBOL(c_fixed_i4), fixed, sizeof(fixed)) != hipSuccess ||
          hipMemcpyToSymbol(HIP_SYMBOL(c_level_codes), vp8_level_codes, sizeof(vp8_level_codes)) != hipSuccess ||
          hipMemcpyToSymbol(HIP_SYMBOL(c_wtrellis), vp8_weight_trellis, sizeof(vp8_weight_trellis)) != hipSuccess)
        return wg::check_launch("encode tables");
      g_tables_ready_mask |= 1ull << dev;
    }
  }
  EncArgs a;
  a.y = y;
  a.u = u;
  a.v = v;
  a.ry = ry;
  a.ru = ru;
  a.rv = rv;
  a.segments = segments;
  a.segs = static_cast<const Segment*>(segs);
  a.segs_pitch = segs_pitch;
  a.proba = proba;
  a.out = static_cast<MbEnc*>(out);
  a.top = static_cast<uint8_t*>(work);
  a.ctl = reinterpret_cast<int*>(a.top + (size_t)n_images * mbw * REC);
  a.y_pitch = y_pitch;
  a.uv_pitch = uv_pitch;
  a.width = width;
  a.height = height;
  a.mbw = mbw;
  a.mbh = mbh;
  a.n_img = n_images;
  a.quality = quality;
  a.order = a.ctl + 8;  // work: records | ctl[4] | tag[4] | order | slack | border
  a.order_tag = a.order - 4;
  a.border = a.order + (size_t)n_images * mbh + n_images;
  a.diag = wg::diag_words(s);
  if (!a.diag) return WG_EHIP;
  a.diag += wg::DIAG_ENCODE;
  // the hand-off records (every tag 0: no row has written), the control words
  // and the progress words, cleared for this launch
  if (hipMemsetAsync(a.top, 0, (size_t)n_images * mbw * REC + sizeof(int) * 4, s) != hipSuccess)
    return wg::check_launch("hipMemsetAsync(encode records + ctl)");
  int cus = 0, per_cu = 0, per_cu_pair = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_encode_rows<true, false>, 64 * WAVES * GROUPS, 0) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_pair, k_encode_rows<true, true>, 128, 0) != hipSuccess ||
      per_cu <= 0 || per_cu_pair <= 0)
    return wg::check_launch("encode occupancy query");
  const int rows = n_images * mbh;
  // a wave pair per row up to three times as many rows as pair workgroups
  // fit at once (mixed 1080p frames with the row schedule: 16 frames 20.2 ->
  // 15.6 ms, 32 frames 20.9 -> 19.5 ms; at 40 frames one wave a row wins,
  // 21.2 vs 21.7 ms, and at 64 clearly, 23.1 vs 30.8 ms: two waves a row
  // halve the rows in flight).  WG_ENCODE_PAIR=0 / 1 forces either schedule.
  bool pair = rows <= 3 * per_cu_pair * cus;
  if (const char* e = getenv("WG_ENCODE_PAIR")) pair = e[0] == '1';
  if (pair) {
    const int grid = rows < per_cu_pair * cus ? rows : per_cu_pair * cus;
    if (method >= 4)
      hipLaunchKernelGGL((k_encode_rows<true, true>), dim3((unsigned)grid), dim3(128), 0, s, a);
    else
      hipLaunchKernelGGL((k_encode_rows<false, true>), dim3((unsigned)grid), dim3(128), 0, s, a);
  } else {
    // each group of a workgroup dequeues bands of WAVES rows
    const int wgs = (n_images * ((mbh + WAVES - 1) / WAVES) + GROUPS - 1) / GROUPS;
    const int grid = wgs < per_cu * cus ? wgs : per_cu * cus;
    if (method >= 4)
      hipLaunchKernelGGL((k_encode_rows<true, false>), dim3((unsigned)grid), dim3(64 * WAVES * GROUPS), 0, s, a);
    else
      hipLaunchKernelGGL((k_encode_rows<false, false>), dim3((unsigned)grid), dim3(64 * WAVES * GROUPS), 0, s, a);
  }
  return wg::check_launch("k_encode_rows");
}

extern "C" int wg_encode_status(const void* work, int32_t mbw, int32_t n_images, void* stream) {
  WG_REQUIRE(work && mbw > 0 && n_images > 0);
  const int* ctl = reinterpret_cast<const int*>(static_cast<const uint8_t*>(work) + (size_t)n_images * mbw * REC);
  return wg::wait_status(ctl + 1, wg::DIAG_ENCODE, wg::as_stream(stream), "wg_encode_status: encode row",
                         "row, image, needed, seen, ticks, block");
}
