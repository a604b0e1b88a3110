/* lossy_rd.c -- TEST INFRASTRUCTURE ONLY.  C restatement of the reference
 * encoder's per-macroblock RD loop, Phase A of encodeFrameParallel
 * (SURVEY.md 8(a) A20), method >= 3:
 *
 *   encodeRow                 internal/lossy/encode_parallel.go:252-338
 *   updateNZContextParallel   :343-430
 *   importBlockParallel       :433-452 (importBlock encode_iterator.go:145-180)
 *   fillPredContextParallel   :455-562
 *   pickBestModeParallel      :565-622
 *   pickBestI16ModeRDParallel :624-737
 *   tryI4ModesRDParallel      :739-846
 *   pickBestI4ModeRD(Trellis)Parallel :848-1028
 *   pickBestUVModeRDParallel  :1030-1114
 *   encodeResidualsParallel   :1166-1356
 *   reconstructMBParallel     :1358-1410
 *   exportParallel            :1412-1495
 *   QuantizeCoeffs / DequantCoeffs / RDScore / TokenCostForCoeffs /
 *   variableLevelCost          internal/lossy/encode_quant.go:16-288
 *   TrellisQuantizeBlock      internal/lossy/encode_trellis.go:23-341
 *   setupSegment / initSegmentQuant internal/lossy/encode.go:1085-1181
 *   isFlatSource16 / isFlat / needsTop4 / needsLeft4 / fixed mode costs
 *                              internal/lossy/encode_analysis.go:345-390, 995-1012, 1481-1534
 *
 * Raster order over macroblocks gives the same result as the reference's
 * row workers: a row reads the shared top arrays only after the row above
 * finished the two macroblocks it reads (encode_parallel.go:286-295).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "vp8_tables.h"

#define BPS 32
#define YOFF (BPS * 1 + 8)
#define UOFF (YOFF + BPS * 16 + BPS)
#define VOFF (UOFF + 16)
#define YUV_SIZE (BPS * 17 + BPS * 9)

/* proba: uint8 [4 types][8 bands][3 ctx][11] */
#define PROBA(pr, t, b, c) ((pr) + (((t) * 8 + (b)) * 3 + (c)) * 11)

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static int maxi(int a, int b) { return a > b ? a : b; }

/* ---------------- segment setup (encode.go:1085-1181) ---------------- */
static void init_squant(or_squant* sq, int dcq, int acq, int type) {
  sq->dc_quant = dcq;
  sq->dc_iquant = (1 << 17) / dcq;
  sq->dc_bias = vp8_bias_matrices[2 * type] << 9;
  sq->dc_zthresh = ((1 << 17) - 1 - sq->dc_bias) / sq->dc_iquant;
  sq->quant = acq;
  sq->iquant = (1 << 17) / acq;
  sq->bias = vp8_bias_matrices[2 * type + 1] << 9;
  sq->zthresh = ((1 << 17) - 1 - sq->bias) / sq->iquant;
  memset(sq->sharpen, 0, sizeof(sq->sharpen));
}

void or_setup_segment(int q, int dq_y1_dc, int dq_y2_dc, int dq_y2_ac, int dq_uv_dc, int dq_uv_ac, int method,
                      int sns_strength, or_segment* s) {
  const int y1dc = vp8_dc_table[clampi(q + dq_y1_dc, 0, 127)];
  const int y1ac = vp8_ac_table[clampi(q, 0, 127)];
  init_squant(&s->y1, y1dc, y1ac, 0);
  int y2dc = vp8_dc_table[clampi(q + dq_y2_dc, 0, 127)] * 2;
  if (y2dc < 8) y2dc = 8;
  const int y2ac = vp8_ac_table2[clampi(q + dq_y2_ac, 0, 127)];
  init_squant(&s->y2, y2dc, y2ac, 1);
  const int uvdc = vp8_dc_table[clampi(q + dq_uv_dc, 0, 117)];
  const int uvac = vp8_ac_table[clampi(q + dq_uv_ac, 0, 127)];
  init_squant(&s->uv, uvdc, uvac, 2);
  const int qi4 = (y1dc + 15 * y1ac + 8) >> 4;
  const int qi16 = (y2dc + 15 * y2ac + 8) >> 4;
  const int quv = (uvdc + 15 * uvac + 8) >> 4;
  s->lambda_i4 = maxi((3 * qi4 * qi4) >> 7, 1);
  s->lambda_i16 = maxi(3 * qi16 * qi16, 1);
  s->lambda_uv = maxi((3 * quv * quv) >> 6, 1);
  s->lambda_mode = maxi((1 * qi4 * qi4) >> 7, 1);
  s->tlambda_i4 = maxi((7 * qi4 * qi4) >> 3, 1);
  s->tlambda_i16 = maxi((qi16 * qi16) >> 2, 1);
  s->tlambda_uv = maxi((quv * quv) << 1, 1);
  s->tlambda_sd = (method >= 4 && sns_strength > 0) ? (sns_strength * qi4) >> 5 : 0;
  for (int i = 0; i < 16; i++) {
    const int qq = i == 0 ? s->y1.dc_quant : s->y1.quant;
    s->y1.sharpen[i] = (int16_t)((vp8_freq_sharpening[i] * qq) >> 11);
  }
}

/* ---------------- quantisation and costs (encode_quant.go) ---------------- */
static int quantize_coeffs(const int16_t* in, int16_t* out, const or_squant* sq, int first) {
  int max_zz = -1;
  if (first == 0) {
    int v = in[0], sign = 1;
    if (v < 0) {
      sign = -1;
      v = -v;
    }
    v += sq->sharpen[0];
    if (v < 0) v = 0;
    int c = (int)(((uint32_t)v * (uint32_t)sq->dc_iquant + (uint32_t)sq->dc_bias) >> 17);
    if (c > 2047) c = 2047;
    out[0] = (int16_t)(sign * c);
    if (c != 0) max_zz = 0;
  } else {
    out[0] = 0;
  }
  for (int n = 1; n < 16; n++) {
    int v = in[n], sign = 1;
    if (v < 0) {
      sign = -1;
      v = -v;
    }
    v += sq->sharpen[n];
    if (v < 0) v = 0;
    int c = (int)(((uint32_t)v * (uint32_t)sq->iquant + (uint32_t)sq->bias) >> 17);
    if (c > 2047) c = 2047;
    out[n] = (int16_t)(sign * c);
    if (c != 0 && vp8_reverse_zigzag[n] > max_zz) max_zz = vp8_reverse_zigzag[n];
  }
  return max_zz + 1;
}

static void dequant_coeffs(const int16_t* in, int16_t* out, const or_squant* sq) {
  out[0] = (int16_t)(in[0] * sq->dc_quant);
  for (int i = 1; i < 16; i++) out[i] = (int16_t)(in[i] * sq->quant);
}

static uint64_t rd_score(int disto, int rate, int lambda) {
  return (uint64_t)(int64_t)rate * (uint64_t)(int64_t)lambda + 256 * (uint64_t)(int64_t)disto;
}

static int bit_cost(int bit, int prob) { return bit ? vp8_entropy_cost[255 - prob] : vp8_entropy_cost[prob]; }

static int variable_level_cost(int level, const uint8_t* p) {
  int idx = level - 1;
  if (idx >= 67) idx = 66;
  int pattern = vp8_level_codes[2 * idx], bits = vp8_level_codes[2 * idx + 1], cost = 0;
  for (int i = 2; pattern != 0; i++) {
    if (pattern & 1) cost += bit_cost(bits & 1, p[i]);
    bits >>= 1;
    pattern >>= 1;
  }
  return cost;
}

static int token_cost(const int16_t* coeffs, int nz_count, int type, const uint8_t* proba, int ctx0, int first) {
  if (nz_count <= first) return vp8_entropy_cost[PROBA(proba, type, vp8_bands[first], ctx0)[0]];
  const int last = nz_count - 1;
  int cost = 0, ctx = ctx0;
  for (int n = first; n < 16; n++) {
    const uint8_t* pp = PROBA(proba, type, vp8_bands[n], ctx);
    int v = coeffs[vp8_zigzag[n]];
    if (v < 0) v = -v;
    if (n > last) {
      cost += vp8_entropy_cost[pp[0]];
      break;
    }
    cost += vp8_entropy_cost[255 - pp[0]];
    if (v == 0) {
      cost += vp8_entropy_cost[pp[1]];
      ctx = 0;
    } else {
      cost += vp8_entropy_cost[255 - pp[1]];
      if (v == 1) {
        cost += vp8_level_fixed_costs[1] + vp8_entropy_cost[pp[2]];
        ctx = 1;
      } else if (v == 2) {
        cost += vp8_level_fixed_costs[2] + vp8_entropy_cost[255 - pp[2]] + vp8_entropy_cost[pp[3]] +
                vp8_entropy_cost[pp[4]];
        ctx = 2;
      } else {
        cost += vp8_level_fixed_costs[v] + variable_level_cost(v, pp);
        ctx = 2;
      }
    }
  }
  return cost;
}

/* fastVariableLevelCost (encode_trellis.go:305-322) equals variable_level_cost. */

/* TrellisQuantizeBlock (encode_trellis.go:23-301) */
static int trellis_quantize(const int16_t* in, int16_t* out, const or_squant* sq, int first, int ctx_type,
                            int init_ctx, const uint8_t* proba, int lambda) {
  { /* pre-scan */
    int nonzero = 0, n = first;
    if (n == 0) {
      int raw = in[vp8_zigzag[0]];
      if (raw < 0) raw = -raw;
      int c0 = raw + sq->sharpen[vp8_zigzag[0]];
      if (c0 < 0) c0 = 0;
      nonzero = ((c0 * sq->dc_iquant) >> 17) > 0;
      n = 1;
    }
    while (!nonzero && n + 3 < 16) {
      int maxc = 0;
      for (int k = 0; k < 4; k++) {
        int raw = in[vp8_zigzag[n + k]];
        if (raw < 0) raw = -raw;
        const int c = raw + sq->sharpen[vp8_zigzag[n + k]];
        if (c > maxc) maxc = c;
      }
      if (maxc > 0 && ((maxc * sq->iquant) >> 17) > 0) nonzero = 1;
      n += 4;
    }
    while (!nonzero && n < 16) {
      int raw = in[vp8_zigzag[n]];
      if (raw < 0) raw = -raw;
      int c0 = raw + sq->sharpen[vp8_zigzag[n]];
      if (c0 < 0) c0 = 0;
      if (((c0 * sq->iquant) >> 17) > 0) nonzero = 1;
      n++;
    }
    if (!nonzero) {
      memset(out, 0, 16 * sizeof(int16_t));
      return 0;
    }
  }
  int16_t inbuf[16];
  memcpy(inbuf, in, sizeof(inbuf));
  memset(out, 0, 16 * sizeof(int16_t));
  if (init_ctx > 2) init_ctx = 2;
  typedef struct {
    int64_t score;
    int16_t level;
    int prev_ctx;
    int valid;
  } state;
  typedef struct {
    int16_t level;
    int prev_ctx;
    int valid;
  } path_entry;
  state prev[3], curr[3];
  path_entry path[16][3];
  memset(path, 0, sizeof(path));
  for (int c = 0; c < 3; c++) prev[c].valid = 0;
  prev[init_ctx].score = 0;
  prev[init_ctx].level = 0;
  prev[init_ctx].prev_ctx = 0;
  prev[init_ctx].valid = 1;
  const int first_band = vp8_bands[first];
  const int skip_rate = bit_cost(0, PROBA(proba, ctx_type, first_band, init_ctx)[0]);
  int64_t best_terminal = (int64_t)skip_rate * lambda;
  int best_last_n = -1, best_last_ctx = -1;
  const int64_t lam = lambda;
  for (int n = first; n < 16; n++) {
    const int zig = vp8_zigzag[n];
    const int band = vp8_bands[n + 1];
    int raw = inbuf[zig], sign = 1;
    if (raw < 0) {
      sign = -1;
      raw = -raw;
    }
    int c0 = raw + sq->sharpen[zig];
    if (c0 < 0) c0 = 0;
    const int quant = n == 0 ? sq->dc_quant : sq->quant;
    const int iquant = n == 0 ? sq->dc_iquant : sq->iquant;
    int L0 = (c0 * iquant) >> 17;
    if (L0 > 2047) L0 = 2047;
    int thresh = (int)(((uint32_t)c0 * (uint32_t)iquant + 65536u) >> 17);
    if (thresh > 2047) thresh = 2047;
    const int64_t weight = vp8_weight_trellis[zig];
    const int64_t c0sq = (int64_t)(c0 * c0);
    const int64_t MAXS = (int64_t)1 << 60;
    for (int c = 0; c < 3; c++) {
      curr[c].valid = 0;
      curr[c].score = MAXS;
    }
    const int has0 = L0 > 0 && L0 <= thresh;
    const int has1 = L0 + 1 <= 2047 && L0 + 1 <= thresh;
    int64_t dd0 = 0, dd1 = 0;
    int nctx0 = 0, nctx1 = 0, fixed0 = 0, fixed1 = 0;
    int16_t sl0 = 0, sl1 = 0;
    if (has0) {
      const int err = c0 - L0 * quant;
      dd0 = weight * ((int64_t)(err * err) - c0sq);
      nctx0 = L0 > 2 ? 2 : L0;
      sl0 = (int16_t)(sign * L0);
      fixed0 = vp8_level_fixed_costs[L0];
    }
    if (has1) {
      const int L1 = L0 + 1;
      const int err = c0 - L1 * quant;
      dd1 = weight * ((int64_t)(err * err) - c0sq);
      nctx1 = L1 > 2 ? 2 : L1;
      sl1 = (int16_t)(sign * L1);
      fixed1 = vp8_level_fixed_costs[L1];
    }
    const int64_t disto0 = 256 * dd0, disto1 = 256 * dd1;
    for (int pc = 0; pc < 3; pc++) {
      if (!prev[pc].valid) continue;
      const int64_t ps = prev[pc].score;
      const uint8_t* p = PROBA(proba, ctx_type, band, pc);
      const int not_eob = vp8_entropy_cost[255 - p[0]];
      const int rate0 = not_eob + vp8_entropy_cost[p[1]];
      const int64_t ts0 = ps + (int64_t)rate0 * lam;
      if (!curr[0].valid || ts0 < curr[0].score) {
        curr[0].score = ts0;
        curr[0].level = 0;
        curr[0].prev_ctx = pc;
        curr[0].valid = 1;
      }
      if (has0 || has1) {
        const int nonzero = not_eob + vp8_entropy_cost[255 - p[1]];
        if (has0) {
          const int r = nonzero + fixed0 + variable_level_cost(L0, p);
          const int64_t ts = ps + (int64_t)r * lam + disto0;
          if (!curr[nctx0].valid || ts < curr[nctx0].score) {
            curr[nctx0].score = ts;
            curr[nctx0].level = sl0;
            curr[nctx0].prev_ctx = pc;
            curr[nctx0].valid = 1;
          }
        }
        if (has1) {
          const int r = nonzero + fixed1 + variable_level_cost(L0 + 1, p);
          const int64_t ts = ps + (int64_t)r * lam + disto1;
          if (!curr[nctx1].valid || ts < curr[nctx1].score) {
            curr[nctx1].score = ts;
            curr[nctx1].level = sl1;
            curr[nctx1].prev_ctx = pc;
            curr[nctx1].valid = 1;
          }
        }
      }
    }
    for (int c = 0; c < 3; c++)
      if (curr[c].valid) {
        path[n][c].level = curr[c].level;
        path[n][c].prev_ctx = curr[c].prev_ctx;
        path[n][c].valid = 1;
      }
    for (int c = 1; c < 3; c++) {
      if (!curr[c].valid) continue;
      int64_t eob = curr[c].score;
      if (n < 15) eob += (int64_t)vp8_entropy_cost[PROBA(proba, ctx_type, band, c)[0]] * lam;
      if (eob < best_terminal) {
        best_terminal = eob;
        best_last_n = n;
        best_last_ctx = c;
      }
    }
    memcpy(prev, curr, sizeof(prev));
  }
  if (best_last_n < 0) return 0;
  int ctx = best_last_ctx, last = 0;
  for (int n = best_last_n; n >= first; n--) {
    if (path[n][ctx].valid) {
      const int zig = vp8_zigzag[n];
      out[zig] = path[n][ctx].level;
      if (out[zig] != 0 && last == 0) last = n + 1;
      ctx = path[n][ctx].prev_ctx;
    }
  }
  for (int n = 0; n < first; n++) out[vp8_zigzag[n]] = 0;
  return last;
}

/* ---------------- helpers (encode_analysis.go) ---------------- */
static int is_flat_source16(const uint8_t* src) {
  const uint8_t v = src[0];
  for (int j = 0; j < 16; j++)
    for (int i = 0; i < 16; i++)
      if (src[j * BPS + i] != v) return 0;
  return 1;
}
static int is_flat(const int16_t* levels, int nblocks, int thresh) {
  int score = 0;
  for (int b = 0; b < nblocks; b++)
    for (int i = 1; i < 16; i++)
      if (levels[b * 16 + i] != 0 && ++score > thresh) return 0;
  return 1;
}
static int needs_top4(int m) { return m == 2 || m == 5 || m == 6 || m == 7 || m == 8 || m == 4 || m == 1; }
static int needs_left4(int m) { return m == 3 || m == 9 || m == 8 || m == 4 || m == 1; }
static int check_mode(int mbx, int mby, int mode) {
  if (mode == 0) {
    if (mbx == 0) return mby == 0 ? 6 : 5;
    return mby == 0 ? 4 : 0;
  }
  return mode;
}

/* VP8FixedCostsI4 (encode_analysis.go:1491-1534, i4SubtreeContains encode_syntax.go:474) */
static int subtree_contains(int node, int mode) {
  if (node <= 0) return -node == mode;
  return subtree_contains(vp8_ymodes_intra4[2 * node], mode) || subtree_contains(vp8_ymodes_intra4[2 * node + 1], mode);
}
static uint16_t fixed_costs_i4[10][10][10];
static int fixed_costs_ready = 0;
static void init_fixed_costs(void) {
  if (fixed_costs_ready) return;
  for (int t = 0; t < 10; t++)
    for (int l = 0; l < 10; l++) {
      const uint8_t* prob = vp8_bmodes_proba + (t * 10 + l) * 9;
      for (int m = 0; m < 10; m++) {
        int cost = 0, bit = subtree_contains(vp8_ymodes_intra4[0], m) ? 0 : 1;
        cost += bit_cost(bit, prob[0]);
        int i = vp8_ymodes_intra4[bit];
        while (i > 0) {
          bit = subtree_contains(vp8_ymodes_intra4[2 * i], m) ? 0 : 1;
          cost += bit_cost(bit, prob[i]);
          i = vp8_ymodes_intra4[2 * i + bit];
        }
        fixed_costs_i4[t][l][m] = (uint16_t)cost;
      }
    }
  fixed_costs_ready = 1;
}
void or_fixed_costs_i4(uint16_t* out) {
  init_fixed_costs();
  memcpy(out, fixed_costs_i4, sizeof(fixed_costs_i4));
}

/* ---------------- per-row worker state ---------------- */
typedef struct {
  uint8_t yuv_in[YUV_SIZE], yuv_out[YUV_SIZE], yuv_out2[YUV_SIZE];
  int16_t best_q[16], best_dq[16];
  int best_nz;
} worker;

static void import_block(const uint8_t* src, int stride, uint8_t* dst, int sx, int sy, int w, int h, int size) {
  for (int j = 0; j < h; j++) {
    memcpy(dst + j * BPS, src + (size_t)(sy + j) * stride + sx, w);
    for (int i = w; i < size; i++) dst[j * BPS + i] = dst[j * BPS + w - 1];
  }
  for (int j = h; j < size; j++) memcpy(dst + j * BPS, dst + (h - 1) * BPS, size);
}

/* pickBestI16ModeRDParallel (:624-737) */
static void pick_best_i16(worker* wk, int mbx, int mby, const or_segment* seg, const uint8_t* proba, uint32_t top_nz,
                          uint32_t left_nz, int top_nz_dc, int left_nz_dc, int* best_mode, int* best_rate,
                          int* best_disto) {
  uint64_t best_score = ~(uint64_t)0;
  *best_mode = 0;
  *best_rate = 0;
  *best_disto = 0;
  const uint8_t* src = wk->yuv_in;
  uint8_t* pred = wk->yuv_out2;
  const int src_flat = is_flat_source16(src + YOFF);
  memcpy(pred, wk->yuv_out, UOFF);
  int dc_ctx = top_nz_dc + left_nz_dc;
  if (dc_ctx > 2) dc_ctx = 2;
  for (int mode = 0; mode < 4; mode++) {
    const int actual = check_mode(mbx, mby, mode);
    if (mode == 2 && mby == 0) continue;
    if (mode == 3 && mbx == 0) continue;
    if (mode == 1 && (mbx == 0 || mby == 0)) continue;
    or_pred_luma16(actual, pred, YOFF);
    int16_t dc_coeffs[16] = {0}, all_q[16][16], tmp[16], q[16];
    int total_rate = vp8_mode_fixed_cost16[mode];
    uint32_t tnz = top_nz & 0x0f, lnz = left_nz & 0x0f;
    for (int by = 0; by < 4; by++) {
      uint32_t l = lnz & 1;
      for (int bx = 0; bx < 4; bx++) {
        const int b = by * 4 + bx, off = YOFF + by * 4 * BPS + bx * 4;
        int ctx = (int)(l + (tnz & 1));
        if (ctx > 2) ctx = 2;
        or_ftransform(src + off, pred + off, tmp);
        dc_coeffs[b] = tmp[0];
        tmp[0] = 0;
        const int nz = quantize_coeffs(tmp, q, &seg->y1, 1);
        memcpy(all_q[b], q, sizeof(q));
        total_rate += token_cost(q, nz, 0, proba, ctx, 1);
        l = nz > 0;
        tnz = (tnz >> 1) | (l << 7);
      }
      tnz >>= 4;
      lnz = (lnz >> 1) | (l << 7);
    }
    int16_t wht[16], qdc[16], whtdq[16], whtbuf[256];
    or_ftransform_wht(dc_coeffs, wht);
    const int nzdc = quantize_coeffs(wht, qdc, &seg->y2, 0);
    total_rate += token_cost(qdc, nzdc, 1, proba, dc_ctx, 0);
    dequant_coeffs(qdc, whtdq, &seg->y2);
    or_transform_wht(whtdq, whtbuf);
    for (int b = 0; b < 16; b++) {
      const int off = YOFF + (b >> 2) * 4 * BPS + (b & 3) * 4;
      int16_t dq[16];
      dequant_coeffs(all_q[b], dq, &seg->y1);
      dq[0] = whtbuf[b * 16];
      or_itransform(pred + off, dq, pred + off, 0);
    }
    int disto = or_sse16x16(src + YOFF, pred + YOFF);
    if (seg->tlambda_sd > 0) disto += (seg->tlambda_sd * or_tdisto16x16(src + YOFF, pred + YOFF) + 128) >> 8;
    if (src_flat && is_flat(&all_q[0][0], 16, 0)) disto *= 2;
    const uint64_t score = rd_score(disto, total_rate, seg->lambda_i16);
    if (score < best_score) {
      best_score = score;
      *best_mode = mode;
      *best_rate = total_rate;
      *best_disto = disto;
    }
  }
}

/* pickBestI4ModeRD(Trellis)Parallel (:848-1028) for one block. */
static int pick_best_i4_block(worker* wk, int src_off, const or_segment* seg, int top_mode, int left_mode,
                              int has_top, int has_left, int nz_ctx, const uint8_t* proba, int max_modes, int trellis,
                              int* out_rate, int* out_disto) {
  uint64_t best_score = ~(uint64_t)0;
  int best_mode = 0;
  *out_rate = 0;
  *out_disto = 0;
  const uint8_t* src = wk->yuv_in + src_off;
  uint8_t* pred = wk->yuv_out2;
  int cand_mode[10], cand_sse[10], nc = 0;
  for (int m = 0; m < 10; m++) {
    if (!has_top && needs_top4(m)) continue;
    if (!has_left && needs_left4(m)) continue;
    or_pred_luma4(m, pred, src_off);
    cand_mode[nc] = m;
    cand_sse[nc] = or_sse4x4(src, pred + src_off);
    nc++;
  }
  int K = max_modes < nc ? max_modes : nc;
  for (int i = 0; i < K; i++) {
    int mi = i;
    for (int j = i + 1; j < nc; j++)
      if (cand_sse[j] < cand_sse[mi]) mi = j;
    if (mi != i) {
      int t = cand_mode[i];
      cand_mode[i] = cand_mode[mi];
      cand_mode[mi] = t;
      t = cand_sse[i];
      cand_sse[i] = cand_sse[mi];
      cand_sse[mi] = t;
    }
  }
  for (int i = 0; i < K; i++) {
    const int mode = cand_mode[i];
    or_pred_luma4(mode, pred, src_off);
    int16_t co[16], q[16], dq[16];
    uint8_t recon[4 * BPS];
    or_ftransform(src, pred + src_off, co);
    const int nz = trellis ? trellis_quantize(co, q, &seg->y1, 0, 3, nz_ctx, proba, seg->tlambda_i4)
                           : quantize_coeffs(co, q, &seg->y1, 0);
    dequant_coeffs(q, dq, &seg->y1);
    or_itransform(pred + src_off, dq, recon, 0);
    int disto = or_sse4x4(src, recon);
    if (seg->tlambda_sd > 0) disto += (seg->tlambda_sd * or_tdisto4x4(src, recon) + 128) >> 8;
    if (256 * (uint64_t)(int64_t)disto >= best_score) continue;
    int rate = 0;
    if (mode > 0 && is_flat(q, 1, 3)) rate = 140;
    rate += token_cost(q, nz, 3, proba, nz_ctx, 0);
    rate += fixed_costs_i4[top_mode][left_mode][mode];
    const uint64_t score = rd_score(disto, rate, seg->lambda_i4);
    if (score < best_score) {
      best_score = score;
      best_mode = mode;
      *out_rate = rate;
      *out_disto = disto;
      memcpy(wk->best_dq, dq, sizeof(dq));
      memcpy(wk->best_q, q, sizeof(q));
      wk->best_nz = nz;
    }
  }
  return best_mode;
}

/* tryI4ModesRDParallel (:739-846) */
static uint64_t try_i4(worker* wk, int mbx, int mby, or_mb_enc* info, const or_segment* seg, uint8_t* modes,
                       const uint8_t* top_m, const uint8_t* left_modes, uint64_t i16_score, uint32_t top_nz,
                       uint32_t left_nz, const uint8_t* proba, int method, int quality) {
  int total_rate = 0, total_disto = 0, total_header = 0;
  memcpy(wk->yuv_out2, wk->yuv_out, YUV_SIZE);
  uint32_t tnz = top_nz & 0x0f, lnz = left_nz & 0x0f, l = 0;
  int early = 0;
  const int max_modes = quality < 50 ? 2 : 3;
  for (int by = 0; by < 4 && !early; by++) {
    l = lnz & 1;
    for (int bx = 0; bx < 4; bx++) {
      const int b = by * 4 + bx;
      const int top_mode = by == 0 ? top_m[bx] : modes[b - 4];
      const int left_mode = bx == 0 ? left_modes[by] : modes[b - 1];
      const int src_off = YOFF + by * 4 * BPS + bx * 4;
      const int has_top = mby > 0 || by > 0, has_left = mbx > 0 || bx > 0;
      int nz_ctx = (int)(l + (tnz & 1));
      if (nz_ctx > 2) nz_ctx = 2;
      int rate, disto;
      const int best = pick_best_i4_block(wk, src_off, seg, top_mode, left_mode, has_top, has_left, nz_ctx, proba,
                                          max_modes, method >= 4, &rate, &disto);
      modes[b] = (uint8_t)best;
      total_rate += rate;
      total_disto += disto;
      total_header += fixed_costs_i4[top_mode][left_mode][best];
      memcpy(info->coeffs + b * 16, wk->best_q, sizeof(wk->best_q));
      const int nz = wk->best_nz;
      info->nz_y[b] = (uint8_t)nz;
      if (rd_score(total_disto, total_rate + 211, seg->lambda_mode) >= i16_score || total_header > 15000) {
        early = 1;
        break;
      }
      or_pred_luma4(best, wk->yuv_out2, src_off);
      or_itransform(wk->yuv_out2 + src_off, wk->best_dq, wk->yuv_out2 + src_off, 0);
      l = nz > 0;
      tnz = (tnz >> 1) | (l << 7);
    }
    tnz >>= 4;
    lnz = (lnz >> 1) | (l << 7);
  }
  if (early) return ~(uint64_t)0;
  total_rate += 211;
  return rd_score(total_disto, total_rate, seg->lambda_mode);
}

/* pickBestUVModeRDParallel (:1030-1114) */
static int pick_best_uv(worker* wk, int mbx, int mby, const or_segment* seg, const uint8_t* proba, uint32_t top_nz,
                        uint32_t left_nz) {
  uint64_t best_score = ~(uint64_t)0;
  int best = 0;
  const uint8_t* src = wk->yuv_in;
  uint8_t* pred = wk->yuv_out2;
  memcpy(pred + UOFF, wk->yuv_out + UOFF, YUV_SIZE - UOFF);
  for (int mode = 0; mode < 4; mode++) {
    const int actual = check_mode(mbx, mby, mode);
    if (mode == 2 && mby == 0) continue;
    if (mode == 3 && mbx == 0) continue;
    if (mode == 1 && (mbx == 0 || mby == 0)) continue;
    or_pred_chroma8(actual, pred, UOFF);
    or_pred_chroma8(actual, pred, VOFF);
    int total_rate = vp8_mode_fixed_cost_uv[mode];
    int16_t levels[8 * 16];
    int bi = 0;
    for (int ch = 0; ch < 4; ch += 2) {
      uint32_t tnz = (top_nz >> (4 + ch)) & 0x0f, lnz = (left_nz >> (4 + ch)) & 0x0f;
      const int plane = ch == 0 ? UOFF : VOFF;
      for (int by = 0; by < 2; by++) {
        uint32_t l = lnz & 1;
        for (int bx = 0; bx < 2; bx++) {
          const int off = plane + by * 4 * BPS + bx * 4;
          int ctx = (int)(l + (tnz & 1));
          if (ctx > 2) ctx = 2;
          int16_t co[16], q[16], dq[16];
          or_ftransform(src + off, pred + off, co);
          const int nz = quantize_coeffs(co, q, &seg->uv, 0);
          total_rate += token_cost(q, nz, 2, proba, ctx, 0);
          memcpy(levels + bi * 16, q, sizeof(q));
          bi++;
          dequant_coeffs(q, dq, &seg->uv);
          or_itransform(pred + off, dq, pred + off, 0);
          l = nz > 0;
          tnz = (tnz >> 1) | (l << 3);
        }
        tnz >>= 2;
        lnz = (lnz >> 1) | (l << 5);
      }
    }
    if (mode > 0 && is_flat(levels, 8, 2)) total_rate += 140 * 8;
    int disto = 0;
    for (int by = 0; by < 2; by++)
      for (int bx = 0; bx < 2; bx++) {
        const int off = by * 4 * BPS + bx * 4;
        disto += or_sse4x4(src + UOFF + off, pred + UOFF + off);
        disto += or_sse4x4(src + VOFF + off, pred + VOFF + off);
      }
    const uint64_t score = rd_score(disto, total_rate, seg->lambda_uv);
    if (score < best_score) {
      best_score = score;
      best = mode;
    }
  }
  return best;
}

/* updateNZContextParallel (:343-430) */
static void update_nz(const or_mb_enc* info, uint32_t* top_nz, uint32_t* left_nz, uint8_t* top_nz_dc,
                      uint8_t* left_nz_dc) {
  const uint32_t tv = *top_nz, lv = *left_nz;
  uint32_t out_t, out_l;
  const int first = info->mb_type == 0 ? 1 : 0;
  if (info->mb_type == 0) {
    const uint8_t d = info->nz_dc > 0;
    *top_nz_dc = d;
    *left_nz_dc = d;
  }
  uint32_t tnz = tv & 0x0f, lnz = lv & 0x0f;
  for (int y = 0; y < 4; y++) {
    uint32_t l = lnz & 1;
    for (int x = 0; x < 4; x++) {
      l = info->nz_y[y * 4 + x] > first;
      tnz = (tnz >> 1) | (l << 7);
    }
    tnz >>= 4;
    lnz = (lnz >> 1) | (l << 7);
  }
  out_t = tnz;
  out_l = lnz >> 4;
  for (int ch = 0; ch < 4; ch += 2) {
    tnz = (tv >> (4 + ch)) & 0x0f;
    lnz = (lv >> (4 + ch)) & 0x0f;
    for (int y = 0; y < 2; y++) {
      uint32_t l = lnz & 1;
      for (int x = 0; x < 2; x++) {
        l = info->nz_uv[(ch / 2) * 4 + y * 2 + x] > 0;
        tnz = (tnz >> 1) | (l << 3);
      }
      tnz >>= 2;
      lnz = (lnz >> 1) | (l << 5);
    }
    out_t |= (tnz << 4) << ch;
    out_l |= (lnz & 0xf0) << ch;
  }
  *top_nz = out_t;
  *left_nz = out_l;
}

void or_encode_frame_rd(uint8_t* yp, uint8_t* up, uint8_t* vp, int width, int height, int mbw, int mbh,
                        const uint8_t* segments, const or_segment* segs, const uint8_t* proba, int method,
                        int quality, or_mb_enc* out) {
  init_fixed_costs();
  const int ys = 16 * mbw, uvs = 8 * mbw;
  uint8_t* top_y = malloc(16 * mbw);
  uint8_t* top_u = malloc(8 * mbw);
  uint8_t* top_v = malloc(8 * mbw);
  uint8_t* top_modes = malloc(4 * mbw);
  uint32_t* top_nz = calloc(mbw, sizeof(uint32_t));
  uint8_t* top_nz_dc = calloc(mbw, 1);
  memset(top_y, 127, 16 * mbw);
  memset(top_u, 127, 8 * mbw);
  memset(top_v, 127, 8 * mbw);
  memset(top_modes, 0, 4 * mbw);
  worker* wk = calloc(1, sizeof(worker));
  for (int mby = 0; mby < mbh; mby++) {
    uint8_t left_y[16], left_u[8], left_v[8], left_modes[4] = {0, 0, 0, 0};
    uint8_t tl_y = 127, tl_u = 127, tl_v = 127;
    uint32_t left_nz = 0;
    uint8_t left_nz_dc = 0;
    memset(left_y, 129, 16);
    memset(left_u, 129, 8);
    memset(left_v, 129, 8);
    for (int mbx = 0; mbx < mbw; mbx++) {
      const int idx = mby * mbw + mbx;
      or_mb_enc* info = out + idx;
      memset(info, 0, sizeof(*info));
      info->segment = segments ? segments[idx] : 0;
      const or_segment* seg = segs + (info->segment & 3);
      /* importBlockParallel */
      const int x = 16 * mbx, y = 16 * mby;
      const int ww = width - x > 16 ? 16 : width - x, hh = height - y > 16 ? 16 : height - y;
      import_block(yp, ys, wk->yuv_in + YOFF, x, y, ww, hh, 16);
      const int uvw = (ww + 1) >> 1, uvh = (hh + 1) >> 1;
      import_block(up, uvs, wk->yuv_in + UOFF, 8 * mbx, 8 * mby, uvw, uvh, 8);
      import_block(vp, uvs, wk->yuv_in + VOFF, 8 * mbx, 8 * mby, uvw, uvh, 8);
      /* fillPredContextParallel */
      uint8_t* o = wk->yuv_out;
      for (int i = 0; i < 16; i++) o[YOFF - BPS + i] = mby > 0 ? top_y[16 * mbx + i] : 127;
      for (int i = 0; i < 4; i++)
        o[YOFF - BPS + 16 + i] =
            mby > 0 ? (mbx < mbw - 1 ? top_y[16 * (mbx + 1) + i] : top_y[16 * mbx + 15]) : 127;
      for (int r = 1; r <= 3; r++)
        for (int i = 0; i < 4; i++) o[YOFF - BPS + 16 + r * 4 * BPS + i] = o[YOFF - BPS + 16 + i];
      o[YOFF - BPS - 1] = (mbx > 0 && mby > 0) ? tl_y : (mby > 0 ? 129 : 127);
      for (int j = 0; j < 16; j++) o[YOFF - 1 + j * BPS] = mbx > 0 ? left_y[j] : 129;
      for (int i = 0; i < 8; i++) {
        o[UOFF - BPS + i] = mby > 0 ? top_u[8 * mbx + i] : 127;
        o[VOFF - BPS + i] = mby > 0 ? top_v[8 * mbx + i] : 127;
      }
      o[UOFF - BPS - 1] = (mbx > 0 && mby > 0) ? tl_u : (mby > 0 ? 129 : 127);
      o[VOFF - BPS - 1] = (mbx > 0 && mby > 0) ? tl_v : (mby > 0 ? 129 : 127);
      for (int j = 0; j < 8; j++) {
        o[UOFF - 1 + j * BPS] = mbx > 0 ? left_u[j] : 129;
        o[VOFF - 1 + j * BPS] = mbx > 0 ? left_v[j] : 129;
      }
      /* pickBestModeParallel (method >= 3) */
      int m16, r16, d16;
      pick_best_i16(wk, mbx, mby, seg, proba, top_nz[mbx], left_nz, top_nz_dc[mbx], left_nz_dc, &m16, &r16, &d16);
      const uint64_t s16 = rd_score(d16, r16, seg->lambda_mode);
      uint8_t modes4[16] = {0}, top_m[4] = {0, 0, 0, 0};
      if (mby > 0) memcpy(top_m, top_modes + 4 * mbx, 4);
      const uint64_t s4 = try_i4(wk, mbx, mby, info, seg, modes4, top_m, left_modes, s16, top_nz[mbx], left_nz, proba,
                                 method, quality);
      int pred_cached = 0, i4_cached = 0;
      if (s4 < s16) {
        info->mb_type = 1;
        memcpy(info->modes, modes4, 16);
        info->score = s4;
        if (method >= 4) {
          i4_cached = 1;
          for (int j = 0; j < 16; j++) memcpy(o + YOFF + j * BPS, wk->yuv_out2 + YOFF + j * BPS, 16);
        }
      } else {
        info->mb_type = 0;
        info->i16_mode = (uint8_t)m16;
        info->score = s16;
        or_pred_luma16(check_mode(mbx, mby, m16), o, YOFF);
        pred_cached = 1;
      }
      info->uv_mode = (uint8_t)pick_best_uv(wk, mbx, mby, seg, proba, top_nz[mbx], left_nz);
      or_pred_chroma8(check_mode(mbx, mby, info->uv_mode), o, UOFF);
      or_pred_chroma8(check_mode(mbx, mby, info->uv_mode), o, VOFF);
      (void)pred_cached; /* the I16 / UV predictions are in yuv_out either way (method >= 3) */
      /* encodeResidualsParallel */
      if (info->mb_type == 0) {
        int16_t dc[16];
        uint32_t nzy = 0, tnz = top_nz[mbx] & 0x0f, lnz = left_nz & 0x0f;
        for (int by = 0; by < 4; by++) {
          uint32_t l = lnz & 1;
          for (int bx = 0; bx < 4; bx++) {
            const int b = by * 4 + bx, off = by * 4 * BPS + bx * 4;
            int16_t* co = info->coeffs + b * 16;
            or_ftransform(wk->yuv_in + YOFF + off, o + YOFF + off, co);
            dc[b] = co[0];
            co[0] = 0;
            int nz;
            if (method >= 4) {
              int ctx = (int)(l + (tnz & 1));
              if (ctx > 2) ctx = 2;
              int16_t tq[16];
              nz = trellis_quantize(co, tq, &seg->y1, 1, 0, ctx, proba, seg->tlambda_i16);
              memcpy(co, tq, sizeof(tq));
            } else {
              int16_t tq[16];
              nz = quantize_coeffs(co, tq, &seg->y1, 1);
              memcpy(co, tq, sizeof(tq));
            }
            info->nz_y[b] = (uint8_t)nz;
            if (nz > 0) {
              nzy |= 1u << b;
              l = 1;
            } else {
              l = 0;
            }
            tnz = (tnz >> 1) | (l << 7);
          }
          tnz >>= 4;
          lnz = (lnz >> 1) | (l << 7);
        }
        int16_t wht[16];
        or_ftransform_wht(dc, wht);
        const int nzdc = quantize_coeffs(wht, info->coeffs + 384, &seg->y2, 0);
        info->nz_dc = (uint8_t)nzdc;
        if (nzdc > 0) nzy |= 1u << 24;
        info->non_zero_y = nzy;
      } else if (i4_cached) {
        uint32_t nzy = 0;
        for (int b = 0; b < 16; b++)
          if (info->nz_y[b] > 0) nzy |= 1u << b;
        info->non_zero_y = nzy;
      } else { /* method 3: re-encode I4 blocks with plain quantisation */
        uint32_t nzy = 0;
        for (int b = 0; b < 16; b++) {
          const int off = (b >> 2) * 4 * BPS + (b & 3) * 4;
          or_pred_luma4(info->modes[b], o, YOFF + off);
          int16_t* co = info->coeffs + b * 16;
          int16_t tq[16], dq[16];
          or_ftransform(wk->yuv_in + YOFF + off, o + YOFF + off, co);
          const int nz = quantize_coeffs(co, tq, &seg->y1, 0);
          memcpy(co, tq, sizeof(tq));
          info->nz_y[b] = (uint8_t)nz;
          if (nz > 0) nzy |= 1u << b;
          dequant_coeffs(co, dq, &seg->y1);
          or_itransform(o + YOFF + off, dq, o + YOFF + off, 0);
        }
        info->non_zero_y = nzy;
      }
      {
        uint32_t nzuv = 0;
        for (int ch = 0; ch < 2; ch++)
          for (int b = 0; b < 4; b++) {
            const int off = (ch ? VOFF : UOFF) + (b >> 1) * 4 * BPS + (b & 1) * 4;
            or_ftransform(wk->yuv_in + off, o + off, info->coeffs + (16 + ch * 4 + b) * 16);
          }
        for (int ch = 0; ch < 2; ch++)
          for (int b = 0; b < 4; b++) {
            int16_t* co = info->coeffs + (16 + ch * 4 + b) * 16;
            int16_t tq[16];
            const int nz = quantize_coeffs(co, tq, &seg->uv, 0);
            memcpy(co, tq, sizeof(tq));
            info->nz_uv[ch * 4 + b] = (uint8_t)nz;
            if (nz > 0) nzuv |= 1u << (ch * 4 + b);
          }
        info->non_zero_uv = nzuv;
      }
      info->skip = info->non_zero_y == 0 && info->non_zero_uv == 0;
      /* reconstructMBParallel */
      if (info->mb_type == 0) {
        int16_t whtdq[16], whtbuf[256];
        dequant_coeffs(info->coeffs + 384, whtdq, &seg->y2);
        or_transform_wht(whtdq, whtbuf);
        for (int b = 0; b < 16; b++) {
          const int off = YOFF + (b >> 2) * 4 * BPS + (b & 3) * 4;
          int16_t dq[16];
          dequant_coeffs(info->coeffs + b * 16, dq, &seg->y1);
          dq[0] = whtbuf[b * 16];
          or_itransform(o + off, dq, o + off, 0);
        }
      }
      for (int b = 0; b < 4; b++) {
        const int off = (b >> 1) * 4 * BPS + (b & 1) * 4;
        int16_t dq[16];
        dequant_coeffs(info->coeffs + (16 + b) * 16, dq, &seg->uv);
        or_itransform(o + UOFF + off, dq, o + UOFF + off, 0);
        dequant_coeffs(info->coeffs + (20 + b) * 16, dq, &seg->uv);
        or_itransform(o + VOFF + off, dq, o + VOFF + off, 0);
      }
      /* exportParallel */
      const int wy = x + 16 > width ? width - x : 16, hy = y + 16 > height ? height - y : 16;
      for (int j = 0; j < hy; j++) memcpy(yp + (size_t)(y + j) * ys + x, o + YOFF + j * BPS, wy);
      for (int j = 0; j < 8; j++) {
        memcpy(up + (size_t)(8 * mby + j) * uvs + 8 * mbx, o + UOFF + j * BPS, 8);
        memcpy(vp + (size_t)(8 * mby + j) * uvs + 8 * mbx, o + VOFF + j * BPS, 8);
      }
      tl_y = top_y[16 * mbx + 15];
      tl_u = top_u[8 * mbx + 7];
      tl_v = top_v[8 * mbx + 7];
      memcpy(top_y + 16 * mbx, o + YOFF + 15 * BPS, 16);
      memcpy(top_u + 8 * mbx, o + UOFF + 7 * BPS, 8);
      memcpy(top_v + 8 * mbx, o + VOFF + 7 * BPS, 8);
      for (int j = 0; j < 16; j++) left_y[j] = o[YOFF + j * BPS + 15];
      for (int j = 0; j < 8; j++) {
        left_u[j] = o[UOFF + j * BPS + 7];
        left_v[j] = o[VOFF + j * BPS + 7];
      }
      if (info->mb_type == 1) {
        for (int i = 0; i < 4; i++) top_modes[4 * mbx + i] = info->modes[12 + i];
        left_modes[0] = info->modes[3];
        left_modes[1] = info->modes[7];
        left_modes[2] = info->modes[11];
        left_modes[3] = info->modes[15];
      } else {
        memset(top_modes + 4 * mbx, 0, 4);
        memset(left_modes, 0, 4);
      }
      update_nz(info, &top_nz[mbx], &left_nz, &top_nz_dc[mbx], &left_nz_dc);
    }
  }
  free(wk);
  free(top_y);
  free(top_u);
  free(top_v);
  free(top_modes);
  free(top_nz);
  free(top_nz_dc);
}

/* ---------------- exported for the per-function KAT tests (tests/test_rd_kats.py) ---------------- */
/* QuantizeCoeffs (encode_quant.go:16-75) */
int or_quantize_coeffs(const int16_t* in, int16_t* out, const or_squant* sq, int first) {
  return quantize_coeffs(in, out, sq, first);
}
/* DequantCoeffs (encode_quant.go:81-101) */
void or_dequant_coeffs(const int16_t* in, int16_t* out, const or_squant* sq) { dequant_coeffs(in, out, sq); }
/* RDScore (encode_quant.go:109-111) */
uint64_t or_rd_score(int disto, int rate, int lambda) { return rd_score(disto, rate, lambda); }
/* TokenCostForCoeffs (encode_quant.go:170-220) */
int or_token_cost(const int16_t* coeffs, int nz_count, int type, const uint8_t* proba, int ctx0, int first) {
  return token_cost(coeffs, nz_count, type, proba, ctx0, first);
}
/* TrellisQuantizeBlock (encode_trellis.go:23-301) */
int or_trellis_quantize(const int16_t* in, int16_t* out, const or_squant* sq, int first, int ctx_type, int init_ctx,
                        const uint8_t* proba, int lambda) {
  return trellis_quantize(in, out, sq, first, ctx_type, init_ctx, proba, lambda);
}
