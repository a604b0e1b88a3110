/*
 * segments.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The encoder's segment analysis after computeAlphas: analysis()
 * (internal/lossy/encode_analysis.go:29-73) -> assignSegments (:737-849,
 * with smoothSegmentMap :76-119) -> setSegmentParams (:122-195:
 * qualityToCompression encode.go:1039, setupFilterStrength encode.go:1276-1320,
 * simplifySegments :197-242), then EncodeFrame's setSegmentProbas
 * (:874-903).  setupSegment for the resulting quantisers is
 * or_setup_segment (lossy_rd.c).
 *
 * Go's int division truncates toward zero, like C's.  The per-segment
 * quantiser uses math.Pow; libm's pow is used here, and
 * tests/test_segments.py shows that no (quality, sns, alpha) input lies close
 * enough to an integer step of 127*(1-c) for the two to disagree.
 */
#include <math.h>
#include <string.h>

#include "oracle.h"
#include "vp8_tables.h"

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static int absi(int v) { return v < 0 ? -v : v; }

/* qualityToCompression, internal/lossy/encode.go:1039-1055 */
double or_quality_to_compression(int quality) {
  if (quality <= 0) return 0.0;
  if (quality >= 100) return 1.0;
  const double c = (double)quality / 100.0;
  const double linear_c = c < 0.75 ? c * (2.0 / 3.0) : 2.0 * c - 1.0;
  return pow(linear_c, 1.0 / 3.0);
}

/* qualityToQIndex, encode.go:1060-1063 */
int or_quality_to_qindex(int quality) {
  return clampi((int)(127.0 * (1.0 - or_quality_to_compression(quality))), 0, 127);
}

/* setSegmentParams' per-segment quantiser, encode_analysis.go:128-142 */
int or_segment_quant(int quality, int sns_strength, int seg_alpha) {
  const int sns = sns_strength < 0 ? 0 : sns_strength;
  const double amp = 0.9 * (double)sns / 100.0 / 128.0;
  const double c_base = or_quality_to_compression(quality);
  const double expn = 1.0 - amp * (double)seg_alpha;
  const double c = pow(c_base, expn);
  return clampi((int)(127.0 * (1.0 - c)), 0, 127);
}

/* one SegmentInfo's fields the analysis touches */
typedef struct {
  int quant, fstrength, alpha, beta;
} seginfo;

/* filterStrengthFromDelta, encode.go:1259-1268 */
static int filter_strength_from_delta(int sharpness, int delta) {
  return vp8_levels_from_delta[sharpness * 64 + clampi(delta, 0, 63)];
}

void or_segment_analysis(const int32_t* alphas, int mbw, int mbh, int uv_alpha_sum, const or_enc_config* cfg,
                         uint8_t* seg_ids, or_frame_segs* info) {
  const int total = mbw * mbh;
  memset(info, 0, sizeof(*info));
  seginfo dqm[4];
  memset(dqm, 0, sizeof(dqm));
  /* analysis(): numSegs = clamp(config.Segments, 1, NumMBSegments) (:30-36) */
  int num_segs = clampi(cfg->segments, 1, 4);
  /* computeAlphas' return value (:308) */
  const int global_uv_alpha = total > 0 ? uv_alpha_sum / total : 0;
  if (num_segs <= 1) { /* :50-57 */
    for (int i = 0; i < total; i++) seg_ids[i] = 0;
    dqm[0].alpha = 0;
    dqm[0].beta = 0;
  } else if (total > 0) {
    /* assignSegments (:737-849) */
    int histo[256] = {0};
    for (int i = 0; i < total; i++) histo[alphas[i]]++;
    int min_a = 0;
    while (min_a <= 255 && histo[min_a] == 0) min_a++;
    int max_a = 255;
    while (max_a > min_a && histo[max_a] == 0) max_a--;
    const int range_a = max_a - min_a;
    int centers[4] = {0, 0, 0, 0};
    for (int k = 0; k < num_segs; k++) centers[k] = min_a + ((2 * k + 1) * range_a) / (2 * num_segs);
    int alpha_map[256] = {0};
    int weighted_avg = 0;
    for (int iter = 0; iter < 6; iter++) { /* maxItersKMeans = 6 (:731) */
      int accum[4] = {0, 0, 0, 0}, dist_accum[4] = {0, 0, 0, 0};
      int n = 0;
      for (int a = min_a; a <= max_a; a++) {
        if (histo[a] == 0) continue;
        while (n + 1 < num_segs && absi(a - centers[n + 1]) < absi(a - centers[n])) n++;
        alpha_map[a] = n;
        dist_accum[n] += a * histo[a];
        accum[n] += histo[a];
      }
      int displaced = 0, total_weight = 0;
      weighted_avg = 0;
      for (int s = 0; s < num_segs; s++) {
        if (accum[s] > 0) {
          const int nc = (dist_accum[s] + accum[s] / 2) / accum[s];
          displaced += absi(centers[s] - nc);
          centers[s] = nc;
          weighted_avg += nc * accum[s];
          total_weight += accum[s];
        }
      }
      if (total_weight > 0) weighted_avg = (weighted_avg + total_weight / 2) / total_weight;
      if (displaced < 5) break;
    }
    for (int i = 0; i < total; i++) seg_ids[i] = (uint8_t)alpha_map[alphas[i]];
    /* smoothSegmentMap (:76-119) when config.Segments > 1 and preprocessing bit 0 */
    if (cfg->segments > 1 && (cfg->preprocessing & 1) && mbw >= 3 && mbh >= 3) {
      uint8_t* tmp = (uint8_t*)__builtin_alloca((size_t)total);
      memcpy(tmp, seg_ids, (size_t)total);
      for (int y = 1; y < mbh - 1; y++)
        for (int x = 1; x < mbw - 1; x++) {
          int cnt[4] = {0, 0, 0, 0};
          for (int dy = -1; dy <= 1; dy++)
            for (int dx = -1; dx <= 1; dx++) cnt[seg_ids[(y + dy) * mbw + x + dx]]++;
          int best = tmp[y * mbw + x];
          for (int s = 0; s < 4; s++)
            if (cnt[s] >= 5) best = s;
          tmp[y * mbw + x] = (uint8_t)best;
        }
      for (int y = 1; y < mbh - 1; y++)
        for (int x = 1; x < mbw - 1; x++) seg_ids[y * mbw + x] = tmp[y * mbw + x];
    }
    /* SetSegmentAlphas (:825-848) */
    int min_c = centers[0], max_c = centers[0];
    for (int s = 1; s < num_segs; s++) {
      if (centers[s] < min_c) min_c = centers[s];
      if (centers[s] > max_c) max_c = centers[s];
    }
    int range_c = max_c - min_c;
    if (range_c == 0) range_c = 1;
    for (int s = 0; s < num_segs; s++) {
      dqm[s].alpha = clampi(255 * (centers[s] - weighted_avg) / range_c, -127, 127);
      dqm[s].beta = clampi(255 * (centers[s] - min_c) / range_c, 0, 255);
    }
  }
  /* setSegmentParams (:122-195) */
  const int sns = cfg->sns_strength < 0 ? 0 : cfg->sns_strength;
  for (int i = 0; i < num_segs; i++) dqm[i].quant = or_segment_quant(cfg->quality, sns, dqm[i].alpha);
  const int base_quant = dqm[0].quant;
  for (int i = num_segs; i < 4; i++) dqm[i].quant = base_quant;
  int dq_uv_ac = (global_uv_alpha - 64) * (6 - -4) / (100 - 30);
  dq_uv_ac = dq_uv_ac * sns / 100;
  dq_uv_ac = clampi(dq_uv_ac, -4, 6);
  const int dq_uv_dc = clampi(-4 * sns / 100, -15, 15);
  /* setupFilterStrength (encode.go:1276-1320) */
  const int sharpness = clampi(cfg->filter_sharpness, 0, 7);
  int filter_level = 0;
  if (cfg->filter_strength > 0) {
    const int level0 = 5 * cfg->filter_strength;
    const int ns = clampi(cfg->segments, 1, 4);
    for (int i = 0; i < ns; i++) {
      const int qstep = vp8_ac_table[clampi(dqm[i].quant, 0, 127)] >> 2;
      const int base = filter_strength_from_delta(sharpness, qstep);
      int f = base * level0 / (256 + dqm[i].beta);
      if (f < 2) f = 0;
      if (f > 63) f = 63;
      dqm[i].fstrength = f;
    }
    filter_level = dqm[0].fstrength;
  }
  /* simplifySegments (:197-242) */
  if (num_segs > 1) {
    int seg_map[4] = {0, 1, 2, 3};
    int num_final = 1;
    for (int s1 = 1; s1 < num_segs; s1++) {
      int found = 0;
      for (int s2 = 0; s2 < num_final; s2++)
        if (dqm[s1].quant == dqm[s2].quant && dqm[s1].fstrength == dqm[s2].fstrength) {
          seg_map[s1] = s2;
          found = 1;
          break;
        }
      if (!found) {
        seg_map[s1] = num_final;
        if (num_final != s1) dqm[num_final] = dqm[s1];
        num_final++;
      }
    }
    if (num_final < num_segs) {
      for (int i = 0; i < total; i++) seg_ids[i] = (uint8_t)seg_map[seg_ids[i]];
      for (int i = num_final; i < num_segs; i++) dqm[i] = dqm[num_final - 1];
    }
    num_segs = num_final;
  }
  /* setSegmentProbas (:874-903) */
  int counts[4] = {0, 0, 0, 0};
  for (int i = 0; i < total; i++) counts[seg_ids[i]]++;
  const int pa[3] = {counts[0] + counts[1], counts[0], counts[2]};
  const int pb[3] = {counts[2] + counts[3], counts[1], counts[3]};
  int all255 = 1;
  for (int k = 0; k < 3; k++) {
    const int t = pa[k] + pb[k];
    const int p = t == 0 ? 255 : (255 * pa[k] + t / 2) / t;
    info->seg_proba[k] = (uint8_t)p;
    if (p != 255) all255 = 0;
  }
  info->update_map = num_segs > 1; /* buildSegmentHeader (:852-857) */
  if (all255) {
    info->update_map = 0;
    for (int i = 0; i < total; i++) seg_ids[i] = 0;
  }
  info->num_segments = num_segs;
  info->base_quant = base_quant;
  info->global_uv_alpha = global_uv_alpha;
  info->dq_uv_ac = dq_uv_ac;
  info->dq_uv_dc = dq_uv_dc;
  info->filter_level = filter_level;
  for (int i = 0; i < 4; i++) {
    info->quant[i] = dqm[i].quant;
    info->fstrength[i] = dqm[i].fstrength;
    info->alpha[i] = dqm[i].alpha;
    info->beta[i] = dqm[i].beta;
  }
}
