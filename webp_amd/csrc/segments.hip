// segments.hip -- the encoder's segment analysis on the GPU: what analysis()
// does after computeAlphas and before Phase A, per image, so the encode
// pipeline stays on the device between k_analysis and k_encode_rows.
//
//   assignSegments   internal/lossy/encode_analysis.go:737-849 (k-means over
//                    the 256-bin alpha histogram, 6 iterations, displaced < 5)
//   smoothSegmentMap :76-119 (preprocessing bit 0)
//   setSegmentParams :122-195 (SNS-modulated per-segment quantiser, dq_uv
//                    deltas, setupFilterStrength encode.go:1276-1320,
//                    simplifySegments :197-242)
//   setSegmentProbas :874-903 (segment map dropped when all three tree
//                    probabilities round to 255)
//   setupSegment     internal/lossy/encode.go:1084-1181 for the 4 segments
//
// One workgroup per image.  The histogram and the per-MB assignment are
// parallel; the k-means itself is 6 passes over 256 bins and runs on one
// lane.  The only floating-point step (math.Pow in the quantiser,
// :128-142) is a host-built table indexed by the segment alpha
// (wg_encoder_config), so the kernel is integer only.
#include <math.h>
#include <string.h>

#include "vp8_tables.h"
#include "wg_common.h"

namespace {

__host__ __device__ inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__host__ __device__ inline int maxi(int a, int b) { return a > b ? a : b; }
__host__ __device__ inline int absi(int v) { return v < 0 ? -v : v; }

// initSegmentQuant, encode.go:1169-1181
__host__ __device__ void init_squant(wg_squant* sq, int dcq, int acq, int type) {
  sq->dc_quant = dcq;
  sq->dc_iquant = (1 << 17) / dcq;
  sq->dc_bias = vp8_bias_matrices[2 * type] << 9;
  sq->dc_zthresh = ((1 << 17) - 1 - sq->dc_bias) / sq->dc_iquant;
  sq->quant = acq;
  sq->iquant = (1 << 17) / acq;
  sq->bias = vp8_bias_matrices[2 * type + 1] << 9;
  sq->zthresh = ((1 << 17) - 1 - sq->bias) / sq->iquant;
  for (int i = 0; i < 16; i++) sq->sharpen[i] = 0;
}

// setupSegment, encode.go:1084-1164.  dq: {y1_dc, y2_dc, y2_ac, uv_dc, uv_ac}
__host__ __device__ void setup_segment(int q, const int* d, int method, int sns, wg_segment* s) {
  const int y1dc = vp8_dc_table[clampi(q + d[0], 0, 127)];
  const int y1ac = vp8_ac_table[clampi(q, 0, 127)];
  init_squant(&s->y1, y1dc, y1ac, 0);
  int y2dc = vp8_dc_table[clampi(q + d[1], 0, 127)] * 2;
  if (y2dc < 8) y2dc = 8;
  const int y2ac = vp8_ac_table2[clampi(q + d[2], 0, 127)];
  init_squant(&s->y2, y2dc, y2ac, 1);
  const int uvdc = vp8_dc_table[clampi(q + d[3], 0, 117)];
  const int uvac = vp8_ac_table[clampi(q + d[4], 0, 127)];
  init_squant(&s->uv, uvdc, uvac, 2);
  const int qi4 = (y1dc + 15 * y1ac + 8) >> 4, qi16 = (y2dc + 15 * y2ac + 8) >> 4, quv = (uvdc + 15 * uvac + 8) >> 4;
  s->lambda_i4 = maxi((3 * qi4 * qi4) >> 7, 1);
  s->lambda_i16 = maxi(3 * qi16 * qi16, 1);
  s->lambda_uv = maxi((3 * quv * quv) >> 6, 1);
  s->lambda_mode = maxi((qi4 * qi4) >> 7, 1);
  s->tlambda_i4 = maxi((7 * qi4 * qi4) >> 3, 1);
  s->tlambda_i16 = maxi((qi16 * qi16) >> 2, 1);
  s->tlambda_uv = maxi((quv * quv) << 1, 1);
  s->tlambda_sd = (method >= 4 && sns > 0) ? (sns * qi4) >> 5 : 0;
  for (int i = 0; i < 16; i++)
    s->y1.sharpen[i] = (int16_t)((vp8_freq_sharpening[i] * (i == 0 ? s->y1.dc_quant : s->y1.quant)) >> 11);
}

struct SegArgs {
  wg_enc_config cfg;
  const int32_t* alphas;  // [n][mbw*mbh]
  const int32_t* uv_sum;  // [n]
  uint8_t* seg_ids;       // [n][mbw*mbh]
  uint8_t* segs;          // [n] x 4 wg_segment, segs_pitch apart
  int64_t segs_pitch;
  wg_frame_segs* info;    // [n] (may be NULL)
  int mbw, mbh;
};

struct SegState {  // one SegmentInfo's analysis fields
  int quant, fstrength, alpha, beta;
};

constexpr int NT = 256;

__global__ __launch_bounds__(NT) void k_segments(SegArgs a) {
  __shared__ int histo[256];
  __shared__ uint8_t amap[256];
  __shared__ int counts[4];
  __shared__ int seg_map[4];
  __shared__ int num_segs_s, smooth_s, reset_s;
  __shared__ SegState dqm[4];
  __shared__ int dq_s[2];
  // thread 0's k-means state lives in LDS, not in dynamically indexed private
  // arrays: a kernel with scratch (private segment) memory, dispatched on a
  // queue for the first time while a persistent kernel runs on another, stalled
  // that kernel's waves for seconds on MI355X (bench.py's first overlapped
  // steps; tools/debug_timeouts.py), so no kernel here uses scratch.
  __shared__ int centers[4], accum[4], dist[4];
  const int tid = threadIdx.x, img = blockIdx.x;
  const int mbw = a.mbw, mbh = a.mbh, total = mbw * mbh;
  const int32_t* al = a.alphas + (int64_t)img * total;
  uint8_t* ids = a.seg_ids + (int64_t)img * total;
  const wg_enc_config& cfg = a.cfg;
  histo[tid] = 0;
  amap[tid] = 0;
  if (tid < 4) counts[tid] = 0;
  __syncthreads();
  const int num_segs0 = clampi(cfg.segments, 1, 4);  // analysis(), encode_analysis.go:30-36
  if (num_segs0 > 1)
    for (int i = tid; i < total; i += NT) atomicAdd(&histo[al[i] & 255], 1);
  __syncthreads();
  if (tid == 0) {
    SegState* d = dqm;
    int* map = seg_map;
    for (int k = 0; k < 4; k++) {
      d[k] = SegState{};
      map[k] = k;
    }
    int num_segs = num_segs0;
    if (num_segs > 1) {
      // assignSegments (:737-849)
      int min_a = 0;
      while (min_a <= 255 && histo[min_a] == 0) min_a++;
      int max_a = 255;
      while (max_a > min_a && histo[max_a] == 0) max_a--;
      const int range_a = max_a - min_a;
      for (int k = 0; k < 4; k++) centers[k] = 0;
      for (int k = 0; k < num_segs; k++) centers[k] = min_a + ((2 * k + 1) * range_a) / (2 * num_segs);
      int weighted_avg = 0;
      for (int iter = 0; iter < 6; iter++) {
        for (int k = 0; k < 4; k++) accum[k] = dist[k] = 0;
        int n = 0;
        for (int al_ = min_a; al_ <= max_a; al_++) {
          const int h = histo[al_];
          if (h == 0) continue;
          while (n + 1 < num_segs && absi(al_ - centers[n + 1]) < absi(al_ - centers[n])) n++;
          amap[al_] = (uint8_t)n;
          dist[n] += al_ * h;
          accum[n] += h;
        }
        int displaced = 0, total_weight = 0;
        weighted_avg = 0;
        for (int s = 0; s < num_segs; s++)
          if (accum[s] > 0) {
            const int nc = (dist[s] + accum[s] / 2) / accum[s];
            displaced += absi(centers[s] - nc);
            centers[s] = nc;
            weighted_avg += nc * accum[s];
            total_weight += accum[s];
          }
        if (total_weight > 0) weighted_avg = (weighted_avg + total_weight / 2) / total_weight;
        if (displaced < 5) break;
      }
      // SetSegmentAlphas (:825-848)
      int min_c = centers[0], max_c = centers[0];
      for (int s = 1; s < num_segs; s++) {
        min_c = min(min_c, centers[s]);
        max_c = max(max_c, centers[s]);
      }
      const int range_c = max_c - min_c == 0 ? 1 : max_c - min_c;
      for (int s = 0; s < num_segs; s++) {
        d[s].alpha = clampi(255 * (centers[s] - weighted_avg) / range_c, -127, 127);
        d[s].beta = clampi(255 * (centers[s] - min_c) / range_c, 0, 255);
      }
    }
    // setSegmentParams (:122-195): quantisers from the host-built pow table
    for (int i = 0; i < num_segs; i++) d[i].quant = cfg.seg_quant[d[i].alpha + 127];
    for (int i = num_segs; i < 4; i++) d[i].quant = d[0].quant;
    const int sns = cfg.sns_strength < 0 ? 0 : cfg.sns_strength;
    const int guv = total > 0 ? a.uv_sum[img] / total : 0;
    dq_s[0] = clampi((guv - 64) * 10 / 70 * sns / 100, -4, 6);  // dqUVAC
    dq_s[1] = clampi(-4 * sns / 100, -15, 15);                  // dqUVDC
    // setupFilterStrength (encode.go:1276-1320)
    if (cfg.filter_strength > 0) {
      const int level0 = 5 * cfg.filter_strength, sharp = clampi(cfg.filter_sharpness, 0, 7);
      for (int i = 0; i < num_segs0; i++) {
        const int qstep = vp8_ac_table[clampi(d[i].quant, 0, 127)] >> 2;
        int f = vp8_levels_from_delta[sharp * 64 + clampi(qstep, 0, 63)] * level0 / (256 + d[i].beta);
        d[i].fstrength = f < 2 ? 0 : min(f, 63);
      }
    }
    // simplifySegments (:197-242)
    if (num_segs > 1) {
      int num_final = 1;
      for (int s1 = 1; s1 < num_segs; s1++) {
        int found = 0;
        for (int s2 = 0; s2 < num_final && !found; s2++)
          if (d[s1].quant == d[s2].quant && d[s1].fstrength == d[s2].fstrength) {
            map[s1] = s2;
            found = 1;
          }
        if (!found) {
          map[s1] = num_final;
          if (num_final != s1) d[num_final] = d[s1];
          num_final++;
        }
      }
      if (num_final < num_segs)
        for (int i = num_final; i < num_segs; i++) d[i] = d[num_final - 1];
      num_segs = num_final;
    }
    num_segs_s = num_segs;
    smooth_s = num_segs0 > 1 && cfg.segments > 1 && (cfg.preprocessing & 1) && mbw >= 3 && mbh >= 3;
  }
  __syncthreads();
  // per-MB segment: alpha map (+ 3x3 majority smoothing), then the simplify remap
  const bool one = num_segs0 <= 1, smooth = smooth_s;
  for (int i = tid; i < total; i += NT) {
    int s = one ? 0 : amap[al[i] & 255];
    if (smooth) {
      const int y = i / mbw, x = i - y * mbw;
      if (y >= 1 && y < mbh - 1 && x >= 1 && x < mbw - 1) {
        int cnt = 0;  // four 8-bit counters
        for (int dy = -1; dy <= 1; dy++)
          for (int dx = -1; dx <= 1; dx++) cnt += 1 << (8 * amap[al[i + dy * mbw + dx] & 255]);
        for (int k = 0; k < 4; k++)
          if (((cnt >> (8 * k)) & 255) >= 5) s = k;
      }
    }
    s = seg_map[s];
    ids[i] = (uint8_t)s;
    atomicAdd(&counts[s], 1);
  }
  __syncthreads();
  if (tid == 0) {
    // setSegmentProbas (:874-903)
    const int pa[3] = {counts[0] + counts[1], counts[0], counts[2]};
    const int pb[3] = {counts[2] + counts[3], counts[1], counts[3]};
    int all255 = 1;
    uint32_t p = 0;  // three probabilities, a byte each (no private array)
    for (int k = 0; k < 3; k++) {
      const int t = pa[k] + pb[k];
      const uint32_t pk = t == 0 ? 255u : (uint32_t)((255 * pa[k] + t / 2) / t);
      p |= pk << (8 * k);
      all255 &= pk == 255;
    }
    reset_s = all255;
    if (a.info) {
      wg_frame_segs& o = a.info[img];
      o.num_segments = num_segs_s;
      o.base_quant = dqm[0].quant;
      o.global_uv_alpha = total > 0 ? a.uv_sum[img] / total : 0;
      o.dq_uv_ac = dq_s[0];
      o.dq_uv_dc = dq_s[1];
      o.filter_level = cfg.filter_strength > 0 ? dqm[0].fstrength : 0;
      o.update_map = num_segs_s > 1 && !all255;
      o.pad = 0;
      for (int k = 0; k < 4; k++) {
        o.quant[k] = dqm[k].quant;
        o.fstrength[k] = dqm[k].fstrength;
        o.alpha[k] = dqm[k].alpha;
        o.beta[k] = dqm[k].beta;
      }
      for (int k = 0; k < 3; k++) o.seg_proba[k] = (uint8_t)(p >> (8 * k));
      o.seg_proba[3] = 0;
      o.pad2[0] = o.pad2[1] = o.pad2[2] = 0;
    }
  }
  __syncthreads();
  if (reset_s)
    for (int i = tid; i < total; i += NT) ids[i] = 0;
  if (tid < 4) {
    const int d[5] = {0, 0, 0, dq_s[1], dq_s[0]};
    wg_segment sg;
    setup_segment(dqm[tid].quant, d, cfg.method, cfg.sns_strength, &sg);
    wg_segment* dst = reinterpret_cast<wg_segment*>(a.segs + img * a.segs_pitch) + tid;
    *dst = sg;
  }
}

}  // namespace

extern "C" int wg_setup_segment(int32_t q, const int32_t* dq, int32_t method, int32_t sns, wg_segment* s) {
  WG_REQUIRE(s);
  const int d[5] = {dq ? dq[0] : 0, dq ? dq[1] : 0, dq ? dq[2] : 0, dq ? dq[3] : 0, dq ? dq[4] : 0};
  setup_segment(q, d, method, sns, s);
  return WG_OK;
}

// qualityToCompression (encode.go:1039-1055) and setSegmentParams' pow
// (encode_analysis.go:128-142) for every segment alpha.
extern "C" int wg_encoder_config(int32_t quality, int32_t method, int32_t sns_strength, int32_t filter_strength,
                                 int32_t filter_sharpness, int32_t filter_type, int32_t segments, int32_t preprocessing,
                                 wg_enc_config* out) {
  WG_REQUIRE(out && quality >= 0 && quality <= 100 && method >= 0 && method <= 6);
  WG_REQUIRE(filter_sharpness >= 0 && filter_sharpness <= 7 && preprocessing >= 0 && preprocessing <= 3);
  memset(out, 0, sizeof(*out));
  out->quality = quality;
  out->method = method;
  out->sns_strength = sns_strength;
  out->filter_strength = filter_strength;
  out->filter_sharpness = filter_sharpness;
  out->filter_type = filter_type;
  out->segments = segments;
  out->preprocessing = preprocessing;
  double c_base;
  if (quality <= 0) {
    c_base = 0.0;
  } else if (quality >= 100) {
    c_base = 1.0;
  } else {
    const double c = (double)quality / 100.0;
    c_base = pow(c < 0.75 ? c * (2.0 / 3.0) : 2.0 * c - 1.0, 1.0 / 3.0);
  }
  const int sns = sns_strength < 0 ? 0 : sns_strength;
  const double amp = 0.9 * (double)sns / 100.0 / 128.0;
  for (int alpha = -127; alpha <= 127; alpha++) {
    const double expn = 1.0 - amp * (double)alpha;
    out->seg_quant[alpha + 127] = (uint8_t)clampi((int)(127.0 * (1.0 - pow(c_base, expn))), 0, 127);
  }
  return WG_OK;
}

extern "C" int wg_segment_analysis(const wg_enc_config* cfg, const int32_t* alphas, const int32_t* uv_sum, int32_t mbw,
                                   int32_t mbh, int32_t n_images, uint8_t* seg_ids, void* segs, int64_t segs_pitch,
                                   wg_frame_segs* info, void* stream) {
  WG_REQUIRE(cfg && alphas && uv_sum && seg_ids && segs);
  WG_REQUIRE(mbw > 0 && mbh > 0 && n_images > 0 && (int64_t)mbw * mbh < (1 << 24));
  WG_REQUIRE(segs_pitch >= (int64_t)(4 * sizeof(wg_segment)) && (segs_pitch & 15) == 0 &&
             (reinterpret_cast<uintptr_t>(segs) & 15) == 0);
  SegArgs a;
  a.cfg = *cfg;
  a.alphas = alphas;
  a.uv_sum = uv_sum;
  a.seg_ids = seg_ids;
  a.segs = static_cast<uint8_t*>(segs);
  a.segs_pitch = segs_pitch;
  a.info = info;
  a.mbw = mbw;
  a.mbh = mbh;
  hipLaunchKernelGGL(k_segments, dim3((unsigned)n_images), dim3(NT), 0, wg::as_stream(stream), a);
  return wg::check_launch("k_segments");
}
