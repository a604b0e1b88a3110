// encode_host.cpp -- host-side segment setup for the encoder RD kernel:
// setupSegment / initSegmentQuant (internal/lossy/encode.go:1085-1181).
#include <string.h>

#include "vp8_tables.h"
#include "wg_common_host.h"

namespace {
int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
int maxi(int a, int b) { return a > b ? a : b; }
void init_squant(wg_squant* sq, int dcq, int acq, int type) {
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
}  // namespace

extern "C" int wg_setup_segment(int32_t q, const int32_t* dq, int32_t method, int32_t sns, wg_segment* s) {
  WG_REQUIRE(s);
  const int d[5] = {dq ? dq[0] : 0, dq ? dq[1] : 0, dq ? dq[2] : 0, dq ? dq[3] : 0, dq ? dq[4] : 0};
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
  return WG_OK;
}
