// vp8_parse.cpp -- host-side VP8 (lossy) bitstream parser: the CPU half of
// the reference's decoder, restated as a parse-all-rows-first pass whose
// output (wg_mb_info + dequantised coefficients per macroblock) feeds
// wg_decode_frames on the GPU (SURVEY.md 8(b) "Parsing moves to a
// parse-all-rows-first CPU pass", 8(f)#2).
//
// Follows, in order:
//   frame / picture header        internal/lossy/decode.go:262-330 (parseHeaders)
//   segment / filter headers      decode.go:333-408
//   token partitions              decode.go:411-444
//   quantiser                     internal/lossy/decode_quant.go:28-75 (ParseQuant)
//   token probabilities           internal/lossy/decode_tree.go:7-31 (parseProba), proba.go:24-43
//   intra modes, per row          decode_tree.go:35-213 (parseIntraModeRow)
//   residual tokens               internal/lossy/decode_mb.go:111-430 (getCoeffs, decodeMB, parseResiduals)
//   filter strengths              internal/lossy/decode_frame.go:220-280 (precomputeFilterStrengths)
//   boolean decoder               internal/bitio/reader_bool.go:1-190
// VP8 parsing is normative (RFC 6386): any correct parser yields the same
// macroblock data; tests pin the whole decode against libwebp's WebPDecodeYUV.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/webpgpu.h"
#include "vp8_tables.h"
#include "wg_common_host.h"

namespace {

// ---------------------------------------------------------------- bool decoder
// The arithmetic of reader_bool.go (GetBit with the 56-bit look-ahead register).
struct BoolReader {
  const uint8_t* buf = nullptr;
  size_t len = 0, pos = 0;
  uint64_t value = 0;
  uint32_t range = 254;  // range - 1
  int bits = -8;
  bool eof = false;

  void init(const uint8_t* b, size_t n) {
    buf = b;
    len = n;
    pos = 0;
    value = 0;
    range = 254;
    bits = -8;
    eof = false;
    load();
  }
  void load() {
    if (pos + 8 <= len) {  // 7 fresh bytes, big-endian order
      uint64_t in = 0;
      for (int k = 0; k < 7; k++) in = (in << 8) | buf[pos + k];
      value = (value << 56) | in;
      pos += 7;
      bits += 56;
    } else if (pos < len) {
      value = (value << 8) | buf[pos++];
      bits += 8;
    } else if (!eof) {
      value <<= 8;
      bits += 8;
      eof = true;
    } else {
      bits = 0;
    }
  }
  int bit(int prob) {
    uint32_t r = range;
    if (bits < 0) load();
    const int p = bits;
    const uint32_t split = (r * (uint32_t)prob) >> 8;
    const uint32_t v = (uint32_t)(value >> p);
    int b;
    if (v > split) {
      b = 1;
      r -= split;
      value -= (uint64_t)(split + 1) << p;
    } else {
      b = 0;
      r = split + 1;
    }
    const int shift = 7 ^ (31 - __builtin_clz(r));
    r <<= shift;
    bits -= shift;
    range = r - 1;
    return b;
  }
  uint32_t get(int n) {
    uint32_t v = 0;
    while (n-- > 0) v |= (uint32_t)bit(0x80) << n;
    return v;
  }
  int32_t get_signed_value(int n) {
    const int32_t v = (int32_t)get(n);
    return bit(0x80) ? -v : v;
  }
  int signed_of(int v) {  // GetSigned (prob 1/2), reader_bool.go:159-177
    if (bits < 0) load();
    const int p = bits;
    const uint32_t split = range >> 1;
    const uint32_t val = (uint32_t)(value >> p);
    const int32_t mask = (int32_t)(split - val) >> 31;
    bits--;
    range = (range + (uint32_t)mask) | 1;
    value -= (uint64_t)((split + 1) & (uint32_t)mask) << p;
    return (v ^ mask) - mask;
  }
};

struct QuantMat {
  int y1[2], y2[2], uv[2];
};
struct FStrength {
  uint8_t limit, ilevel, inner, hev;
};

constexpr int kNumTypes = 4, kNumBands = 8, kNumCtx = 3, kNumProbas = 11;

struct Parser {
  BoolReader br;
  BoolReader parts[8];
  int num_parts_m1 = 0;
  int width = 0, height = 0, mbw = 0, mbh = 0;
  // segment header
  bool use_segment = false, update_map = false, absolute_delta = true;
  int8_t seg_q[4] = {0, 0, 0, 0}, seg_f[4] = {0, 0, 0, 0};
  uint8_t seg_proba[3] = {255, 255, 255};
  // filter header
  bool simple = false, use_lf_delta = false;
  int level = 0, sharpness = 0, ref_lf_delta0 = 0, mode_lf_delta0 = 0;
  int filter_type = 0;
  QuantMat dqm[4];
  uint8_t proba[kNumTypes][kNumBands][kNumCtx][kNumProbas];
  bool use_skip = false;
  int skip_p = 0;
  FStrength fstr[4][2];
};

int fail(const char* msg) {
  wg::set_error(msg);
  return WG_EINVAL;
}

int clampi(int v, int hi) { return v < 0 ? 0 : (v > hi ? hi : v); }

int parse_headers(Parser& P, const uint8_t* data, size_t size) {
  if (size < 10) return fail("vp8: truncated header");
  const uint32_t bits = data[0] | (data[1] << 8) | (data[2] << 16);
  const bool key = (bits & 1) == 0;
  const int profile = (bits >> 1) & 7;
  const bool show = (bits >> 4) & 1;
  const uint32_t part0 = bits >> 5;
  if (profile > 3) return fail("vp8: bad profile");
  if (!show) return fail("vp8: frame not displayable");
  if (!key) return fail("vp8: not a keyframe");
  const uint8_t* b = data + 3;
  if (b[0] != 0x9d || b[1] != 0x01 || b[2] != 0x2a) return fail("vp8: bad signature");
  P.width = (b[3] | (b[4] << 8)) & 0x3fff;
  P.height = (b[5] | (b[6] << 8)) & 0x3fff;
  if (P.width == 0 || P.height == 0) return fail("vp8: zero dimensions");
  P.mbw = (P.width + 15) >> 4;
  P.mbh = (P.height + 15) >> 4;
  b += 7;
  size_t left = size - 10;
  if (part0 > left) return fail("vp8: bad partition length");
  BoolReader& br = P.br;
  br.init(b, part0);
  const uint8_t* tokens = b + part0;
  size_t tokens_len = left - part0;

  br.bit(0x80);  // colorspace
  br.bit(0x80);  // clamp type
  // segment header (decode.go:333-375)
  P.use_segment = br.bit(0x80);
  if (P.use_segment) {
    P.update_map = br.bit(0x80);
    if (br.bit(0x80)) {
      P.absolute_delta = br.bit(0x80);
      for (int s = 0; s < 4; s++) P.seg_q[s] = br.bit(0x80) ? (int8_t)br.get_signed_value(7) : 0;
      for (int s = 0; s < 4; s++) P.seg_f[s] = br.bit(0x80) ? (int8_t)br.get_signed_value(6) : 0;
    }
    if (P.update_map)
      for (int s = 0; s < 3; s++) P.seg_proba[s] = br.bit(0x80) ? (uint8_t)br.get(8) : 255;
  }
  if (br.eof) return fail("vp8: premature EOF in segment header");
  // filter header (decode.go:378-408)
  P.simple = br.bit(0x80);
  P.level = (int)br.get(6);
  P.sharpness = (int)br.get(3);
  P.use_lf_delta = br.bit(0x80);
  if (P.use_lf_delta && br.bit(0x80)) {
    for (int i = 0; i < 4; i++)
      if (br.bit(0x80)) {
        const int v = br.get_signed_value(6);
        if (i == 0) P.ref_lf_delta0 = v;
      }
    for (int i = 0; i < 4; i++)
      if (br.bit(0x80)) {
        const int v = br.get_signed_value(6);
        if (i == 0) P.mode_lf_delta0 = v;
      }
  }
  P.filter_type = P.level == 0 ? 0 : (P.simple ? 1 : 2);
  // token partitions (decode.go:411-444)
  P.num_parts_m1 = (1 << br.get(2)) - 1;
  const int last = P.num_parts_m1;
  if (tokens_len < (size_t)3 * last) return fail("vp8: not enough data for partition sizes");
  const uint8_t* sz = tokens;
  const uint8_t* start = tokens + 3 * last;
  size_t size_left = tokens_len - 3 * last;
  for (int p = 0; p < last; p++) {
    const size_t psize = sz[0] | (sz[1] << 8) | (sz[2] << 16);
    if (psize > size_left) return fail("vp8: partition size exceeds data");
    P.parts[p].init(start, psize);
    start += psize;
    size_left -= psize;
    sz += 3;
  }
  P.parts[last].init(start, size_left);
  // quantiser (decode_quant.go:28-66)
  const int base_q0 = (int)br.get(7);
  int dq[5];
  for (int k = 0; k < 5; k++) dq[k] = br.bit(0x80) ? br.get_signed_value(4) : 0;
  const int dqy1_dc = dq[0], dqy2_dc = dq[1], dqy2_ac = dq[2], dquv_dc = dq[3], dquv_ac = dq[4];
  for (int i = 0; i < 4; i++) {
    int q;
    if (P.use_segment) {
      q = P.seg_q[i];
      if (!P.absolute_delta) q += base_q0;
    } else {
      if (i > 0) {
        P.dqm[i] = P.dqm[0];
        continue;
      }
      q = base_q0;
    }
    QuantMat& m = P.dqm[i];
    m.y1[0] = vp8_dc_table[clampi(q + dqy1_dc, 127)];
    m.y1[1] = vp8_ac_table[clampi(q, 127)];
    m.y2[0] = vp8_dc_table[clampi(q + dqy2_dc, 127)] * 2;
    m.y2[1] = (vp8_ac_table[clampi(q + dqy2_ac, 127)] * 101581) >> 16;
    if (m.y2[1] < 8) m.y2[1] = 8;
    m.uv[0] = vp8_dc_table[clampi(q + dquv_dc, 117)];
    m.uv[1] = vp8_ac_table[clampi(q + dquv_ac, 127)];
  }
  br.bit(0x80);  // update_proba flag (ignored for key frames)
  // token probabilities (decode_tree.go:7-31)
  int k = 0;
  for (int t = 0; t < kNumTypes; t++)
    for (int bd = 0; bd < kNumBands; bd++)
      for (int c = 0; c < kNumCtx; c++)
        for (int p = 0; p < kNumProbas; p++, k++)
          P.proba[t][bd][c][p] =
              br.bit(vp8_coeffs_update_proba[k]) ? (uint8_t)br.get(8) : vp8_coeffs_proba0[k];
  P.use_skip = br.bit(0x80);
  if (P.use_skip) P.skip_p = (int)br.get(8);
  // filter strengths (decode_frame.go:220-280)
  for (int s = 0; s < 4; s++) {
    int base = P.use_segment ? P.seg_f[s] + (P.absolute_delta ? 0 : P.level) : P.level;
    for (int i4 = 0; i4 <= 1; i4++) {
      FStrength& f = P.fstr[s][i4];
      int lv = base;
      if (P.use_lf_delta) {
        lv += P.ref_lf_delta0;
        if (i4) lv += P.mode_lf_delta0;
      }
      lv = lv < 0 ? 0 : (lv > 63 ? 63 : lv);
      if (lv > 0) {
        int il = lv;
        if (P.sharpness > 0) {
          il >>= (P.sharpness > 4) ? 2 : 1;
          if (il > 9 - P.sharpness) il = 9 - P.sharpness;
        }
        if (il < 1) il = 1;
        f.ilevel = (uint8_t)il;
        f.limit = (uint8_t)(2 * lv + il);
        f.hev = lv >= 40 ? 2 : (lv >= 15 ? 1 : 0);
      } else {
        f.limit = 0;
        f.ilevel = 0;
        f.hev = 0;
      }
      f.inner = (uint8_t)i4;
    }
  }
  return WG_OK;
}

// getCoeffs (decode_mb.go:111-270): tokens of one 4x4 block starting at
// position n, dequantised into out[zigzag]; returns the index after the last
// non-zero coefficient (16 when the block runs to the end).
int get_coeffs(BoolReader& br, const uint8_t (*bands)[kNumCtx][kNumProbas], int ctx, int dq0, int dq1, int n,
               int16_t* out) {
  const uint8_t* p = bands[vp8_bands[n]][ctx];
  for (; n < 16; n++) {
    if (!br.bit(p[0])) return n;
    while (!br.bit(p[1])) {
      n++;
      if (n == 16) return 16;
      p = bands[vp8_bands[n]][0];
    }
    const uint8_t (*next)[kNumProbas] = bands[vp8_bands[n + 1]];
    int v;
    if (!br.bit(p[2])) {
      v = 1;
      p = next[1];
    } else {
      if (!br.bit(p[3])) {
        if (!br.bit(p[4])) v = 2;
        else v = 3 + br.bit(p[5]);
      } else if (!br.bit(p[6])) {
        if (!br.bit(p[7])) {
          v = 5 + br.bit(159);
        } else {
          v = 7 + 2 * br.bit(165);
          v += br.bit(145);
        }
      } else {
        const int b1 = br.bit(p[8]);
        const int b0 = br.bit(p[9 + b1]);
        const int cat = 2 * b1 + b0;
        static const uint8_t* const kCat[4] = {vp8_cat3, vp8_cat4, vp8_cat5, vp8_cat6};
        v = 0;
        for (const uint8_t* tp = kCat[cat]; *tp; tp++) v = v + v + br.bit(*tp);
        v += 3 + (8 << cat);
      }
      p = next[2];
    }
    const int dq = n == 0 ? dq0 : dq1;
    out[vp8_zigzag[n]] = (int16_t)(br.signed_of(v) * dq);
  }
  return 16;
}

uint32_t nz_code_bits(uint32_t nz_coeffs, int nz, int dc_nz) {
  nz_coeffs <<= 2;
  nz_coeffs |= nz > 3 ? 3 : (nz > 1 ? 2 : (uint32_t)dc_nz);
  return nz_coeffs;
}

// inverse WHT of the I16 DCs into the 16 luma blocks (transforms.go:223-252)
void transform_wht(const int16_t* in, int16_t* out) {
  int tmp[16];
  for (int i = 0; i < 4; i++) {
    const int a0 = in[i] + in[12 + i], a1 = in[4 + i] + in[8 + i];
    const int a2 = in[4 + i] - in[8 + i], a3 = in[i] - in[12 + i];
    tmp[i] = a0 + a1;
    tmp[8 + i] = a0 - a1;
    tmp[4 + i] = a3 + a2;
    tmp[12 + i] = a3 - a2;
  }
  for (int i = 0; i < 4; i++) {
    const int dc = tmp[4 * i] + 3;
    const int a0 = dc + tmp[4 * i + 3], a1 = tmp[4 * i + 1] + tmp[4 * i + 2];
    const int a2 = tmp[4 * i + 1] - tmp[4 * i + 2], a3 = dc - tmp[4 * i + 3];
    out[16 * (4 * i + 0)] = (int16_t)((a0 + a1) >> 3);
    out[16 * (4 * i + 1)] = (int16_t)((a3 + a2) >> 3);
    out[16 * (4 * i + 2)] = (int16_t)((a0 - a1) >> 3);
    out[16 * (4 * i + 3)] = (int16_t)((a3 - a2) >> 3);
  }
}

struct NzCtx {
  uint8_t nz = 0, nz_dc = 0;
};

// parseResiduals (decode_mb.go:328-430) for one macroblock.
void parse_residuals(Parser& P, BoolReader& tbr, NzCtx& mb, NzCtx& left, wg_mb_info& info, int16_t* dst) {
  const QuantMat& q = P.dqm[info.segment & 3];
  memset(dst, 0, 384 * sizeof(int16_t));
  uint32_t non_zero_y = 0, non_zero_uv = 0;
  int first;
  int ac_type;
  if (!info.is_i4x4) {
    int16_t dc[16] = {0};
    const int ctx = mb.nz_dc + left.nz_dc;
    const int nz = get_coeffs(tbr, P.proba[1], ctx, q.y2[0], q.y2[1], 0, dc);
    mb.nz_dc = left.nz_dc = nz > 0;
    if (nz > 1) {
      transform_wht(dc, dst);
    } else {
      const int16_t dc0 = (int16_t)((dc[0] + 3) >> 3);
      for (int i = 0; i < 256; i += 16) dst[i] = dc0;
    }
    first = 1;
    ac_type = 0;
  } else {
    first = 0;
    ac_type = 3;
  }
  uint32_t tnz = mb.nz & 0x0f, lnz = left.nz & 0x0f;
  int16_t* d = dst;
  for (int y = 0; y < 4; y++) {
    uint32_t l = lnz & 1, nz_coeffs = 0;
    for (int x = 0; x < 4; x++) {
      const int ctx = (int)(l + (tnz & 1));
      const int nz = get_coeffs(tbr, P.proba[ac_type], ctx, q.y1[0], q.y1[1], first, d);
      l = nz > first;
      tnz = (tnz >> 1) | (l << 7);
      nz_coeffs = nz_code_bits(nz_coeffs, nz, d[0] != 0);
      d += 16;
    }
    tnz >>= 4;
    lnz = (lnz >> 1) | (l << 7);
    non_zero_y = (non_zero_y << 8) | nz_coeffs;
  }
  uint32_t out_t = tnz, out_l = lnz >> 4;
  for (int ch = 0; ch < 4; ch += 2) {
    uint32_t nz_coeffs = 0;
    tnz = mb.nz >> (4 + ch);
    lnz = left.nz >> (4 + ch);
    for (int y = 0; y < 2; y++) {
      uint32_t l = lnz & 1;
      for (int x = 0; x < 2; x++) {
        const int ctx = (int)(l + (tnz & 1));
        const int nz = get_coeffs(tbr, P.proba[2], ctx, q.uv[0], q.uv[1], 0, d);
        l = nz > 0;
        tnz = (tnz >> 1) | (l << 3);
        nz_coeffs = nz_code_bits(nz_coeffs, nz, d[0] != 0);
        d += 16;
      }
      tnz >>= 2;
      lnz = (lnz >> 1) | (l << 5);
    }
    non_zero_uv |= nz_coeffs << (4 * ch);
    out_t |= (tnz << 4) << ch;
    out_l |= (lnz & 0xf0) << ch;
  }
  mb.nz = (uint8_t)out_t;
  left.nz = (uint8_t)out_l;
  info.non_zero_y = non_zero_y;
  info.non_zero_uv = non_zero_uv;
}

// parseIntraModeRow (decode_tree.go:35-213) for one macroblock.
int parse_modes(Parser& P, uint8_t* top, uint8_t* left, wg_mb_info& info) {
  BoolReader& br = P.br;
  if (P.update_map)
    info.segment = !br.bit(P.seg_proba[0]) ? (uint8_t)br.bit(P.seg_proba[1]) : (uint8_t)(br.bit(P.seg_proba[2]) + 2);
  else
    info.segment = 0;
  info.skip = P.use_skip ? (uint8_t)br.bit(P.skip_p) : 0;
  info.is_i4x4 = !br.bit(145);
  if (!info.is_i4x4) {
    int ymode;
    if (br.bit(156)) ymode = br.bit(128) ? 1 /*TM*/ : 3 /*H*/;
    else ymode = br.bit(163) ? 2 /*V*/ : 0 /*DC*/;
    info.imodes[0] = (uint8_t)ymode;
    memset(top, ymode, 4);
    memset(left, ymode, 4);
  } else {
    for (int y = 0; y < 4; y++) {
      int ymode = left[y];
      for (int x = 0; x < 4; x++) {
        const uint8_t* prob = vp8_bmodes_proba + (top[x] * 10 + ymode) * 9;
        int i = vp8_ymodes_intra4[br.bit(prob[0])];
        while (i > 0) i = vp8_ymodes_intra4[2 * i + br.bit(prob[i])];
        ymode = -i;
        if (ymode >= 10) return fail("vp8: invalid 4x4 intra mode");
        top[x] = (uint8_t)ymode;
        info.imodes[y * 4 + x] = (uint8_t)ymode;
      }
      left[y] = (uint8_t)ymode;
    }
  }
  if (!br.bit(142)) info.uv_mode = 0;
  else if (!br.bit(114)) info.uv_mode = 2;
  else info.uv_mode = br.bit(183) ? 1 : 3;
  return WG_OK;
}

// Locate the VP8 frame inside a RIFF/WEBP container ("VP8 " chunk), or accept
// a raw VP8 frame (container parsing: the reference's internal/container).
bool find_vp8(const uint8_t* d, size_t n, const uint8_t** frame, size_t* len) {
  if (n >= 12 && !memcmp(d, "RIFF", 4) && !memcmp(d + 8, "WEBP", 4)) {
    size_t off = 12;
    while (off + 8 <= n) {
      const size_t csz = d[off + 4] | (d[off + 5] << 8) | (d[off + 6] << 16) | ((size_t)d[off + 7] << 24);
      if (!memcmp(d + off, "VP8 ", 4)) {
        if (off + 8 + csz > n) return false;
        *frame = d + off + 8;
        *len = csz;
        return true;
      }
      off += 8 + csz + (csz & 1);
    }
    return false;
  }
  *frame = d;
  *len = n;
  return true;
}

}  // namespace

extern "C" int wg_vp8_parse(const uint8_t* data, size_t size, int32_t* dims, wg_mb_info* mb, int16_t* coeffs,
                            int64_t max_mbs) {
  WG_REQUIRE(data && dims);
  const uint8_t* frame;
  size_t len;
  if (!find_vp8(data, size, &frame, &len)) return fail("vp8: no VP8 chunk in RIFF container");
  Parser P;
  const int rc = parse_headers(P, frame, len);
  if (rc != WG_OK) return rc;
  dims[0] = P.width;
  dims[1] = P.height;
  dims[2] = P.filter_type;
  dims[3] = P.mbw;
  dims[4] = P.mbh;
  if (!mb) return WG_OK;  // header query
  WG_REQUIRE(coeffs && max_mbs >= (int64_t)P.mbw * P.mbh);
  std::vector<uint8_t> intra_t(4 * (size_t)P.mbw, 0);  // B_DC_PRED
  std::vector<NzCtx> nz_top(P.mbw);
  for (int y = 0; y < P.mbh; y++) {
    uint8_t intra_l[4] = {0, 0, 0, 0};
    NzCtx nz_left;
    BoolReader& tbr = P.parts[y & P.num_parts_m1];
    for (int x = 0; x < P.mbw; x++) {
      wg_mb_info& info = mb[(size_t)y * P.mbw + x];
      memset(&info, 0, sizeof(info));
      const int r = parse_modes(P, &intra_t[4 * x], intra_l, info);
      if (r != WG_OK) return r;
      int16_t* co = coeffs + ((size_t)y * P.mbw + x) * 384;
      const bool skip = P.use_skip && info.skip;
      if (!skip) {
        parse_residuals(P, tbr, nz_top[x], nz_left, info, co);
      } else {
        nz_left.nz = nz_top[x].nz = 0;
        if (!info.is_i4x4) nz_left.nz_dc = nz_top[x].nz_dc = 0;
        info.non_zero_y = info.non_zero_uv = 0;
        memset(co, 0, 384 * sizeof(int16_t));
      }
      info.skip = skip;
      if (P.filter_type > 0) {  // decodeMB (decode_mb.go:290-296)
        const FStrength& f = P.fstr[info.segment & 3][info.is_i4x4 ? 1 : 0];
        info.f_limit = f.limit;
        info.f_ilevel = f.ilevel;
        info.f_inner = (uint8_t)(f.inner || !skip);
        info.hev_thresh = f.hev;
      }
      if (tbr.eof) return fail("vp8: premature end of data");
    }
    if (P.br.eof) return fail("vp8: premature end of data (modes)");
  }
  return WG_OK;
}
