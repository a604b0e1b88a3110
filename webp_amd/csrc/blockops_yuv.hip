// blockops_yuv.hip -- the rest of the block-level layer of include/webpgpu.h:
// the internal/dsp functions that the frame kernels run fused (k_upsample,
// k_import, k_ssim, the encoder's distortion) exposed one reference function
// at a time, batched over n caller-owned instances, so a Go host can replace
// each function variable one for one (SURVEY 8(b) layer 1):
//
//   UpsampleLinePair / UpsampleLinePairNRGBA   upsample.go:45-236,
//                                              upsample_direct_amd64.go:10-134
//   PointSampleRow                             upsample.go:238-245
//   ConvertARGBToY / ConvertARGBToUV           yuv.go:270-330
//   AccumulateRGBA                             yuv.go:486-547
//   ConvertRGBA32ToUV / ...Dithered + VP8Random  yuv.go:553-576, random.go:17-79
//   SSE / PSNRFromSSE                          ssim.go:163-181
//   DistoStats accumulation / SSIMFromStats[Clipped]  ssim.go:12-112
//
// Every output element is independent except the dithered conversion, whose
// VP8Random draws are a serial sequence per instance (one lane per instance,
// its 55-word table in LDS).  All of it is byte / integer work bounded by
// HBM; the fixed-point arithmetic is wg_yuv.h's, shared with the frame kernels.
#include "wg_common.h"
#include "wg_dsp.h"
#include "wg_yuv.h"

namespace {
using namespace wg;

constexpr int TPB = 256;

// ---- UpsampleLinePair[NRGBA]: one thread per (instance, output column) ----
struct LpArgs {
  const uint8_t *top_y, *bot_y, *top_u, *top_v, *bot_u, *bot_v, *alpha_top, *alpha_bot;
  uint8_t *top_dst, *bot_dst;
  int64_t y_step, uv_step, dst_step, alpha_step;
  int width, nrgba;
};

__device__ __forceinline__ void put_px(uint8_t* dst, int x, int nrgba, uint32_t rgba) {
  if (nrgba) {
    *reinterpret_cast<uint32_t*>(dst + 4 * x) = rgba;  // callers' rows are 4-byte aligned (checked)
  } else {
    dst[3 * x] = byte_of(rgba, 0);
    dst[3 * x + 1] = byte_of(rgba, 1);
    dst[3 * x + 2] = byte_of(rgba, 2);
  }
}

// The per-channel form of the packed-UV diamond kernel: the u and v halves of
// loadUV's word never carry into each other and only their low 8 bits are
// kept, so each channel is the same integer expression on its own.
__global__ void __launch_bounds__(TPB) k_line_pairs(const LpArgs a) {
  const int x = blockIdx.x * TPB + threadIdx.x;
  const int64_t i = blockIdx.y;
  const int w = a.width;
  if (x >= w) return;
  const uint8_t* cu[2] = {a.top_u + i * a.uv_step, a.bot_u + i * a.uv_step};
  const uint8_t* cv[2] = {a.top_v + i * a.uv_step, a.bot_v + i * a.uv_step};
  const bool bot = a.bot_y != nullptr;
  int tu, tv, bu, bv;  // the interpolated chroma of the top / bottom pixel
  const bool edge = x == 0 || ((w & 1) == 0 && x == w - 1);
  if (edge) {  // vertical interpolation only: first pixel, and the last one of even widths
    const int c = x == 0 ? 0 : (w - 1) >> 1;
    const int tlu = cu[0][c], lu = cu[1][c], tlv = cv[0][c], lv = cv[1][c];
    tu = (3 * tlu + lu + 2) >> 2;
    tv = (3 * tlv + lv + 2) >> 2;
    bu = (3 * lu + tlu + 2) >> 2;
    bv = (3 * lv + tlv + 2) >> 2;
  } else {
    const int c = (x + 1) >> 1;  // the pair (2c - 1, 2c)
    int o[2][2];
#pragma unroll
    for (int ch = 0; ch < 2; ch++) {
      const uint8_t* const* p = ch ? cv : cu;
      const int tl = p[0][c - 1], t = p[0][c], l = p[1][c - 1], cur = p[1][c];
      const int avg = tl + t + l + cur + 8;
      const int diag12 = (avg + 2 * (t + l)) >> 3, diag03 = (avg + 2 * (tl + cur)) >> 3;
      o[ch][0] = (x & 1) ? (diag12 + tl) >> 1 : (diag03 + t) >> 1;   // top
      o[ch][1] = (x & 1) ? (diag03 + l) >> 1 : (diag12 + cur) >> 1;  // bottom
    }
    tu = o[0][0], tv = o[1][0], bu = o[0][1], bv = o[1][1];
  }
  const int at = a.alpha_top ? a.alpha_top[i * a.alpha_step + x] : 255;
  put_px(a.top_dst + i * a.dst_step, x, a.nrgba, yuv_to_rgba(a.top_y[i * a.y_step + x], tu, tv, at));
  if (bot) {
    const int ab = a.alpha_bot ? a.alpha_bot[i * a.alpha_step + x] : 255;
    put_px(a.bot_dst + i * a.dst_step, x, a.nrgba, yuv_to_rgba(a.bot_y[i * a.y_step + x], bu, bv, ab));
  }
}

// ---- PointSampleRow: one thread per (instance, pair of output pixels) ----
// A pixel pair shares its chroma sample; its 6 RGB bytes leave as three 2-B
// stores where the rows are 2-byte aligned, else as byte stores.
__global__ void __launch_bounds__(TPB) k_point_sample(const uint8_t* y, const uint8_t* u, const uint8_t* v,
                                                      int64_t y_step, int64_t uv_step, uint8_t* dst, int64_t dst_step,
                                                      int width, int wide) {
  const int c = blockIdx.x * TPB + threadIdx.x;  // chroma column = pixels 2c, 2c + 1
  const int64_t i = blockIdx.y;
  if (2 * c >= width) return;
  const uint8_t* yr = y + i * y_step;
  const int cu = u[i * uv_step + c], cv = v[i * uv_step + c];
  const uint32_t p0 = yuv_to_rgba(yr[2 * c], cu, cv, 0);
  uint8_t* d = dst + i * dst_step + 6 * (int64_t)c;
  if (2 * c + 1 < width) {
    const uint32_t p1 = yuv_to_rgba(yr[2 * c + 1], cu, cv, 0);
    if (wide) {  // r0 g0 | b0 r1 | g1 b1
      uint16_t* h = reinterpret_cast<uint16_t*>(d);
      h[0] = (uint16_t)(p0 & 0xffff);
      h[1] = (uint16_t)(((p0 >> 16) & 0xff) | (p1 & 0xff) << 8);
      h[2] = (uint16_t)((p1 >> 8) & 0xffff);
    } else {
      d[0] = byte_of(p0, 0), d[1] = byte_of(p0, 1), d[2] = byte_of(p0, 2);
      d[3] = byte_of(p1, 0), d[4] = byte_of(p1, 1), d[5] = byte_of(p1, 2);
    }
  } else {
    d[0] = byte_of(p0, 0), d[1] = byte_of(p0, 1), d[2] = byte_of(p0, 2);
  }
}

// ---- ConvertARGBToY: one thread per (instance, pixel) ----
__global__ void __launch_bounds__(TPB) k_argb_to_y(const uint32_t* argb, int64_t argb_pitch, uint8_t* y,
                                                   int64_t y_pitch, int width) {
  const int x = blockIdx.x * TPB + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (x >= width) return;
  const uint32_t p = argb[i * argb_pitch + x];
  y[i * y_pitch + x] = (uint8_t)rgb_to_y((int)byte_of(p, 2), (int)byte_of(p, 1), (int)byte_of(p, 0));
}

// ---- ConvertARGBToUV: one thread per (instance, U/V sample) ----
// A pair's channels are doubled into the sum-of-4 scale (the odd last pixel
// x4); do_store writes the sample, else rounds it into the existing one.
__global__ void __launch_bounds__(TPB) k_argb_to_uv(const uint32_t* argb, int64_t argb_pitch, uint8_t* u, uint8_t* v,
                                                    int64_t uv_pitch, int src_width, int do_store) {
  const int k = blockIdx.x * TPB + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (k >= (src_width + 1) >> 1) return;
  const uint32_t* p = argb + i * argb_pitch + 2 * (int64_t)k;
  int r, g, b;
  if (2 * k + 1 < src_width) {
    const uint32_t v0 = p[0], v1 = p[1];
    r = 2 * ((int)byte_of(v0, 2) + (int)byte_of(v1, 2));
    g = 2 * ((int)byte_of(v0, 1) + (int)byte_of(v1, 1));
    b = 2 * ((int)byte_of(v0, 0) + (int)byte_of(v1, 0));
  } else {
    const uint32_t v0 = p[0];
    r = 4 * (int)byte_of(v0, 2);
    g = 4 * (int)byte_of(v0, 1);
    b = 4 * (int)byte_of(v0, 0);
  }
  int tu = clip_uv(-9719 * r - 19081 * g + 28800 * b), tv = clip_uv(28800 * r - 24116 * g - 4684 * b);
  uint8_t* uo = u + i * uv_pitch + k;
  uint8_t* vo = v + i * uv_pitch + k;
  if (!do_store) {
    tu = (*uo + tu + 1) >> 1;
    tv = (*vo + tv + 1) >> 1;
  }
  *uo = (uint8_t)tu;
  *vo = (uint8_t)tv;
}

// ---- AccumulateRGBA: one thread per (instance, 2x2 quad) ----
struct AccArgs {
  const uint8_t *r, *g, *b, *a;
  uint16_t* dst;
  int64_t in_pitch, dst_pitch;
  int stride, width;
  GammaTabs tabs;
};

__global__ void __launch_bounds__(TPB) k_accumulate_rgba(const AccArgs p) {
  __shared__ uint32_t tl[256], tg[34];
  tl[threadIdx.x] = p.tabs.to_lin[threadIdx.x];
  if (threadIdx.x < 34) tg[threadIdx.x] = p.tabs.to_gamma[threadIdx.x];
  __syncthreads();
  const int q = blockIdx.x * TPB + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (q >= (p.width + 1) >> 1) return;
  const int j = 2 * q, s = p.stride;
  const bool odd = j + 1 >= p.width;  // the odd last column: SUM2 vertically (:519-546)
  const int j1 = odd ? j : j + 1;
  const uint8_t* A = p.a + i * p.in_pitch;
  const uint32_t a0 = A[j], a1 = A[j1], a2 = A[j + s], a3 = A[j1 + s];
  const uint32_t ta = odd ? 2 * (a0 + a2) : a0 + a1 + a2 + a3;
  const bool plain = ta == 4 * 255 || ta == 0;
  const uint32_t inv = plain ? 0u : (1u << 19) / ta;  // kInvAlpha[ta] (yuv.go:343-447)
  uint16_t* d = p.dst + i * p.dst_pitch + 4 * (int64_t)q;
  const uint8_t* ch[3] = {p.r + i * p.in_pitch, p.g + i * p.in_pitch, p.b + i * p.in_pitch};
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const uint32_t l0 = tl[ch[c][j]], l1 = tl[ch[c][j1]], l2 = tl[ch[c][j + s]], l3 = tl[ch[c][j1 + s]];
    int v;
    if (plain)  // SUM4 / SUM2 then LinearToGamma (shift 0 / 1)
      v = odd ? lin_to_gamma(tg, l0 + l2, 1) : lin_to_gamma(tg, l0 + l1 + l2 + l3, 0);
    else  // LinearToGammaWeighted: divideByAlpha = (sum * kInvAlpha) >> (19 - 2)
      v = lin_to_gamma(tg, ((a0 * l0 + a1 * l1 + a2 * l2 + a3 * l3) * inv) >> 17, 0);
    d[c] = (uint16_t)v;
  }
  d[3] = (uint16_t)ta;
}

// ---- ConvertRGBA32ToUV: one thread per (instance, column) ----
__global__ void __launch_bounds__(TPB) k_rgba32_to_uv(const uint16_t* rgb, int64_t rgb_pitch, uint8_t* u, uint8_t* v,
                                                      int64_t uv_pitch, int width) {
  const int x = blockIdx.x * TPB + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (x >= width) return;
  const uint16_t* p = rgb + i * rgb_pitch + 4 * (int64_t)x;
  const int r = p[0], g = p[1], b = p[2];
  u[i * uv_pitch + x] = (uint8_t)clip_uv(-9719 * r - 19081 * g + 28800 * b);  // rounding YUV_HALF << 2
  v[i * uv_pitch + x] = (uint8_t)clip_uv(28800 * r - 24116 * g - 4684 * b);
}

// ---- ConvertRGBA32ToUVDithered: one lane per instance (VP8Random is serial) ----
constexpr int DITHER_T = 64;
__global__ void __launch_bounds__(DITHER_T) k_rgba32_to_uv_dithered(const uint16_t* rgb, int64_t rgb_pitch, uint8_t* u,
                                                                    uint8_t* v, int64_t uv_pitch, int width,
                                                                    wg_random* state, int n) {
  __shared__ uint32_t tab[DITHER_T][56];
  const int t = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * DITHER_T + t;
  if (i >= n) return;
  wg_random* st = state + i;
  for (int k = 0; k < 55; k++) tab[t][k] = st->tab[k];
  int i1 = st->index1, i2 = st->index2;
  const int amp = st->amp;
  auto bits18 = [&]() {  // RandomBits(rg, YUV_FIX + 2) (random.go:54-79)
    int64_t diff = (int64_t)tab[t][i1] - (int64_t)tab[t][i2];
    if (diff < 0) diff += (int64_t)1 << 31;
    tab[t][i1] = (uint32_t)diff;
    if (++i1 == 55) i1 = 0;
    if (++i2 == 55) i2 = 0;
    int64_t d = (int64_t)(int32_t)((uint32_t)diff << 1) >> (32 - 18);
    d = (d * amp) >> 8;
    return (int)(d + (1 << 17));
  };
  const uint16_t* p = rgb + i * rgb_pitch;
  uint8_t* uo = u + i * uv_pitch;
  uint8_t* vo = v + i * uv_pitch;
  for (int x = 0; x < width; x++) {
    const int r = p[4 * x], g = p[4 * x + 1], b = p[4 * x + 2];
    const int ru = bits18();  // U's draw first, then V's (yuv.go:573-574)
    uo[x] = (uint8_t)clip_uv(-9719 * r - 19081 * g + 28800 * b, ru);
    const int rv = bits18();
    vo[x] = (uint8_t)clip_uv(28800 * r - 24116 * g - 4684 * b, rv);
  }
  for (int k = 0; k < 55; k++) st->tab[k] = tab[t][k];
  st->index1 = i1;
  st->index2 = i2;
}

// ---- SSE and DistoStats: block-strided reductions per instance ----
// grid (chunks, n); every sum is an integer sum (uint64 SSE, Go's wrapping
// uint32 DistoStats fields), so the reduction order does not matter.
struct RedArgs {
  const uint8_t *pix, *ref;
  int64_t pix_pitch, ref_pitch;
  int pix_stride, ref_stride, width, height;
};

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(TPB) k_sse(const RedArgs a, unsigned long long* out) {
  const int64_t i = blockIdx.y;
  const uint8_t* P = a.pix + i * a.pix_pitch;
  const uint8_t* R = a.ref + i * a.ref_pitch;
  const int64_t total = (int64_t)a.width * a.height;
  uint64_t s = 0;
  for (int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x; k < total; k += (int64_t)gridDim.x * TPB) {
    const int y = (int)(k / a.width), x = (int)(k % a.width);
    const int d = (int)P[(int64_t)y * a.pix_stride + x] - (int)R[(int64_t)y * a.ref_stride + x];
    s += (uint64_t)(d * d);
  }
  s = wave_sum64(s);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd(out + i, (unsigned long long)s);
}

__global__ void __launch_bounds__(TPB) k_disto_stats(const RedArgs a, wg_disto_stats* out) {
  const int64_t i = blockIdx.y;
  const uint8_t* P = a.pix + i * a.pix_pitch;
  const uint8_t* R = a.ref + i * a.ref_pitch;
  const int64_t total = (int64_t)a.width * a.height;
  uint32_t w = 0, xm = 0, ym = 0, xxm = 0, xym = 0, yym = 0;
  for (int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x; k < total; k += (int64_t)gridDim.x * TPB) {
    const int y = (int)(k / a.width), x = (int)(k % a.width);
    const uint32_t px = P[(int64_t)y * a.pix_stride + x], ry = R[(int64_t)y * a.ref_stride + x];
    w++;  // DistoStats.Accumulate (ssim.go:19-27)
    xm += px;
    ym += ry;
    xxm += px * px;
    xym += px * ry;
    yym += ry * ry;
  }
  w = wave_sum32(w), xm = wave_sum32(xm), ym = wave_sum32(ym);
  xxm = wave_sum32(xxm), xym = wave_sum32(xym), yym = wave_sum32(yym);
  if ((threadIdx.x & 63) == 0 && w) {
    unsigned* o = reinterpret_cast<unsigned*>(out + i);
    atomicAdd(o + 0, w);
    atomicAdd(o + 1, xm);
    atomicAdd(o + 2, ym);
    atomicAdd(o + 3, xxm);
    atomicAdd(o + 4, xym);
    atomicAdd(o + 5, yym);
  }
}

__global__ void __launch_bounds__(TPB) k_ssim_from_stats(const wg_disto_stats* st, int clipped, double* out, int n) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const wg_disto_stats s = st[i];
  const SsimStats ss = {s.w, s.xm, s.ym, s.xxm, s.xym, s.yym};
  // SSIMFromStatsClipped: N = W; SSIMFromStats: 0 for W == 0, else N = kWeightSum
  out[i] = clipped ? ssim_calc(ss, s.w) : (s.w == 0 ? 0.0 : ssim_calc(ss, 16 * 16));
}

// ---- PSNRFromSSE: Go's math.Log10 restated (src/math/log10.go, log.go) ----
// Log10(x) = log2(x) * (Ln2 / Ln10), log2 by Frexp + Log, Log the FreeBSD
// e_log.c polynomial; no multiply-add is fused (Go on amd64 does not fuse
// either), so the doubles are Go's.
__device__ double go_log(double x) {
#pragma clang fp contract(off)
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

__global__ void __launch_bounds__(TPB) k_psnr_from_sse(const unsigned long long* sse, const int64_t* count, double* out,
                                                       int n) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const uint64_t e = sse[i];
  const int64_t c = count[i];
  if (e == 0 || c == 0) {
    out[i] = 99.0;  // ssim.go:164-166
    return;
  }
  const double mse = (double)e / (double)c;
  const double x = 255.0 * 255.0 / mse;
  int ex;
  const double frac = frexp(x, &ex);
  const double l2 = frac == 0.5 ? (double)(ex - 1) : go_log(frac) * 0x1.71547652b82fep+0 + (double)ex;
  out[i] = 10.0 * (l2 * 0x1.34413509f79ffp-2);  // Ln2 / Ln10, correctly rounded
}

unsigned grid_x(int64_t work, int cap) {
  const int64_t b = (work + TPB - 1) / TPB;
  return (unsigned)(b < 1 ? 1 : (b > cap ? cap : b));
}

}  // namespace

extern "C" {

int wg_upsample_line_pairs(int32_t format, const uint8_t* top_y, const uint8_t* bot_y, int64_t y_step,
                           const uint8_t* top_u, const uint8_t* top_v, const uint8_t* bot_u, const uint8_t* bot_v,
                           int64_t uv_step, uint8_t* top_dst, uint8_t* bot_dst, int64_t dst_step,
                           const uint8_t* alpha_top, const uint8_t* alpha_bot, int64_t alpha_step, int32_t width,
                           int32_t n, void* stream) {
  WG_REQUIRE(format == 0 || format == 1);
  WG_REQUIRE(top_y && top_u && top_v && bot_u && bot_v && top_dst && (!bot_y || bot_dst));
  WG_REQUIRE(width >= 0 && n >= 0 && n <= 65535);
  WG_REQUIRE(format == 1 || (!alpha_top && !alpha_bot));
  if (format == 1)
    WG_REQUIRE(((reinterpret_cast<uintptr_t>(top_dst) | reinterpret_cast<uintptr_t>(bot_dst) | (uintptr_t)dst_step) &
                3) == 0);
  if (width == 0 || n == 0) return WG_OK;
  LpArgs a = {top_y, bot_y, top_u, top_v, bot_u, bot_v, alpha_top, alpha_bot, top_dst, bot_dst,
              y_step, uv_step, dst_step, alpha_step, width, format};
  hipLaunchKernelGGL(k_line_pairs, dim3(blocks_for(width, TPB), (unsigned)n), dim3(TPB), 0, as_stream(stream), a);
  return check_launch("k_line_pairs");
}

int wg_point_sample_rows(const uint8_t* y, const uint8_t* u, const uint8_t* v, int64_t y_step, int64_t uv_step,
                         uint8_t* dst, int64_t dst_step, int32_t width, int32_t n, void* stream) {
  WG_REQUIRE(y && u && v && dst && width >= 0 && n >= 0 && n <= 65535);
  if (width == 0 || n == 0) return WG_OK;
  const int wide = ((reinterpret_cast<uintptr_t>(dst) | (uintptr_t)dst_step) & 1) == 0;
  hipLaunchKernelGGL(k_point_sample, dim3(blocks_for((width + 1) >> 1, TPB), (unsigned)n), dim3(TPB), 0,
                     as_stream(stream), y, u, v, y_step, uv_step, dst, dst_step, width, wide);
  return check_launch("k_point_sample");
}

int wg_convert_argb_to_y(const uint32_t* argb, int64_t argb_pitch, uint8_t* y, int64_t y_pitch, int32_t width,
                         int32_t n, void* stream) {
  WG_REQUIRE(argb && y && width >= 0 && n >= 0 && n <= 65535);
  if (width == 0 || n == 0) return WG_OK;
  hipLaunchKernelGGL(k_argb_to_y, dim3(blocks_for(width, TPB), (unsigned)n), dim3(TPB), 0, as_stream(stream), argb,
                     argb_pitch, y, y_pitch, width);
  return check_launch("k_argb_to_y");
}

int wg_convert_argb_to_uv(const uint32_t* argb, int64_t argb_pitch, uint8_t* u, uint8_t* v, int64_t uv_pitch,
                          int32_t src_width, int32_t do_store, int32_t n, void* stream) {
  WG_REQUIRE(argb && u && v && src_width >= 0 && n >= 0 && n <= 65535);
  if (src_width == 0 || n == 0) return WG_OK;
  hipLaunchKernelGGL(k_argb_to_uv, dim3(blocks_for((src_width + 1) >> 1, TPB), (unsigned)n), dim3(TPB), 0,
                     as_stream(stream), argb, argb_pitch, u, v, uv_pitch, src_width, do_store ? 1 : 0);
  return check_launch("k_argb_to_uv");
}

int wg_accumulate_rgba(const uint8_t* r, const uint8_t* g, const uint8_t* b, const uint8_t* a, int32_t stride,
                       int64_t in_pitch, uint16_t* dst, int64_t dst_pitch, int32_t width, int32_t n, void* stream) {
  WG_REQUIRE(r && g && b && a && dst && width >= 0 && n >= 0 && n <= 65535);
  if (width == 0 || n == 0) return WG_OK;
  AccArgs p;
  p.r = r, p.g = g, p.b = b, p.a = a, p.dst = dst;
  p.in_pitch = in_pitch, p.dst_pitch = dst_pitch, p.stride = stride, p.width = width;
  p.tabs = host_tabs();
  hipLaunchKernelGGL(k_accumulate_rgba, dim3(blocks_for((width + 1) >> 1, TPB), (unsigned)n), dim3(TPB), 0,
                     as_stream(stream), p);
  return check_launch("k_accumulate_rgba");
}

int wg_convert_rgba32_to_uv(const uint16_t* rgb, int64_t rgb_pitch, uint8_t* u, uint8_t* v, int64_t uv_pitch,
                            int32_t width, int32_t n, void* stream) {
  WG_REQUIRE(rgb && u && v && width >= 0 && n >= 0 && n <= 65535);
  if (width == 0 || n == 0) return WG_OK;
  hipLaunchKernelGGL(k_rgba32_to_uv, dim3(blocks_for(width, TPB), (unsigned)n), dim3(TPB), 0, as_stream(stream), rgb,
                     rgb_pitch, u, v, uv_pitch, width);
  return check_launch("k_rgba32_to_uv");
}

int wg_convert_rgba32_to_uv_dithered(const uint16_t* rgb, int64_t rgb_pitch, uint8_t* u, uint8_t* v, int64_t uv_pitch,
                                     int32_t width, wg_random* state, int32_t n, void* stream) {
  WG_REQUIRE(rgb && u && v && state && width >= 0 && n >= 0);
  if (width == 0 || n == 0) return WG_OK;
  hipLaunchKernelGGL(k_rgba32_to_uv_dithered, dim3(blocks_for(n, DITHER_T)), dim3(DITHER_T), 0, as_stream(stream),
                     rgb, rgb_pitch, u, v, uv_pitch, width, state, n);
  return check_launch("k_rgba32_to_uv_dithered");
}

void wg_random_init_host(wg_random* rg, float dithering) {  // InitRandom, random.go:39-52
  static const uint32_t kTable[55] = {
      0x0de15230, 0x03b31886, 0x775faccb, 0x1c88626a, 0x68385c55, 0x14b3b828, 0x4a85fef8, 0x49ddb84b,
      0x64fcf397, 0x5c550289, 0x4a290000, 0x0d7ec1da, 0x5940b7ab, 0x5492577d, 0x4e19ca72, 0x38d38c69,
      0x0c01ee65, 0x32a1755f, 0x5437f652, 0x5abb2c32, 0x0faa57b1, 0x73f533e7, 0x685feeda, 0x7563cce2,
      0x6e990e83, 0x4730a7ed, 0x4fc0d9c6, 0x496b153c, 0x4f1403fa, 0x541afb0c, 0x73990b32, 0x26d7cb1c,
      0x6fcc3706, 0x2cbb77d8, 0x75762f2a, 0x6425ccdd, 0x24b35461, 0x0a7d8715, 0x220414a8, 0x141ebf67,
      0x56b41583, 0x73e502e3, 0x44cab16f, 0x28264d42, 0x73baaefb, 0x0a50ebed, 0x1d6ab6fb, 0x0d3ad40b,
      0x35db3b68, 0x2b081e83, 0x77ce6b95, 0x5181e5f0, 0x78853bbc, 0x009f9494, 0x27e5ed3c};
  if (!rg) return;
  for (int k = 0; k < 55; k++) rg->tab[k] = kTable[k];
  rg->index1 = 0;
  rg->index2 = 31;
  rg->amp = dithering < 0.0f ? 0 : (dithering > 1.0f ? 1 << 8 : (int32_t)((float)(1 << 8) * dithering));
}

int wg_sse_planes(const uint8_t* pix, const uint8_t* ref, int32_t width, int32_t height, int32_t pix_stride,
                  int32_t ref_stride, int64_t pix_pitch, int64_t ref_pitch, uint64_t* out, int32_t n, void* stream) {
  WG_REQUIRE(pix && ref && out && width >= 0 && height >= 0 && n >= 0 && n <= 65535);
  WG_REQUIRE(pix_stride >= width && ref_stride >= width);
  if (n == 0) return WG_OK;
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(out, 0, sizeof(uint64_t) * (size_t)n, s) != hipSuccess) return check_launch("hipMemsetAsync(sse)");
  if ((int64_t)width * height == 0) return WG_OK;
  RedArgs a = {pix, ref, pix_pitch, ref_pitch, pix_stride, ref_stride, width, height};
  hipLaunchKernelGGL(k_sse, dim3(grid_x((int64_t)width * height, 1024), (unsigned)n), dim3(TPB), 0, s, a,
                     reinterpret_cast<unsigned long long*>(out));
  return check_launch("k_sse");
}

int wg_psnr_from_sse(const uint64_t* sse, const int64_t* count, double* out, int32_t n, void* stream) {
  WG_REQUIRE(sse && count && out && n >= 0);
  if (n == 0) return WG_OK;
  hipLaunchKernelGGL(k_psnr_from_sse, dim3(blocks_for(n, TPB)), dim3(TPB), 0, as_stream(stream),
                     reinterpret_cast<const unsigned long long*>(sse), count, out, n);
  return check_launch("k_psnr_from_sse");
}

int wg_disto_stats_blocks(const uint8_t* pix, const uint8_t* ref, int32_t width, int32_t height, int32_t pix_stride,
                          int32_t ref_stride, int64_t pix_pitch, int64_t ref_pitch, wg_disto_stats* out, int32_t n,
                          void* stream) {
  WG_REQUIRE(pix && ref && out && width >= 0 && height >= 0 && n >= 0 && n <= 65535);
  WG_REQUIRE(pix_stride >= width && ref_stride >= width);
  if (n == 0) return WG_OK;
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(out, 0, sizeof(wg_disto_stats) * (size_t)n, s) != hipSuccess)
    return check_launch("hipMemsetAsync(disto)");
  if ((int64_t)width * height == 0) return WG_OK;
  RedArgs a = {pix, ref, pix_pitch, ref_pitch, pix_stride, ref_stride, width, height};
  hipLaunchKernelGGL(k_disto_stats, dim3(grid_x((int64_t)width * height, 1024), (unsigned)n), dim3(TPB), 0, s, a, out);
  return check_launch("k_disto_stats");
}

int wg_ssim_from_stats(const wg_disto_stats* stats, int32_t clipped, double* out, int32_t n, void* stream) {
  WG_REQUIRE(stats && out && n >= 0);
  if (n == 0) return WG_OK;
  hipLaunchKernelGGL(k_ssim_from_stats, dim3(blocks_for(n, TPB)), dim3(TPB), 0, as_stream(stream), stats,
                     clipped ? 1 : 0, out, n);
  return check_launch("k_ssim_from_stats");
}

}  // extern "C"
