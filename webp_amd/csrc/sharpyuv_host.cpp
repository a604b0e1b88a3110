// sharpyuv_host.cpp -- the gamma tables of SharpYUV, built on the host once
// per (device, transfer function) and kept resident.
//
// sRGB (initGammaTables, sharpyuv/gamma.go:48-88): g2l[1026] (gamma -> 16-bit
// linear, 10-bit index) then l2g[514] (16-bit linear -> gamma, 9-bit index,
// interpolated by the kernels like fixedPointInterpolation), uint32.
//
// Every other transfer function of gamma.go:125-446 (BT.709/601/2020,
// BT.470M/BG, SMPTE 240, linear, log100, log100*sqrt10, IEC 61966, BT.1361,
// PQ, SMPTE 428, HLG): GammaToLinear over the 1024 10-bit codes in g2l, and
// LinearToGamma over every 16-bit linear value the conversion can produce
// (0 .. max(g2l)) as a direct uint16 table after the sRGB block.  The Go code
// works in float32 with float64 pow/log10/exp/log; so does this (a libm
// evaluation in long double gives the same tables, tests/test_sharpyuv.py).
#include <string.h>

#include <vector>
#include <hip/hip_runtime_api.h>
#include <math.h>

#include <algorithm>
#include <mutex>

#include "wg_common_host.h"

namespace {

constexpr int kG2L = 1026, kL2G = 514, kMaxDev = 64, kMaxTf = 19;
std::mutex g_mu;
void* g_tabs[kMaxDev][kMaxTf] = {{nullptr}};
int g_lut_n[kMaxDev][kMaxTf] = {{0}};

float powf_go(float b, float e) { return (float)pow((double)b, (double)e); }
float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
float roundf_go(float x) { return x < 0 ? (float)ceil((double)(x - 0.5f)) : (float)floor((double)(x + 0.5f)); }

// toLinear* (gamma.go:166-346); constant expressions written out as the
// exact decimal the Go constant folds to, rounded once to float32
float to_lin(float g, int tf) {
  const float k709 = (float)(1.0 / 0.45);
  switch (tf) {
    case 1: case 6: case 14: case 15:
      if (g < 0) return 0;
      if (g < 0.0812428582986315f) return g / 4.5f;
      if (g < 1) return powf_go((g + 0.09929682680944f) / 1.09929682680944f, k709);
      return 1;
    case 4: return powf_go(clampf(g, 0, 1), 2.2f);
    case 5: return powf_go(clampf(g, 0, 1), 2.8f);
    case 7:
      if (g < 0) return 0;
      if (g < 0.09128634211778f) return g / 4.0f;
      if (g < 1) return powf_go((g + 0.111572195921731f) / 1.111572195921731f, k709);
      return 1;
    case 9: return g <= 0 ? 0.005f : powf_go(10.0f, 2.0f * (std::min(g, 1.0f) - 1.0f));
    case 10: return g <= 0 ? 0.00158113883f : powf_go(10.0f, 2.5f * (std::min(g, 1.0f) - 1.0f));
    case 11:
      if (g <= -0.0812428582986315f) return powf_go((-g + 0.09929682680944f) / -1.09929682680944f, k709);
      if (g < 0.0812428582986315f) return g / 4.5f;
      return powf_go((g + 0.09929682680944f) / 1.09929682680944f, k709);
    case 12:
      if (g < -0.25f) return -0.25f;
      if (g < 0) return powf_go((g - 0.02482420670236f) / -0.27482420670236f, k709) / -4.0f;
      if (g < 0.0812428582986315f) return g / 4.5f;
      if (g < 1) return powf_go((g + 0.09929682680944f) / 1.09929682680944f, k709);
      return 1;
    case 16:
      if (g > 0) {
        const float pg = powf_go(g, (float)(32.0 / 2523.0));
        const float num = std::max(pg - 0.8359375f, 0.0f);
        const float den = std::max(18.8515625f - 18.6875f * pg, 1.401298464324817e-45f);
        return powf_go(num / den, (float)(4096.0 / 653.0));
      }
      return 0;
    case 17: return powf_go(std::max(g, 0.0f), 2.6f) / 0.91655527974030934f;
    case 18:
      if (g < 0) return 0;
      if (g <= 0.5f) return powf_go((g * g) * (float)(1.0 / 3.0), 1.2f);
      return powf_go(((float)exp((double)((g - 0.55991073f) / 0.17883277f)) + 0.28466892f) / 12.0f, 1.2f);
    default: return 0;
  }
}
// fromLinear* (gamma.go:178-356)
float from_lin(float l, int tf) {
  switch (tf) {
    case 1: case 6: case 14: case 15:
      if (l < 0) return 0;
      if (l < 0.018053968510807f) return l * 4.5f;
      if (l < 1) return 1.09929682680944f * powf_go(l, 0.45f) - 0.09929682680944f;
      return 1;
    case 4: return powf_go(clampf(l, 0, 1), (float)(1.0 / 2.2));
    case 5: return powf_go(clampf(l, 0, 1), (float)(1.0 / 2.8));
    case 7:
      if (l < 0) return 0;
      if (l < 0.022821585529445f) return l * 4.0f;
      if (l < 1) return 1.111572195921731f * powf_go(l, 0.45f) - 0.111572195921731f;
      return 1;
    case 9: return l < 0.01f ? 0 : 1.0f + (float)log10((double)std::min(l, 1.0f)) / 2.0f;
    case 10: return l < 0.00316227766f ? 0 : 1.0f + (float)log10((double)std::min(l, 1.0f)) / 2.5f;
    case 11:
      if (l <= -0.018053968510807f) return -1.09929682680944f * powf_go(-l, 0.45f) + 0.09929682680944f;
      if (l < 0.018053968510807f) return l * 4.5f;
      return 1.09929682680944f * powf_go(l, 0.45f) - 0.09929682680944f;
    case 12:
      if (l < -0.25f) return -0.25f;
      if (l < 0) return -0.27482420670236f * powf_go(-4.0f * l, 0.45f) + 0.02482420670236f;
      if (l < 0.018053968510807f) return l * 4.5f;
      if (l < 1) return 1.09929682680944f * powf_go(l, 0.45f) - 0.09929682680944f;
      return 1;
    case 16:
      if (l > 0) {
        const float pl = powf_go(l, (float)(653.0 / 4096.0));
        return powf_go((0.8359375f + 18.8515625f * pl) / (1.0f + 18.6875f * pl), (float)(2523.0 / 32.0));
      }
      return 0;
    case 17: return powf_go(0.91655527974030934f * std::max(l, 0.0f), (float)(1.0 / 2.6));
    case 18:
      l = powf_go(l, (float)(1.0 / 1.2));
      if (l < 0) return 0;
      if (l <= (float)(1.0 / 12.0)) return (float)sqrt((double)(3.0f * l));
      return 0.17883277f * (float)log((double)(12.0f * l - 0.28466892f)) + 0.55991073f;
    default: return 0;
  }
}

// GammaToLinear / LinearToGamma at bitDepth 10 (gamma.go:360-446), tf != sRGB
void build_tf(int tf, uint32_t* g2l, std::vector<uint16_t>& l2g) {
  uint32_t mx = 0;
  for (int v = 0; v < 1024; v++) {
    g2l[v] = tf == 8 ? (uint32_t)v : (uint32_t)(int64_t)roundf_go(to_lin((float)v / 1023.0f, tf) * 65535.0f);
    mx = std::max(mx, g2l[v]);
  }
  g2l[1024] = g2l[1025] = g2l[1023];
  l2g.resize(mx + 1);
  for (uint32_t v = 0; v <= mx; v++)
    l2g[v] = tf == 8 ? (uint16_t)v : (uint16_t)(int64_t)roundf_go(from_lin((float)v / 65535.0f, tf) * 1023.0f);
}

void build(uint32_t* g2l, uint32_t* l2g) {
  const double a = 0.09929682680944, thresh = 0.018053968510807;
  const double gamma_f = 1.0 / 0.45, final_scale = 65536.0;
  const double norm = 1.0 / 1024.0, a_rec = 1.0 / (1.0 + a);
  for (int v = 0; v <= 1024; v++) {
    const double g = norm * (double)v;
    const double value = g <= thresh * 4.5 ? g / 4.5 : pow(a_rec * (g + a), gamma_f);
    g2l[v] = (uint32_t)(value * final_scale + 0.5);
  }
  g2l[1025] = g2l[1024];
  const double scale = 1.0 / 512.0;
  for (int v = 0; v <= 512; v++) {
    const double g = scale * (double)v;
    const double value = g <= thresh ? 4.5 * g : (1.0 + a) * pow(g, 1.0 / gamma_f) - a;
    l2g[v] = (uint32_t)(final_scale * value + 0.5);
  }
  l2g[513] = l2g[512];
}

}  // namespace

namespace wg {

// Device tables for transfer function tf: g2l[1026] + l2g[514] (uint32) and,
// for tf != sRGB, the direct LinearToGamma table (uint16) right after them;
// *lut_n = its length (0 for sRGB).
const void* sharpyuv_tables_device(int tf, int* lut_n) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev || tf < 0 || tf >= kMaxTf) {
    set_error("sharpyuv: hipGetDevice failed or bad transfer function");
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(g_mu);
  if (!g_tabs[dev][tf]) {
    std::vector<uint32_t> h(kG2L + kL2G, 0u);
    std::vector<uint16_t> lut;
    if (tf == 13)
      build(h.data(), h.data() + kG2L);
    else
      build_tf(tf, h.data(), lut);
    const size_t bytes = sizeof(uint32_t) * h.size() + sizeof(uint16_t) * lut.size();
    void* d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess ||
        hipMemcpy(d, h.data(), sizeof(uint32_t) * h.size(), hipMemcpyHostToDevice) != hipSuccess ||
        (!lut.empty() && hipMemcpy(static_cast<uint8_t*>(d) + sizeof(uint32_t) * h.size(), lut.data(),
                                   sizeof(uint16_t) * lut.size(), hipMemcpyHostToDevice) != hipSuccess)) {
      set_error("sharpyuv: cannot upload the gamma tables");
      if (d) (void)hipFree(d);
      return nullptr;
    }
    g_tabs[dev][tf] = d;
    g_lut_n[dev][tf] = (int)lut.size();
  }
  *lut_n = g_lut_n[dev][tf];
  return g_tabs[dev][tf];
}

}  // namespace wg

extern "C" int wg_sharpyuv_tables_host(uint32_t* g2l, uint32_t* l2g) {
  WG_REQUIRE(g2l && l2g);
  build(g2l, l2g);
  return WG_OK;
}

/* GammaToLinear over the 10-bit codes (g2l[1024]) and the LinearToGamma
 * table the kernels use for transfer function tf (host; *n receives its
 * length; l2g may be NULL to query it). */
extern "C" int wg_sharpyuv_transfer_tables_host(int32_t tf, uint32_t* g2l, uint16_t* l2g, int32_t* n) {
  WG_REQUIRE(g2l && n && tf >= 0 && tf < kMaxTf && tf != 13);
  uint32_t h[kG2L];
  std::vector<uint16_t> lut;
  build_tf(tf, h, lut);
  memcpy(g2l, h, sizeof(uint32_t) * 1024);
  if (l2g) {
    WG_REQUIRE(*n >= (int32_t)lut.size());
    memcpy(l2g, lut.data(), sizeof(uint16_t) * lut.size());
  }
  *n = (int32_t)lut.size();
  return WG_OK;
}
