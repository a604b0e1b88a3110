// sharpyuv_host.cpp -- the sRGB gamma tables of SharpYUV (initGammaTables,
// sharpyuv/gamma.go:48-88), built once per device and kept resident:
// g2l[1026] (gamma -> 16-bit linear, 10-bit index) then l2g[514]
// (16-bit linear -> gamma, 9-bit index), uint32.  The reference builds them
// with Go's math.Pow; libm pow here (the values are rounded to integers; the
// whole conversion is pinned against libsharpyuv in the tests).
#include <hip/hip_runtime_api.h>
#include <math.h>

#include <mutex>

#include "wg_common_host.h"

namespace {

constexpr int kG2L = 1026, kL2G = 514, kMaxDev = 64;
std::mutex g_mu;
void* g_tabs[kMaxDev] = {nullptr};

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

const void* sharpyuv_tables_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) {
    set_error("sharpyuv: hipGetDevice failed");
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(g_mu);
  if (!g_tabs[dev]) {
    uint32_t h[kG2L + kL2G];
    build(h, h + kG2L);
    void* d = nullptr;
    if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) {
      set_error("sharpyuv: cannot upload the gamma tables");
      if (d) (void)hipFree(d);
      return nullptr;
    }
    g_tabs[dev] = d;
  }
  return g_tabs[dev];
}

}  // namespace wg

extern "C" int wg_sharpyuv_tables_host(uint32_t* g2l, uint32_t* l2g) {
  WG_REQUIRE(g2l && l2g);
  build(g2l, l2g);
  return WG_OK;
}
