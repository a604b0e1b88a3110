// vp8l_host.cpp -- host side of the VP8L predictor transform: the fastSLog2
// table of the reference (internal/lossless/encode_histogram.go:355-368,
// fastSLog2LUT[i] = i * math.Log2(i)), built once per device and kept
// resident (512 KB).  math.Log2 is Go's standard library (src/math/log.go,
// log10.go: frexp reduction + the FreeBSD e_log.c polynomial), restated
// operation for operation; this file is compiled with -ffp-contract=off so
// no multiply-add is fused and the doubles equal Go's.
#include <hip/hip_runtime_api.h>
#include <math.h>

#include <mutex>
#include <vector>

#include "wg_common_host.h"

namespace {

double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01;
  const double L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01;
  const double L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01;
  const double L7 = 1.479819860511658591e-01;
  int ki;
  double f1 = frexp(x, &ki);
  if (f1 < 0.70710678118654752440) {  // Go: Sqrt2/2
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

double go_log2(double x) {
  int e;
  const double frac = frexp(x, &e);
  if (frac == 0.5) return (double)(e - 1);
  return go_log(frac) * 0x1.71547652b82fep+0 /* Go const 1/Ln2 */ + (double)e;
}

constexpr int kLut = 65536;
constexpr int kMaxDev = 64;
std::mutex g_mu;
double* g_lut[kMaxDev] = {nullptr};

}  // namespace

namespace wg {

const double* vp8l_slog2_lut_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) {
    set_error("vp8l: hipGetDevice failed");
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(g_mu);
  if (!g_lut[dev]) {
    std::vector<double> h(kLut);
    h[0] = 0;
    for (int i = 1; i < kLut; i++) h[i] = (double)i * go_log2((double)i);
    void* d = nullptr;
    if (hipMalloc(&d, kLut * sizeof(double)) != hipSuccess ||
        hipMemcpy(d, h.data(), kLut * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
      set_error("vp8l: cannot upload the slog2 table");
      if (d) (void)hipFree(d);
      return nullptr;
    }
    g_lut[dev] = static_cast<double*>(d);
  }
  return g_lut[dev];
}

}  // namespace wg

// Host copy of the table (tests compare it with the oracle's).
extern "C" int wg_vp8l_slog2_lut_host(double* out, int32_t n) {
  WG_REQUIRE(out && n > 0 && n <= kLut);
  out[0] = 0;
  for (int i = 1; i < n; i++) out[i] = (double)i * go_log2((double)i);
  return WG_OK;
}
