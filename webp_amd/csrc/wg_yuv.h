// wg_yuv.h -- YUV <-> RGB arithmetic of internal/dsp/yuv.go shared by the
// import (k_import), upsample (k_upsample) and block-level (blockops_yuv.hip)
// kernels: the gamma tables (built on the host with float64 pow, as
// InitGammaTables), LinearToGamma, RGBToY / VP8ClipUV, and YUVToRGB.
#pragma once
#include <math.h>

#include <mutex>

#include "wg_dsp.h"

namespace wg {

struct GammaTabs {
  uint32_t to_lin[256];  // kGammaToLinearTab
  uint32_t to_gamma[34]; // kLinearToGammaTab
};

inline GammaTabs host_tabs() {  // InitGammaTables, yuv.go:193-215
  static GammaTabs t;
  static std::once_flag once;
  std::call_once(once, [] {
    for (int i = 0; i < 256; i++) {
      const double v = (double)i / 255.0;
      t.to_lin[i] = (uint32_t)((v <= 0 ? 0.0 : pow(v, 0.80)) * 4095.0 + 0.5);
    }
    const double scale = 128.0 / 4095.0;
    for (int i = 0; i <= 32; i++) {
      const double v = scale * (double)i;
      t.to_gamma[i] = (uint32_t)((v <= 0 ? 0.0 : pow(v, 1.0 / 0.80)) * 255.0 + 0.5);
    }
    t.to_gamma[33] = 255;
  });
  return t;
}

__device__ __forceinline__ int lin_to_gamma(const uint32_t* tg, uint32_t base, int shift) {  // yuv.go:236-249
  const int v = (int)base << shift;
  const int pos = min(v >> 9, 31);
  const int x = v & 511;
  const int y = (int)tg[pos + 1] * x + (int)tg[pos] * (512 - x);
  return (y + 64) >> 7;
}

__device__ __forceinline__ int rgb_to_y(int r, int g, int b) {  // yuv.go:151
  return (16839 * r + 33059 * g + 6420 * b + (1 << 15) + (16 << 16)) >> 16;
}
__device__ __forceinline__ int clip_uv(int uv, int rnd = 1 << 17) {  // VP8ClipUV :138 (rounding YUV_HALF<<2 by default)
  uv = (uv + rnd + (128 << 18)) >> 18;
  return (uv & ~0xff) == 0 ? uv : (uv < 0 ? 0 : 255);
}

// clip to [0, 16383] then >> 6 (v < 0 -> 0, v > 16383 -> 255): one v_med3
__device__ __forceinline__ int yuv_clip(int v) { return min(max(v, 0), 16383) >> 6; }

// MultHi (yuv.go:38) of a byte and a 16-bit constant on the full-rate 24-bit
// multiplier.  Written as asm: hipcc turned both "*" and __umul24 into the
// quarter-rate v_mul_lo_u32 once it lost the operands' range.
template <uint32_t K>
__device__ __forceinline__ int mult_hi(int x) {
  uint32_t r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(x), "v"(K));
  return (int)(r >> 8);
}

// YUVToRGB (yuv.go:71-109)
__device__ __forceinline__ uint32_t yuv_to_rgba(int y, int u, int v, int a) {
  const int yy = mult_hi<19077>(y);
  const int r = yuv_clip(yy + mult_hi<26149>(v) - 14234);
  const int g = yuv_clip(yy - mult_hi<6419>(u) - mult_hi<13320>(v) + 8708);
  const int b = yuv_clip(yy + mult_hi<33050>(u) - 17685);
  return pack4(r, g, b, a);
}

}  // namespace wg
