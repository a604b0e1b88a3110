// import.hip -- RGBA -> padded YUV420 planes for the VP8 encoder on gfx950
// (replaces VP8Encoder.importImage, internal/lossy/encode.go:671-943,
// non-dithered direct-pixel path; arithmetic of internal/dsp/yuv.go).
//
// Streaming kernel: one thread per 2 rows x 8 columns of the padded frame
// (four 2x2 chroma quads).  Reads 2x32 B of RGBA, writes 2x8 B of Y and 4 B
// each of U and V.  Gamma tables (yuv.go:193-215) are built on the host with
// float64 pow, passed in the kernel argument block and staged in LDS.
// Padding replicates the last column / row exactly as the reference's clamp.
#include <math.h>
#include <mutex>

#include "wg_common.h"
#include "wg_dsp.h"

namespace {
using namespace wg;

struct GammaTabs {
  uint32_t to_lin[256];  // kGammaToLinearTab
  uint32_t to_gamma[34]; // kLinearToGammaTab
};

GammaTabs host_tabs() {  // InitGammaTables, yuv.go:193-215
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
__device__ __forceinline__ int clip_uv(int uv) {  // VP8ClipUV :138 with rounding YUV_HALF<<2
  uv = (uv + (1 << 17) + (128 << 18)) >> 18;
  return (uv & ~0xff) == 0 ? uv : (uv < 0 ? 0 : 255);
}

// One 2x2 quad: gamma-correct (alpha-weighted when 0 < sum(A) < 1020) average
// of R, G, B, then RGBToU / RGBToV on the sum-of-4 values.  Returns u | v << 8.
__device__ __forceinline__ uint32_t quad_uv(const uint32_t* tl, const uint32_t* tg, uint32_t p0, uint32_t p1,
                                         uint32_t p2, uint32_t p3, int has_alpha) {
  const uint32_t a0 = has_alpha ? p0 >> 24 : 255u, a1 = has_alpha ? p1 >> 24 : 255u;
  const uint32_t a2 = has_alpha ? p2 >> 24 : 255u, a3 = has_alpha ? p3 >> 24 : 255u;
  const uint32_t ta = a0 + a1 + a2 + a3;
  const bool plain = (ta == 4 * 255) || (ta == 0);
  const uint32_t inv = plain ? 0u : (1u << 19) / ta;  // kInvAlpha[ta], yuv.go:343-447
  int c3[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const int sh = 8 * c;
    const uint32_t l0 = tl[(p0 >> sh) & 0xff], l1 = tl[(p1 >> sh) & 0xff];
    const uint32_t l2 = tl[(p2 >> sh) & 0xff], l3 = tl[(p3 >> sh) & 0xff];
    const uint32_t sum = plain ? l0 + l1 + l2 + l3 : ((a0 * l0 + a1 * l1 + a2 * l2 + a3 * l3) * inv) >> 17;
    c3[c] = lin_to_gamma(tg, sum, 0);
  }
  int u = clip_uv(-9719 * c3[0] - 19081 * c3[1] + 28800 * c3[2]);
  int v = clip_uv(28800 * c3[0] - 24116 * c3[1] - 4684 * c3[2]);
  // Keep the two clamps separate: hipcc (ROCm 7.2) otherwise fuses
  // "sat_u8(x>>18) | sat_u8(y>>18)<<8" into v_ashr_pk_u8_i32 and then assumes
  // the upper 16 bits of that result are zero, which the hardware does not
  // guarantee -- V picked up stray bits.  (Found by the parity tests.)
  asm volatile("" : "+v"(u));
  asm volatile("" : "+v"(v));
  return (uint32_t)u | ((uint32_t)v << 8);
}

struct ImportArgs {
  const uint8_t* rgba;
  uint8_t *y, *u, *v;
  int64_t rgba_pitch, y_pitch, uv_pitch;
  int w, h, stride, has_alpha, padw, padh, groups;  // groups = padw / 8
  int aligned;  // rows start 16-byte aligned -> 2 x 16 B loads per row
  GammaTabs tabs;
};

__global__ __launch_bounds__(256) void k_import(const ImportArgs a, int64_t total) {
  __shared__ uint32_t tl[256];
  __shared__ uint32_t tg[34];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) tl[i] = a.tabs.to_lin[i];
  if (threadIdx.x < 34) tg[threadIdx.x] = a.tabs.to_gamma[threadIdx.x];
  __syncthreads();
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int g = tid % a.groups;
  const int64_t rest = tid / a.groups;
  const int yp = rest % (a.padh / 2);
  const int img = (int)(rest / (a.padh / 2));
  const int x0 = 8 * g;
  const uint8_t* src = a.rgba + img * a.rgba_pitch;

  // gather 2 rows x 8 pixels (clamped to the real image)
  uint32_t px[2][8];
  const bool fast = a.aligned && x0 + 8 <= a.w;  // same path for both rows
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int sy = min(2 * yp + r, a.h - 1);
    const uint8_t* row = src + (int64_t)sy * a.stride;
    if (fast) {
      const uint4 q0 = *reinterpret_cast<const uint4*>(row + 4 * x0);
      const uint4 q1 = *reinterpret_cast<const uint4*>(row + 4 * x0 + 16);
      px[r][0] = q0.x; px[r][1] = q0.y; px[r][2] = q0.z; px[r][3] = q0.w;
      px[r][4] = q1.x; px[r][5] = q1.y; px[r][6] = q1.z; px[r][7] = q1.w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; i++) px[r][i] = *reinterpret_cast<const uint32_t*>(row + 4 * min(x0 + i, a.w - 1));
    }
  }
  // Y (encode.go:757-793)
#pragma unroll
  for (int r = 0; r < 2; r++) {
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t p = px[r][i];
      const uint32_t yv = (uint32_t)rgb_to_y(p & 0xff, (p >> 8) & 0xff, (p >> 16) & 0xff);
      if (i < 4) lo |= yv << (8 * i);
      else hi |= yv << (8 * (i - 4));
    }
    *reinterpret_cast<uint2*>(a.y + img * a.y_pitch + (int64_t)(2 * yp + r) * a.padw + x0) = make_uint2(lo, hi);
  }
  // U/V: AccumulateRGBA (yuv.go:486-517) + ConvertRGBA32ToUV (:553-562)
  const uint32_t uv0 = quad_uv(tl, tg, px[0][0], px[0][1], px[1][0], px[1][1], a.has_alpha);
  const uint32_t uv1 = quad_uv(tl, tg, px[0][2], px[0][3], px[1][2], px[1][3], a.has_alpha);
  const uint32_t uv2 = quad_uv(tl, tg, px[0][4], px[0][5], px[1][4], px[1][5], a.has_alpha);
  const uint32_t uv3 = quad_uv(tl, tg, px[0][6], px[0][7], px[1][6], px[1][7], a.has_alpha);
  const uint32_t uo = (uv0 & 0xff) | ((uv1 & 0xff) << 8) | ((uv2 & 0xff) << 16) | ((uv3 & 0xff) << 24);
  const uint32_t vo = (uv0 >> 8) | ((uv1 >> 8) << 8) | ((uv2 >> 8) << 16) | ((uv3 >> 8) << 24);
  const int64_t co = img * a.uv_pitch + (int64_t)yp * (a.padw / 2) + x0 / 2;
  *reinterpret_cast<uint32_t*>(a.u + co) = uo;
  *reinterpret_cast<uint32_t*>(a.v + co) = vo;
}

}  // namespace

extern "C" int wg_import_rgba(const uint8_t* rgba, int32_t w, int32_t h, int32_t stride, int64_t rgba_pitch,
                              int32_t has_alpha, uint8_t* y, uint8_t* u, uint8_t* v, int64_t y_pitch,
                              int64_t uv_pitch, int32_t n_images, void* stream) {
  WG_REQUIRE(rgba && y && u && v);
  WG_REQUIRE(w > 0 && h > 0 && n_images > 0 && stride >= 4 * w && (stride & 3) == 0);
  WG_REQUIRE((reinterpret_cast<uintptr_t>(rgba) & 3) == 0 && (rgba_pitch & 3) == 0);
  const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4;
  WG_REQUIRE(((reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(v)) &
              3) == 0 && (y_pitch & 7) == 0 && (uv_pitch & 3) == 0);
  WG_REQUIRE(y_pitch >= (int64_t)256 * mbw * mbh && uv_pitch >= (int64_t)64 * mbw * mbh);
  ImportArgs a;
  a.rgba = rgba;
  a.y = y;
  a.u = u;
  a.v = v;
  a.rgba_pitch = rgba_pitch;
  a.y_pitch = y_pitch;
  a.uv_pitch = uv_pitch;
  a.w = w;
  a.h = h;
  a.stride = stride;
  a.has_alpha = has_alpha ? 1 : 0;
  a.padw = 16 * mbw;
  a.padh = 16 * mbh;
  a.groups = a.padw / 8;
  a.tabs = host_tabs();
  a.aligned = ((reinterpret_cast<uintptr_t>(rgba) | (uintptr_t)stride | (uintptr_t)rgba_pitch) & 15) == 0;
  const int64_t total = (int64_t)n_images * (a.padh / 2) * a.groups;
  hipLaunchKernelGGL(k_import, dim3(wg::blocks_for(total, 256)), dim3(256), 0, wg::as_stream(stream), a, total);
  return wg::check_launch("k_import");
}
