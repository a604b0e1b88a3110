// import.hip -- RGBA -> padded YUV420 planes for the VP8 encoder on gfx950
// (replaces VP8Encoder.importImage, internal/lossy/encode.go:671-943,
// non-dithered direct-pixel path; arithmetic of internal/dsp/yuv.go).
//
// Streaming kernel: one thread per 2 rows x 4 columns of the padded frame
// (two 2x2 chroma quads), walking 8 row pairs.  Reads 2x16 B of RGBA, writes
// 2x4 B of Y and 2 B each of U and V per row pair.  Gamma tables (yuv.go:193-215) are built on the host with
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
  int w, h, stride, has_alpha, padw, padh;
  int chunks;    // padw / 4: 4-pixel chunks per row
  int pairs;     // n_images * padh / 2 row pairs in the batch
  int rp;        // row pairs walked per block (>= IM_RP; grid.y stays <= 65535)
  int aligned;   // rows start 16-byte aligned -> one 16 B load per row and chunk
  GammaTabs tabs;
};

constexpr int IM_T = 256;   // threads per block: 256 chunks = 1024 columns of a row pair
constexpr int IM_RP = 8;    // minimum row pairs walked per block (amortises the table fill)

// Thread = one 4-pixel chunk of a row pair (two 2x2 chroma quads).  Lane i of
// a wave loads bytes [16i, 16i + 16) of each of the two RGBA rows, so every
// load instruction is one contiguous 1 KB span, and stores 4 B of Y per row
// and 2 B each of U and V (contiguous 256 B / 128 B per wave instruction).
__global__ __launch_bounds__(IM_T) void k_import(const ImportArgs a) {
  __shared__ uint32_t tl[256];
  __shared__ uint32_t tg[34];
  for (int i = threadIdx.x; i < 256; i += IM_T) tl[i] = a.tabs.to_lin[i];
  if (threadIdx.x < 34) tg[threadIdx.x] = a.tabs.to_gamma[threadIdx.x];
  __syncthreads();
  const int cx = blockIdx.x * IM_T + threadIdx.x;
  if (cx >= a.chunks) return;
  const int x0 = 4 * cx;
  const bool fast = a.aligned && x0 + 4 <= a.w;
  const int hp = a.padh >> 1;
  const int pair_end = min((int)(blockIdx.y + 1) * a.rp, a.pairs);
  for (int pr = blockIdx.y * a.rp; pr < pair_end; pr++) {
    const int img = pr / hp, yp = pr - img * hp;
    const uint8_t* src = a.rgba + img * a.rgba_pitch;
    uint32_t px[2][4];
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const uint8_t* row = src + (int64_t)min(2 * yp + r, a.h - 1) * a.stride;
      if (fast) {
        const uint4 q = *reinterpret_cast<const uint4*>(row + 4 * x0);
        px[r][0] = q.x; px[r][1] = q.y; px[r][2] = q.z; px[r][3] = q.w;
      } else {
#pragma unroll
        for (int i = 0; i < 4; i++) px[r][i] = *reinterpret_cast<const uint32_t*>(row + 4 * min(x0 + i, a.w - 1));
      }
    }
    // Y (encode.go:757-793)
#pragma unroll
    for (int r = 0; r < 2; r++) {
      uint32_t yw = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t p = px[r][i];
        yw |= (uint32_t)rgb_to_y(p & 0xff, (p >> 8) & 0xff, (p >> 16) & 0xff) << (8 * i);
      }
      *reinterpret_cast<uint32_t*>(a.y + img * a.y_pitch + (int64_t)(2 * yp + r) * a.padw + x0) = yw;
    }
    // U/V: AccumulateRGBA (yuv.go:486-517) + ConvertRGBA32ToUV (:553-562)
    const uint32_t uv0 = quad_uv(tl, tg, px[0][0], px[0][1], px[1][0], px[1][1], a.has_alpha);
    const uint32_t uv1 = quad_uv(tl, tg, px[0][2], px[0][3], px[1][2], px[1][3], a.has_alpha);
    const int64_t co = img * a.uv_pitch + (int64_t)yp * (a.padw >> 1) + (x0 >> 1);
    *reinterpret_cast<uint16_t*>(a.u + co) = (uint16_t)((uv0 & 0xff) | ((uv1 & 0xff) << 8));
    *reinterpret_cast<uint16_t*>(a.v + co) = (uint16_t)((uv0 >> 8) | (uv1 & 0xff00));
  }
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
  a.chunks = a.padw / 4;
  WG_REQUIRE((int64_t)n_images * (a.padh / 2) < (1ll << 31) / 2);
  a.pairs = n_images * (a.padh / 2);
  a.tabs = host_tabs();
  a.aligned = ((reinterpret_cast<uintptr_t>(rgba) | (uintptr_t)stride | (uintptr_t)rgba_pitch) & 15) == 0;
  a.rp = max(IM_RP, (int)wg::blocks_for(a.pairs, 65535));
  const dim3 grid(wg::blocks_for(a.chunks, IM_T), wg::blocks_for(a.pairs, a.rp));
  hipLaunchKernelGGL(k_import, grid, dim3(IM_T), 0, wg::as_stream(stream), a);
  return wg::check_launch("k_import");
}
