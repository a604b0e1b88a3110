// import.hip -- RGBA -> padded YUV420 planes for the VP8 encoder on gfx950
// (replaces VP8Encoder.importImage, internal/lossy/encode.go:671-943, the
// direct-pixel paths with and without dithering; arithmetic of
// internal/dsp/yuv.go, VP8Random of internal/dsp/random.go).
//
// Dithering (Preprocessing bit 1, encode.go:690-695, :793-809, :903-940):
// the reference draws one VP8Random value per padded pixel for Y in raster
// order, then two per chroma pixel (U, V) row pair by row pair, from a
// generator seeded identically for every image.  The stream therefore
// depends only on the padded frame size: wg_dither_plan runs the generator
// once on the host and leaves the draws in device memory (Y as int16, U/V as
// int32, 4 B per pixel), and the import kernel reads each pixel's draw next
// to its RGBA -- a per-size noise table instead of a serial generator.
//
// Streaming kernel: one thread per 2 rows x 4 columns of the padded frame
// (two 2x2 chroma quads), walking 8 row pairs.  Reads 2x16 B of RGBA, writes
// 2x4 B of Y and 2 B each of U and V per row pair.  Gamma tables (yuv.go:193-215) are built on the host with
// float64 pow, passed in the kernel argument block and staged in LDS.
// Padding replicates the last column / row exactly as the reference's clamp.
#include <math.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "wg_common.h"
#include "wg_dsp.h"
#include "wg_yuv.h"

namespace {
using namespace wg;

// One 2x2 quad: gamma-correct (alpha-weighted when 0 < sum(A) < 1020) average
// of R, G, B, then RGBToU / RGBToV on the sum-of-4 values.  Returns u | v << 8.
__device__ __forceinline__ uint32_t quad_uv(const uint32_t* tl, const uint32_t* tg, uint32_t p0, uint32_t p1,
                                         uint32_t p2, uint32_t p3, int has_alpha, int rnd_u = 1 << 17,
                                         int rnd_v = 1 << 17) {
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
  int u = clip_uv(-9719 * c3[0] - 19081 * c3[1] + 28800 * c3[2], rnd_u);
  int v = clip_uv(28800 * c3[0] - 24116 * c3[1] - 4684 * c3[2], rnd_v);
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
  int amp;       // VP8Random amplitude (dithered variant)
  const int16_t* dither_y;   // [padh][padw] RandomBits(16) draws before scaling
  const int32_t* dither_uv;  // [padh/2][padw] RandomBits(18) draws, U and V interleaved
  GammaTabs tabs;
};

constexpr int IM_T = 256;   // threads per block: 256 chunks = 1024 columns of a row pair
constexpr int IM_RP = 8;    // minimum row pairs walked per block (amortises the table fill)

// Thread = one 4-pixel chunk of a row pair (two 2x2 chroma quads).  Lane i of
// a wave loads bytes [16i, 16i + 16) of each of the two RGBA rows, so every
// load instruction is one contiguous 1 KB span, and stores 4 B of Y per row
// and 2 B each of U and V (contiguous 256 B / 128 B per wave instruction).
// RandomBits2's scaling of a draw (random.go:68-70): (d * amp) >> 8 + half
__device__ __forceinline__ int dither_round(int d, int amp, int half) { return ((d * amp) >> 8) + half; }

template <bool DITHER>
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
    // Y (encode.go:757-793; dithered: RGBToYRounding with RandomBits(16), :793-809)
    int dy[2][4] = {{1 << 15, 1 << 15, 1 << 15, 1 << 15}, {1 << 15, 1 << 15, 1 << 15, 1 << 15}};
    int duv[4] = {1 << 17, 1 << 17, 1 << 17, 1 << 17};
    if (DITHER) {
#pragma unroll
      for (int r = 0; r < 2; r++) {
        const uint2 q = *reinterpret_cast<const uint2*>(a.dither_y + (int64_t)(2 * yp + r) * a.padw + x0);
        dy[r][0] = dither_round((int16_t)(q.x & 0xffff), a.amp, 1 << 15);
        dy[r][1] = dither_round((int16_t)(q.x >> 16), a.amp, 1 << 15);
        dy[r][2] = dither_round((int16_t)(q.y & 0xffff), a.amp, 1 << 15);
        dy[r][3] = dither_round((int16_t)(q.y >> 16), a.amp, 1 << 15);
      }
      const int4 q = *reinterpret_cast<const int4*>(a.dither_uv + (int64_t)yp * a.padw + x0);
      duv[0] = dither_round(q.x, a.amp, 1 << 17);
      duv[1] = dither_round(q.y, a.amp, 1 << 17);
      duv[2] = dither_round(q.z, a.amp, 1 << 17);
      duv[3] = dither_round(q.w, a.amp, 1 << 17);
    }
#pragma unroll
    for (int r = 0; r < 2; r++) {
      uint32_t yw = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t p = px[r][i];
        const int yv = DITHER ? (16839 * (int)(p & 0xff) + 33059 * (int)((p >> 8) & 0xff) + 6420 * (int)((p >> 16) & 0xff) +
                                 dy[r][i] + (16 << 16)) >> 16
                              : rgb_to_y(p & 0xff, (p >> 8) & 0xff, (p >> 16) & 0xff);
        yw |= (uint32_t)(yv & 0xff) << (8 * i);
      }
      *reinterpret_cast<uint32_t*>(a.y + img * a.y_pitch + (int64_t)(2 * yp + r) * a.padw + x0) = yw;
    }
    // U/V: AccumulateRGBA (yuv.go:486-517) + ConvertRGBA32ToUV (:553-562) or
    // ConvertRGBA32ToUVDithered (:568-576)
    const uint32_t uv0 = quad_uv(tl, tg, px[0][0], px[0][1], px[1][0], px[1][1], a.has_alpha, duv[0], duv[1]);
    const uint32_t uv1 = quad_uv(tl, tg, px[0][2], px[0][3], px[1][2], px[1][3], a.has_alpha, duv[2], duv[3]);
    const int64_t co = img * a.uv_pitch + (int64_t)yp * (a.padw >> 1) + (x0 >> 1);
    *reinterpret_cast<uint16_t*>(a.u + co) = (uint16_t)((uv0 & 0xff) | ((uv1 & 0xff) << 8));
    *reinterpret_cast<uint16_t*>(a.v + co) = (uint16_t)((uv0 >> 8) | (uv1 & 0xff00));
  }
}

}  // namespace

namespace {
int launch_import(const uint8_t* rgba, int32_t w, int32_t h, int32_t stride, int64_t rgba_pitch, int32_t has_alpha,
                  uint8_t* y, uint8_t* u, uint8_t* v, int64_t y_pitch, int64_t uv_pitch, int32_t n_images, int amp,
                  const void* plan, void* stream) {
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
  a.amp = amp;
  a.dither_y = static_cast<const int16_t*>(plan);
  a.dither_uv = plan ? reinterpret_cast<const int32_t*>(static_cast<const int16_t*>(plan) + (int64_t)a.padw * a.padh)
                     : nullptr;
  const dim3 grid(wg::blocks_for(a.chunks, IM_T), wg::blocks_for(a.pairs, a.rp));
  if (plan)
    hipLaunchKernelGGL(k_import<true>, grid, dim3(IM_T), 0, wg::as_stream(stream), a);
  else
    hipLaunchKernelGGL(k_import<false>, grid, dim3(IM_T), 0, wg::as_stream(stream), a);
  return wg::check_launch("k_import");
}
}  // namespace

extern "C" int wg_import_rgba(const uint8_t* rgba, int32_t w, int32_t h, int32_t stride, int64_t rgba_pitch,
                              int32_t has_alpha, uint8_t* y, uint8_t* u, uint8_t* v, int64_t y_pitch,
                              int64_t uv_pitch, int32_t n_images, void* stream) {
  return launch_import(rgba, w, h, stride, rgba_pitch, has_alpha, y, u, v, y_pitch, uv_pitch, n_images, 0, nullptr,
                       stream);
}

// webp.Encode's dithering strength (encode.go (root):517-521, float32) and
// InitRandom's amplitude (random.go:39-49).
extern "C" int32_t wg_dither_amp(float quality, int32_t preprocessing) {
  if (!(preprocessing & 2)) return 0;
  const float x = quality / 100.0f;
  const float x2 = x * x;
  const float dithering = 1.0f + (0.5f - 1.0f) * x2 * x2;
  if (dithering < 0.0f) return 0;
  if (dithering > 1.0f) return 1 << 8;
  return (int32_t)((float)(1 << 8) * dithering);
}

extern "C" size_t wg_dither_plan_bytes(int32_t w, int32_t h) {
  if (w <= 0 || h <= 0) return 0;
  const size_t padw = 16 * (size_t)((w + 15) >> 4), padh = 16 * (size_t)((h + 15) >> 4);
  return padw * padh * 2 + padw * (padh / 2) * 4;
}

// The VP8Random stream of one image (InitRandom + RandomBits2 before the
// amplitude, random.go:24-72) in the order importImage draws it.
extern "C" int wg_dither_plan_host(int32_t w, int32_t h, void* plan_host) {
  WG_REQUIRE(plan_host && w > 0 && h > 0);
  const int64_t padw = 16 * (int64_t)((w + 15) >> 4), padh = 16 * (int64_t)((h + 15) >> 4);
  static const uint32_t kTab[55] = {
      0x0de15230, 0x03b31886, 0x775faccb, 0x1c88626a, 0x68385c55, 0x14b3b828, 0x4a85fef8, 0x49ddb84b, 0x64fcf397,
      0x5c550289, 0x4a290000, 0x0d7ec1da, 0x5940b7ab, 0x5492577d, 0x4e19ca72, 0x38d38c69, 0x0c01ee65, 0x32a1755f,
      0x5437f652, 0x5abb2c32, 0x0faa57b1, 0x73f533e7, 0x685feeda, 0x7563cce2, 0x6e990e83, 0x4730a7ed, 0x4fc0d9c6,
      0x496b153c, 0x4f1403fa, 0x541afb0c, 0x73990b32, 0x26d7cb1c, 0x6fcc3706, 0x2cbb77d8, 0x75762f2a, 0x6425ccdd,
      0x24b35461, 0x0a7d8715, 0x220414a8, 0x141ebf67, 0x56b41583, 0x73e502e3, 0x44cab16f, 0x28264d42, 0x73baaefb,
      0x0a50ebed, 0x1d6ab6fb, 0x0d3ad40b, 0x35db3b68, 0x2b081e83, 0x77ce6b95, 0x5181e5f0, 0x78853bbc, 0x009f9494,
      0x27e5ed3c};  // kRandomTable, random.go:24-35
  uint32_t tab[55];
  memcpy(tab, kTab, sizeof(tab));
  int i1 = 0, i2 = 31;
  auto next = [&]() -> uint32_t {  // the raw 31-bit draw, RandomBits2 :55-66
    int64_t d = (int64_t)tab[i1] - (int64_t)tab[i2];
    if (d < 0) d += (int64_t)1 << 31;
    tab[i1] = (uint32_t)d;
    if (++i1 == 55) i1 = 0;
    if (++i2 == 55) i2 = 0;
    return (uint32_t)d;
  };
  int16_t* py = static_cast<int16_t*>(plan_host);
  for (int64_t k = 0; k < padw * padh; k++) py[k] = (int16_t)((int32_t)(next() << 1) >> 16);
  int32_t* puv = reinterpret_cast<int32_t*>(py + padw * padh);
  for (int64_t k = 0; k < padw * (padh / 2); k++) puv[k] = (int32_t)(next() << 1) >> 14;
  return WG_OK;
}

extern "C" int wg_dither_plan(int32_t w, int32_t h, void* plan, void* stream) {
  WG_REQUIRE(plan && w > 0 && h > 0 && (reinterpret_cast<uintptr_t>(plan) & 15) == 0);
  const size_t bytes = wg_dither_plan_bytes(w, h);
  std::vector<uint8_t> host(bytes);
  const int rc = wg_dither_plan_host(w, h, host.data());
  if (rc) return rc;
  hipStream_t s = wg::as_stream(stream);
  if (hipMemcpyAsync(plan, host.data(), bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return wg::check_launch("wg_dither_plan copy");
  return WG_OK;
}

extern "C" int wg_import_rgba_dithered(const uint8_t* rgba, int32_t w, int32_t h, int32_t stride, int64_t rgba_pitch,
                                       int32_t has_alpha, int32_t amp, const void* plan, uint8_t* y, uint8_t* u,
                                       uint8_t* v, int64_t y_pitch, int64_t uv_pitch, int32_t n_images,
                                       void* stream) {
  WG_REQUIRE(plan && (reinterpret_cast<uintptr_t>(plan) & 15) == 0 && amp >= 0 && amp <= 256);
  return launch_import(rgba, w, h, stride, rgba_pitch, has_alpha, y, u, v, y_pitch, uv_pitch, n_images, amp, plan,
                       stream);
}
