// upsample.hip -- "fancy" 4:2:0 -> 4:4:4 chroma upsampling + YUV->RGB to
// NRGBA on gfx950: replaces buildNRGBA (webp.go:379-450) and the line-pair
// kernel it drives, UpsampleLinePairNRGBA (upsample.go:130-236,
// upsample_direct_amd64.go:10-134).
//
// The reference walks overlapping line pairs; every output pixel is a pure
// function of one luma sample and a 2x2 chroma neighbourhood, so here each
// thread produces 8 consecutive pixels of one output row.  Which two chroma
// rows a luma row reads, and whether it takes the "top" or "bottom" half of
// the diamond kernel, follows buildNRGBA's row schedule exactly:
//   row 0 -> chroma (0, 0), top;  odd r -> ((r-1)/2, (r+1)/2 or (r-1)/2 on the
//   last row of an even-height image), top;  even r>0 -> (r/2-1, r/2), bottom.
// u and v are computed per channel (the packed-uint32 LOAD_UV trick of
// upsample.go:14-16 never carries between the halves).
#include "wg_common.h"
#include "wg_dsp.h"

namespace {
using namespace wg;

__device__ __forceinline__ int yuv_clip(int v) { return v < 0 ? 0 : (v > 16383 ? 255 : (v >> 6)); }

// YUVToRGB (yuv.go:71-109)
__device__ __forceinline__ uint32_t yuv_to_rgba(int y, int u, int v, int a) {
  const int yy = (y * 19077) >> 8;
  const int r = yuv_clip(yy + ((v * 26149) >> 8) - 14234);
  const int g = yuv_clip(yy - ((u * 6419) >> 8) - ((v * 13320) >> 8) + 8708);
  const int b = yuv_clip(yy + ((u * 33050) >> 8) - 17685);
  return pack4(r, g, b, a);
}

// Interpolated chroma sample for pixel x = x0 + i (upsample.go:140-230).
// t[] / b[] hold chroma columns x0/2-1 .. x0/2+4 of the two chroma rows, so
// with i a compile-time constant every index below is static.
template <int I>
__device__ __forceinline__ int up_chroma(const int* t, const int* b, int x0, int w, bool top) {
  constexpr int K = ((I + 1) >> 1) + 1;  // window index of pair k = (x+1)/2
  const int x = x0 + I;
  if (x == 0) return top ? (3 * t[1] + b[1] + 2) >> 2 : (3 * b[1] + t[1] + 2) >> 2;
  if ((I & 1) && x == w - 1 && (w & 1) == 0)  // trailing pixel of an even width: vertical only
    return top ? (3 * t[K - 1] + b[K - 1] + 2) >> 2 : (3 * b[K - 1] + t[K - 1] + 2) >> 2;
  const int tl = t[K - 1], tt = t[K], l = b[K - 1], cur = b[K];
  const int avg = tl + tt + l + cur + 8;
  const int diag12 = (avg + 2 * (tt + l)) >> 3;
  const int diag03 = (avg + 2 * (tl + cur)) >> 3;
  if (I & 1) return top ? (diag12 + tl) >> 1 : (diag03 + l) >> 1;
  return top ? (diag03 + tt) >> 1 : (diag12 + cur) >> 1;
}

template <int I>
__device__ __forceinline__ uint32_t up_pixel(const int* tu, const int* bu, const int* tv, const int* bv, int x0, int w,
                                             bool top, const uint8_t* yrow, const uint8_t* arow) {
  const int x = min(x0 + I, w - 1);
  return yuv_to_rgba(yrow[x], up_chroma<I>(tu, bu, x0, w, top), up_chroma<I>(tv, bv, x0, w, top),
                     arow ? arow[x] : 255);
}

struct UpArgs {
  const uint8_t *y, *u, *v, *alpha;
  uint8_t* out;
  int64_t y_pitch, uv_pitch, a_pitch, out_pitch;
  int y_stride, uv_stride, w, h, groups;  // groups = ceil(w / 8)
};

__global__ __launch_bounds__(256) void k_upsample(const UpArgs a, int64_t total) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int g = tid % a.groups;
  const int64_t rest = tid / a.groups;
  const int r = rest % a.h;
  const int img = (int)(rest / a.h);
  const int w = a.w, h = a.h;

  int ct, cb;
  bool top;
  if (r == 0) { ct = cb = 0; top = true; }
  else if (r & 1) { ct = (r - 1) >> 1; cb = (r == h - 1) ? ct : ct + 1; top = true; }
  else { ct = (r >> 1) - 1; cb = r >> 1; top = false; }

  const int x0 = 8 * g;
  const int cw = (w + 1) >> 1;
  const int kbase = (x0 >> 1) - 1;  // chroma columns kbase .. kbase+5 cover pixels x0..x0+7
  const uint8_t* U = a.u + img * a.uv_pitch;
  const uint8_t* V = a.v + img * a.uv_pitch;
  int tu[6], bu[6], tv[6], bv[6];
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const int c = min(max(kbase + k, 0), cw - 1);
    tu[k] = U[(int64_t)ct * a.uv_stride + c];
    bu[k] = U[(int64_t)cb * a.uv_stride + c];
    tv[k] = V[(int64_t)ct * a.uv_stride + c];
    bv[k] = V[(int64_t)cb * a.uv_stride + c];
  }
  const uint8_t* yrow = a.y + img * a.y_pitch + (int64_t)r * a.y_stride;
  const uint8_t* arow = a.alpha ? a.alpha + img * a.a_pitch + (int64_t)r * w : nullptr;
  uint8_t* orow = a.out + img * a.out_pitch + (int64_t)r * 4 * w;
  uint32_t px[8];
  px[0] = up_pixel<0>(tu, bu, tv, bv, x0, w, top, yrow, arow);
  px[1] = up_pixel<1>(tu, bu, tv, bv, x0, w, top, yrow, arow);
  px[2] = up_pixel<2>(tu, bu, tv, bv, x0, w, top, yrow, arow);
  px[3] = up_pixel<3>(tu, bu, tv, bv, x0, w, top, yrow, arow);
  px[4] = up_pixel<4>(tu, bu, tv, bv, x0, w, top, yrow, arow);
  px[5] = up_pixel<5>(tu, bu, tv, bv, x0, w, top, yrow, arow);
  px[6] = up_pixel<6>(tu, bu, tv, bv, x0, w, top, yrow, arow);
  px[7] = up_pixel<7>(tu, bu, tv, bv, x0, w, top, yrow, arow);
  if (x0 + 8 <= w && ((reinterpret_cast<uintptr_t>(orow + 4 * x0) & 15) == 0)) {
    *reinterpret_cast<uint4*>(orow + 4 * x0) = make_uint4(px[0], px[1], px[2], px[3]);
    *reinterpret_cast<uint4*>(orow + 4 * x0 + 16) = make_uint4(px[4], px[5], px[6], px[7]);
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++)
      if (x0 + i < w) *reinterpret_cast<uint32_t*>(orow + 4 * (x0 + i)) = px[i];
  }
}

}  // namespace

extern "C" int wg_upsample_nrgba(const uint8_t* y, int32_t y_stride, int64_t y_pitch, const uint8_t* u,
                                 const uint8_t* v, int32_t uv_stride, int64_t uv_pitch, const uint8_t* alpha,
                                 int64_t a_pitch, int32_t w, int32_t h, uint8_t* out, int64_t out_pitch,
                                 int32_t n_images, void* stream) {
  WG_REQUIRE(y && u && v && out && w > 0 && h > 0 && n_images > 0);
  WG_REQUIRE(y_stride >= w && uv_stride >= (w + 1) / 2 && out_pitch >= (int64_t)4 * w * h);
  WG_REQUIRE((reinterpret_cast<uintptr_t>(out) & 3) == 0 && (out_pitch & 3) == 0);
  UpArgs a;
  a.y = y;
  a.u = u;
  a.v = v;
  a.alpha = alpha;
  a.out = out;
  a.y_pitch = y_pitch;
  a.uv_pitch = uv_pitch;
  a.a_pitch = a_pitch;
  a.out_pitch = out_pitch;
  a.y_stride = y_stride;
  a.uv_stride = uv_stride;
  a.w = w;
  a.h = h;
  a.groups = (w + 7) / 8;
  const int64_t total = (int64_t)n_images * h * a.groups;
  hipLaunchKernelGGL(k_upsample, dim3(wg::blocks_for(total, 256)), dim3(256), 0, wg::as_stream(stream), a, total);
  return wg::check_launch("k_upsample");
}
