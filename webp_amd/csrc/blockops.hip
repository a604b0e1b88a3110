// blockops.hip -- the internal/dsp function variables as batched GPU entry
// points (the "block-level layer" of include/webpgpu.h).  Each kernel runs
// the same device functions (wg_dsp.h) that the frame kernels use, over n
// independent caller-owned instance buffers, so the parity tests exercise
// the production arithmetic one reference function at a time.
#include "wg_common.h"
#include "wg_dsp.h"

namespace {
using namespace wg;

constexpr int TPB = 256;

// ---- predictors: one thread per (instance, row, 4-pixel group) ----
__global__ void k_pred4(const uint8_t* modes, uint8_t* bufs, int64_t stride, const int32_t* offs, int off,
                        int n) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= 4LL * n) return;
  const int64_t i = tid >> 2;
  const int r = tid & 3;
  uint8_t* buf = bufs + i * stride;
  const int o = offs ? offs[i] : off;
  int X, T[8], L[4];
  pred4_ctx(buf, o, X, T, L);
  const uint32_t p = pred4_row(modes[i], r, X, T, L);
  uint8_t* d = buf + o + r * WG_BPS;
  d[0] = byte_of(p, 0); d[1] = byte_of(p, 1); d[2] = byte_of(p, 2); d[3] = byte_of(p, 3);
}

template <int SIZE>
__global__ void k_predsq(const uint8_t* modes, uint8_t* bufs, int64_t stride, const int32_t* offs, int off, int n) {
  constexpr int PER = SIZE * SIZE / 4;  // 4-pixel groups per block
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (int64_t)PER * n) return;
  const int64_t i = tid / PER;
  const int g = tid % PER, py = g / (SIZE / 4), px = 4 * (g % (SIZE / 4));
  uint8_t* d = bufs + i * stride + (offs ? offs[i] : off);
  const int mode = modes[i];
  const int dc = predsq_dc(mode, d, SIZE);
  const uint32_t p = predsq_row4(mode, d, px, py, dc);
  // all threads of this instance read the border first; the border is
  // outside the block so the writes below never race with those reads.
  uint8_t* o = d + py * WG_BPS + px;
  o[0] = byte_of(p, 0); o[1] = byte_of(p, 1); o[2] = byte_of(p, 2); o[3] = byte_of(p, 3);
}

// ---- decoder transforms: one thread per (instance, block, row) ----
__global__ void k_transform(int kind, const int16_t* coeffs, int64_t cpitch, uint8_t* dst, int64_t dstride, int n) {
  const int nblk = (kind == 1) ? 2 : (kind >= 4 ? 4 : 1);
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (int64_t)n * nblk * 4) return;
  const int64_t i = tid / (nblk * 4);
  const int k = (tid / 4) % nblk, r = tid & 3;
  const int16_t* in = coeffs + i * cpitch + 16 * k;
  // block placement: Transform doTwo -> +4; UV -> 0, 4, 4*BPS, 4*BPS+4
  const int boff = (kind >= 4) ? ((k & 1) * 4 + (k >> 1) * 4 * WG_BPS) : 4 * k;
  uint8_t* d = dst + i * dstride + boff + r * WG_BPS;
  int res[4];
  int code = 3;
  if (kind == 2) code = 2;
  else if (kind == 3) code = 1;
  else if (kind == 5) code = in[0] != 0 ? 1 : 0;  // transformDCUV :203-216
  dec_residual_row(in, code, r, res);
  for (int c = 0; c < 4; c++) d[c] = clip8(d[c] + res[c]);
}

__global__ void k_twht(const int16_t* in, int16_t* out, int n, int forward) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int v[16];
  for (int k = 0; k < 16; k++) v[k] = in[16 * i + k];
  int16_t o[16];
  if (forward) {
    fwht(v, o);
    for (int k = 0; k < 16; k++) out[16 * i + k] = o[k];
  } else {
    iwht(v, o);  // DC of block k goes to out[16*k] (transforms.go:245-250); other entries untouched
    for (int k = 0; k < 16; k++) out[256 * i + 16 * k] = o[k];
  }
}

// ---- encoder ITransform: dst = clip(ref + IDCT(in)), one thread per (instance, block, row)
__global__ void k_itransform(const uint8_t* ref, const int16_t* in, uint8_t* dst, int64_t bstride, int two, int n) {
  const int nblk = two ? 2 : 1;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (int64_t)n * nblk * 4) return;
  const int64_t i = tid / (nblk * 4);
  const int k = (tid / 4) % nblk, r = tid & 3;
  int res[4];
  dec_residual_row(in + 32 * i + 16 * k, 3, r, res);
  const uint8_t* s = ref + i * bstride + 4 * k + r * WG_BPS;
  uint8_t* d = dst + i * bstride + 4 * k + r * WG_BPS;
  int px[4];
  for (int c = 0; c < 4; c++) px[c] = s[c];
  for (int c = 0; c < 4; c++) d[c] = clip8(px[c] + res[c]);
}

__global__ void k_ftransform(const uint8_t* src, const uint8_t* ref, int64_t bstride, int16_t* out, int two, int n) {
  const int nblk = two ? 2 : 1;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (int64_t)n * nblk) return;
  const int64_t i = tid / nblk;
  const int k = tid % nblk;
  const uint8_t* s = src + i * bstride + 4 * k;
  const uint8_t* p = ref + i * bstride + 4 * k;
  int d[16];
  for (int y = 0; y < 4; y++)
    for (int x = 0; x < 4; x++) d[4 * y + x] = s[x + y * WG_BPS] - p[x + y * WG_BPS];
  int16_t o[16];
  fdct4x4(d, o);
  for (int c = 0; c < 16; c++) out[(16 * nblk) * i + 16 * k + c] = o[c];
}

__global__ void k_metric(int kind, const uint8_t* pix, const uint8_t* ref, int64_t bstride, int32_t* out, int n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* a = pix + i * bstride;
  const uint8_t* b = ref + i * bstride;
  int v = 0;
  if (kind == 0) v = sse_nxn(a, b, 4);
  else if (kind == 1) v = sse_nxn(a, b, 16);
  else if (kind == 2) v = tdisto4x4(a, b);
  else
    for (int y = 0; y < 16; y += 4)
      for (int x = 0; x < 16; x += 4) v += tdisto4x4(a + x + y * WG_BPS, b + x + y * WG_BPS);
  out[i] = v;
}

__global__ void k_ssim_get(const uint8_t* s1, const uint8_t* s2, int64_t bstride, int rs, const int32_t* xywh,
                           double* out, int n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* a = s1 + i * bstride;
  const uint8_t* b = s2 + i * bstride;
  const uint32_t kw[7] = {1, 2, 3, 4, 3, 2, 1};
  SsimStats s = {0, 0, 0, 0, 0, 0};
  int x0 = 0, x1 = 6, y0 = 0, y1 = 6, xo = 3, yo = 3;
  if (xywh) {  // SSIMGetClipped :132-160 (window centred on (xo, yo))
    xo = xywh[4 * i];
    yo = xywh[4 * i + 1];
    const int W = xywh[4 * i + 2], H = xywh[4 * i + 3];
    x0 = max(xo - 3, 0); x1 = min(xo + 3, W - 1);
    y0 = max(yo - 3, 0); y1 = min(yo + 3, H - 1);
  }
  for (int y = y0; y <= y1; y++)
    for (int x = x0; x <= x1; x++) {
      const uint32_t w = kw[3 + x - xo] * kw[3 + y - yo];
      const uint32_t p = a[x + y * rs], q = b[x + y * rs];
      s.w += w; s.xm += w * p; s.ym += w * q;
      s.xxm += w * p * p; s.xym += w * p * q; s.yym += w * q * q;
    }
  out[i] = xywh ? ssim_calc(s, s.w) : ssim_calc(s, 256);
}

// ---- loop filters: one thread per (instance, plane, sample along the edge) ----
__global__ void k_filter(int kind, uint8_t* p, int64_t bstride, int base, int stride, int uv_delta,
                         const int32_t* thr, const int32_t* ith, const int32_t* hev, int n) {
  const bool chroma = kind >= 8;
  const int len = chroma ? 8 : 16, planes = chroma ? 2 : 1;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (int64_t)n * planes * len) return;
  const int64_t i = tid / (planes * len);
  const int pl = (tid / len) % planes, s = tid % len;
  uint8_t* buf = p + i * bstride + (pl ? uv_delta : 0);
  const int t = thr[i];
  const int it = ith ? ith[i] : 0, h = hev ? hev[i] : 0;
  // V* filters cross a horizontal edge (step = stride, samples along x);
  // H* filters cross a vertical edge (step = 1, samples along y).
  const bool vert = (kind % 2) == 0;
  const int step = vert ? stride : 1, along = vert ? 1 : stride;
  switch (kind) {
    case 0: case 1:
      f_simple(buf, base + s * along, step, t);
      break;
    case 2: case 3:
      for (int k = 1; k <= 3; k++) f_simple(buf, base + 4 * k * step + s * along, step, t);
      break;
    case 4: case 5: case 8: case 9:
      f_complex(buf, base + s * along, step, t, it, h, false);
      break;
    case 6: case 7:
      for (int k = 1; k <= 3; k++) f_complex(buf, base + 4 * k * step + s * along, step, t, it, h, true);
      break;
    default:  // 10, 11: VFilter8i / HFilter8i
      f_complex(buf, base + 4 * step + s * along, step, t, it, h, true);
      break;
  }
}

}  // namespace

#define LAUNCH(kern, nthreads, ...)                                                                   \
  do {                                                                                                \
    if ((nthreads) > 0)                                                                               \
      hipLaunchKernelGGL(kern, dim3(wg::blocks_for((nthreads), TPB)), dim3(TPB), 0, wg::as_stream(stream), \
                         __VA_ARGS__);                                                                \
    return wg::check_launch(#kern);                                                                   \
  } while (0)

extern "C" {

int wg_pred_luma4(const uint8_t* modes, uint8_t* bufs, int64_t buf_stride, const int32_t* offs, int32_t off,
                  int32_t n, void* stream) {
  WG_REQUIRE(n >= 0 && (n == 0 || (modes && bufs)));
  LAUNCH(k_pred4, 4LL * n, modes, bufs, buf_stride, offs, off, n);
}
int wg_pred_luma16(const uint8_t* modes, uint8_t* bufs, int64_t buf_stride, const int32_t* offs, int32_t off,
                   int32_t n, void* stream) {
  WG_REQUIRE(n >= 0 && (n == 0 || (modes && bufs)));
  LAUNCH(k_predsq<16>, 64LL * n, modes, bufs, buf_stride, offs, off, n);
}
int wg_pred_chroma8(const uint8_t* modes, uint8_t* bufs, int64_t buf_stride, const int32_t* offs, int32_t off,
                    int32_t n, void* stream) {
  WG_REQUIRE(n >= 0 && (n == 0 || (modes && bufs)));
  LAUNCH(k_predsq<8>, 16LL * n, modes, bufs, buf_stride, offs, off, n);
}
int wg_transform(int32_t kind, const int16_t* coeffs, int64_t coeff_pitch, uint8_t* dst, int64_t dst_stride,
                 int32_t n, void* stream) {
  WG_REQUIRE(kind >= 0 && kind <= 5 && n >= 0 && (n == 0 || (coeffs && dst)));
  const int nblk = (kind == 1) ? 2 : (kind >= 4 ? 4 : 1);
  LAUNCH(k_transform, (int64_t)n * nblk * 4, kind, coeffs, coeff_pitch, dst, dst_stride, n);
}
int wg_transform_wht(const int16_t* in, int16_t* out, int32_t n, void* stream) {
  WG_REQUIRE(n >= 0 && (n == 0 || (in && out)));
  LAUNCH(k_twht, (int64_t)n, in, out, n, 0);
}
int wg_ftransform_wht(const int16_t* in, int16_t* out, int32_t n, void* stream) {
  WG_REQUIRE(n >= 0 && (n == 0 || (in && out)));
  LAUNCH(k_twht, (int64_t)n, in, out, n, 1);
}
int wg_itransform(const uint8_t* ref, const int16_t* in, uint8_t* dst, int64_t blk_stride, int32_t do_two,
                  int32_t n, void* stream) {
  WG_REQUIRE(n >= 0 && (n == 0 || (ref && in && dst)));
  LAUNCH(k_itransform, (int64_t)n * (do_two ? 2 : 1) * 4, ref, in, dst, blk_stride, do_two, n);
}
int wg_ftransform(const uint8_t* src, const uint8_t* ref, int64_t blk_stride, int16_t* out, int32_t two, int32_t n,
                  void* stream) {
  WG_REQUIRE(n >= 0 && (n == 0 || (src && ref && out)));
  LAUNCH(k_ftransform, (int64_t)n * (two ? 2 : 1), src, ref, blk_stride, out, two, n);
}
int wg_metric(int32_t kind, const uint8_t* pix, const uint8_t* ref, int64_t blk_stride, int32_t* out, int32_t n,
              void* stream) {
  WG_REQUIRE(kind >= 0 && kind <= 3 && n >= 0 && (n == 0 || (pix && ref && out)));
  LAUNCH(k_metric, (int64_t)n, kind, pix, ref, blk_stride, out, n);
}
int wg_ssim_get(const uint8_t* s1, const uint8_t* s2, int64_t buf_stride, int32_t row_stride, const int32_t* xywh,
                double* out, int32_t n, void* stream) {
  WG_REQUIRE(n >= 0 && (n == 0 || (s1 && s2 && out)));
  LAUNCH(k_ssim_get, (int64_t)n, s1, s2, buf_stride, row_stride, xywh, out, n);
}
int wg_filter(int32_t kind, uint8_t* p, int64_t buf_stride, int32_t base, int32_t stride, int32_t uv_delta,
              const int32_t* thresh, const int32_t* ithresh, const int32_t* hev, int32_t n, void* stream) {
  WG_REQUIRE(kind >= 0 && kind <= 11 && n >= 0 && (n == 0 || (p && thresh)));
  WG_REQUIRE(kind < 4 || n == 0 || (ithresh && hev));
  const int64_t per = kind >= 8 ? 16 : 16;  // 2 planes x 8 samples, or 16 samples
  LAUNCH(k_filter, (int64_t)n * per, kind, p, buf_stride, base, stride, uv_delta, thresh, ithresh, hev, n);
}

}  // extern "C"
