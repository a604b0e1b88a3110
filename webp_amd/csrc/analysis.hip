// analysis.hip -- encoder pre-analysis (per-macroblock complexity alpha) on
// gfx950: replaces computeAlphas / computeMBAlphaDCTWith /
// computeMBUVAlphaDCTWith (internal/lossy/encode_analysis.go:245-700).
//
// One thread per macroblock: adjacent threads own horizontally adjacent MBs,
// so each 16-byte row load of the Y plane is coalesced across the wave.  The
// |coeff|>>3 histograms (32 bins) live in LDS as [bin][thread] words so every
// ds_add hits a distinct bank.  DC/TM predictions are built from the SOURCE
// plane with the analysis' own border rules (generateI16Prediction :455-552).
#include "wg_common.h"
#include "wg_dsp.h"

namespace {
using namespace wg;

constexpr int TPB = 64;

struct AnArgs {
  const uint8_t *y, *u, *v;
  int64_t y_pitch, uv_pitch;
  int w, h, mbw, mbh;
  int32_t *alphas, *lum, *uva, *uv_sum;
};

__device__ __forceinline__ void histo_add(uint32_t* bins, const int16_t c[16]) {
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int v = min(abs((int)c[k]) >> 3, 31);
    atomicAdd(&bins[v * TPB], 1u);
  }
}
// GetAlpha (collectHistogramAlphaWith :584-600); clears the bins
__device__ __forceinline__ int histo_alpha(uint32_t* bins) {
  int maxv = 0, last = 1;
  for (int k = 0; k < 32; k++) {
    const int d = (int)bins[k * TPB];
    bins[k * TPB] = 0;
    if (d > 0) {
      maxv = max(maxv, d);
      last = k;
    }
  }
  const int alpha = maxv > 1 ? 2 * 255 * last / maxv : 0;
  return min(alpha, 255);
}

__global__ __launch_bounds__(TPB) void k_analysis(const AnArgs a, int64_t total) {
  __shared__ uint32_t bins_all[32 * TPB];
  uint32_t* bins = bins_all + threadIdx.x;
  for (int k = 0; k < 32; k++) bins[k * TPB] = 0;
  const int64_t tid_raw = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = tid_raw < total;  // no early exit: the uv_sum reduction below is wave-wide
  const int64_t tid = valid ? tid_raw : total - 1;
  const int mbs = a.mbw * a.mbh;
  const int img = (int)(tid / mbs);
  const int idx = (int)(tid % mbs);
  const int mbx = idx % a.mbw, mby = idx / a.mbw;
  const int ys = 16 * a.mbw, uvs = 8 * a.mbw;
  const uint8_t* Y = a.y + img * a.y_pitch;
  const uint8_t* U = a.u + img * a.uv_pitch;
  const uint8_t* V = a.v + img * a.uv_pitch;
  const int x0 = 16 * mbx, y0 = 16 * mby;

  // ---- luma (generateI16Prediction :455-552 + collectHistogramAlphaWith :559-600);
  //      source rows / columns are clamped to the real image like the reference ----
  const bool full_w = x0 + 16 <= a.w;
  const uint8_t* top_row = Y + (int64_t)(y0 - 1) * ys;  // valid only when mby > 0
  int best = 256;
  for (int mode = 0; mode < 2; mode++) {
    if (mode == 1 && (mbx == 0 || mby == 0)) continue;
    int dc = 128, tl = 128;
    if (mode == 0) {
      int sum = 0, count = 0;
      if (mby > 0) {
        for (int i = 0; i < 16; i++) sum += top_row[min(x0 + i, a.w - 1)];
        count += 16;
      }
      if (mbx > 0) {
        for (int j = 0; j < 16; j++) sum += Y[(int64_t)min(y0 + j, a.h - 1) * ys + x0 - 1];
        count += 16;
      }
      if (count > 0) dc = (sum + count / 2) / count;
    } else {
      tl = top_row[x0 - 1];
    }
    for (int by = 0; by < 4; by++) {
      int left4[4] = {128, 128, 128, 128};  // only read when mbx > 0 (TM mode)
      if (mode == 1)
#pragma unroll
        for (int r = 0; r < 4; r++) left4[r] = Y[(int64_t)min(y0 + 4 * by + r, a.h - 1) * ys + x0 - 1];
      for (int bx = 0; bx < 4; bx++) {
        uint32_t top4 = 0;
        if (mode == 1) {
          if (full_w) top4 = *reinterpret_cast<const uint32_t*>(top_row + x0 + 4 * bx);
          else
            for (int c = 0; c < 4; c++) top4 |= (uint32_t)top_row[min(x0 + 4 * bx + c, a.w - 1)] << (8 * c);
        }
        int d[16];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const uint8_t* row = Y + (int64_t)min(y0 + 4 * by + r, a.h - 1) * ys;
          uint32_t w4;
          if (full_w) {
            w4 = *reinterpret_cast<const uint32_t*>(row + x0 + 4 * bx);
          } else {
            w4 = 0;
            for (int c = 0; c < 4; c++) w4 |= (uint32_t)row[min(x0 + 4 * bx + c, a.w - 1)] << (8 * c);
          }
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const int pr = mode == 0 ? dc : clip8((int)byte_of(top4, c) + left4[r] - tl);
            d[4 * r + c] = (int)byte_of(w4, c) - pr;
          }
        }
        int16_t co[16];
        fdct4x4(d, co);
        histo_add(bins, co);
      }
    }
    best = min(best, histo_alpha(bins));
  }
  const int lum = min(best, 255);

  // ---- chroma (computeMBUVAlphaDCTWith :613-728), planes are MB-padded ----
  const int ux0 = 8 * mbx, uy0 = 8 * mby;
  int dcu = 128, dcv = 128;
  {
    int su = 0, sv = 0, count = 0;
    if (mby > 0)
      for (int i = 0; i < 8; i++) {
        su += U[(int64_t)(uy0 - 1) * uvs + ux0 + i];
        sv += V[(int64_t)(uy0 - 1) * uvs + ux0 + i];
        count++;
      }
    if (mbx > 0)
      for (int j = 0; j < 8; j++) {
        su += U[(int64_t)(uy0 + j) * uvs + ux0 - 1];
        sv += V[(int64_t)(uy0 + j) * uvs + ux0 - 1];
        count++;
      }
    if (count > 0) {
      dcu = (su + count / 2) / count;
      dcv = (sv + count / 2) / count;
    }
  }
  for (int by = 0; by < 2; by++)
    for (int bx = 0; bx < 2; bx++)
      for (int pl = 0; pl < 2; pl++) {
        const uint8_t* P = pl ? V : U;
        const int dcp = pl ? dcv : dcu;
        int d[16];
        for (int r = 0; r < 4; r++) {
          const uint32_t w4 = *reinterpret_cast<const uint32_t*>(P + (int64_t)(uy0 + 4 * by + r) * uvs + ux0 + 4 * bx);
          for (int c = 0; c < 4; c++) d[4 * r + c] = (int)byte_of(w4, c) - dcp;
        }
        int16_t co[16];
        fdct4x4(d, co);
        histo_add(bins, co);
      }
  const int uva = histo_alpha(bins);

  int mixed = 255 - ((3 * lum + uva + 2) >> 2);
  mixed = min(max(mixed, 0), 255);
  const int64_t o = (int64_t)img * mbs + idx;
  if (valid) {
    a.alphas[o] = mixed;
    if (a.lum) a.lum[o] = lum;
    if (a.uva) a.uva[o] = uva;
  }
  if (a.uv_sum) {
    // one atomic per (wave, image) instead of one per macroblock: the per-MB
    // form serialised ~8k atomics on each image's counter.
    const int img0 = __shfl(img, 0, 64);
    const bool uniform = __all(img == img0);
    if (uniform) {
      int s = valid ? uva : 0;
      for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
      if ((threadIdx.x & 63) == 0) atomicAdd(&a.uv_sum[img], s);
    } else if (valid) {
      atomicAdd(&a.uv_sum[img], uva);
    }
  }
}

}  // namespace

extern "C" int wg_analysis_alphas(const uint8_t* y, const uint8_t* u, const uint8_t* v, int32_t w, int32_t h,
                                  int64_t y_pitch, int64_t uv_pitch, int32_t n_images, int32_t* alphas,
                                  int32_t* lum, int32_t* uva, int32_t* uv_sum, void* stream) {
  WG_REQUIRE(y && u && v && alphas && w > 0 && h > 0 && n_images > 0);
  WG_REQUIRE((reinterpret_cast<uintptr_t>(y) & 15) == 0 && (y_pitch & 15) == 0);
  WG_REQUIRE(((reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(v)) & 3) == 0 && (uv_pitch & 3) == 0);
  AnArgs a;
  a.y = y;
  a.u = u;
  a.v = v;
  a.y_pitch = y_pitch;
  a.uv_pitch = uv_pitch;
  a.w = w;
  a.h = h;
  a.mbw = (w + 15) >> 4;
  a.mbh = (h + 15) >> 4;
  a.alphas = alphas;
  a.lum = lum;
  a.uva = uva;
  a.uv_sum = uv_sum;
  hipStream_t s = wg::as_stream(stream);
  if (uv_sum && hipMemsetAsync(uv_sum, 0, sizeof(int32_t) * n_images, s) != hipSuccess)
    return wg::check_launch("hipMemsetAsync(uv_sum)");
  const int64_t total = (int64_t)n_images * a.mbw * a.mbh;
  hipLaunchKernelGGL(k_analysis, dim3(wg::blocks_for(total, TPB)), dim3(TPB), 0, s, a, total);
  return wg::check_launch("k_analysis");
}
