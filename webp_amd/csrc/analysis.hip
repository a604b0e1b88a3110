// analysis.hip -- encoder pre-analysis (per-macroblock complexity alpha) on
// gfx950: replaces computeAlphas / computeMBAlphaDCTWith /
// computeMBUVAlphaDCTWith (internal/lossy/encode_analysis.go:245-700).
//
// Four lanes per macroblock, lane = one row of 4x4 blocks (sixteen MBs per
// wave): each lane predicts, transforms and bins its four luma blocks for
// both modes and two of the eight chroma blocks.  The |coeff|>>3 histograms
// live in LDS as private per-lane columns; GetAlpha's max count and last
// non-empty bin are reductions over the MB's 4 lanes.  DC/TM predictions are
// built from the SOURCE plane with the analysis' own border rules
// (generateI16Prediction :455-552).  (One lane per MB left the chip
// latency-bound on 8k waves; sixteen lanes per MB spent twice the VALU on
// reductions and idle chroma lanes.)
#include "wg_common.h"
#include "wg_dsp.h"

namespace {
using namespace wg;

constexpr int TPB = 256;
constexpr int LPM = 4;  // lanes per macroblock
constexpr int MBS_PER_BLOCK = TPB / LPM;

struct AnArgs {
  const uint8_t *y, *u, *v;
  int64_t y_pitch, uv_pitch;
  int w, h, mbw, mbh;
  int total;  // macroblocks in the batch
  int32_t *alphas, *lum, *uva, *uv_sum;
};

// sum / max over the 4 lanes of this lane's macroblock
__device__ __forceinline__ int sum4(int v) {
  v += __shfl_xor(v, 1, 4);
  return v + __shfl_xor(v, 2, 4);
}
__device__ __forceinline__ int max4(int v) {
  v = max(v, __shfl_xor(v, 1, 4));
  return max(v, __shfl_xor(v, 2, 4));
}

// Histograms: every lane owns a private column of 16 words in LDS, word k
// holding bins 2k and 2k+1 as 16-bit counts ([word][thread] layout, so the
// lane's ds_add never meets another lane's bank).  A shared per-MB histogram
// serialised on same-bin atomics (smooth content puts most coefficients in
// bin 0).
__device__ __forceinline__ void histo_add(uint32_t* col, const int16_t c[16]) {
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int v = min(abs((int)c[k]) >> 3, 31);
    atomicAdd(&col[(v >> 1) * TPB], 1u << (16 * (v & 1)));
  }
}
// GetAlpha (collectHistogramAlphaWith :584-600) over the MB's 4 columns:
// lane l sums words 4l..4l+3 (bins 8l..8l+7) over the MB's columns, read in a
// lane-rotated order (conflict-free), then clears its own column.  Every lane
// of the MB returns the alpha.
__device__ __forceinline__ int histo_alpha(uint32_t (*bins)[TPB], int slot, int l) {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  uint32_t sum[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < LPM; j++) {
    const int c = LPM * slot + ((j + l) & 3);
#pragma unroll
    for (int k = 0; k < 4; k++) sum[k] += bins[4 * l + k][c];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < 16; k++) bins[k][LPM * slot + l] = 0;
  int maxv = 0, last = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int lo = (int)(sum[k] & 0xffff), hi = (int)(sum[k] >> 16);
    maxv = max(maxv, max(lo, hi));
    last = lo > 0 ? 8 * l + 2 * k : last;
    last = hi > 0 ? 8 * l + 2 * k + 1 : last;
  }
  maxv = max4(maxv);
  last = max4(last);
  const int alpha = maxv > 1 ? 2 * 255 * last / maxv : 0;
  return min(alpha, 255);
}

// 4 bytes of a source row at x, clamped to the image width
__device__ __forceinline__ uint32_t row4(const uint8_t* row, int x, int w, bool full) {
  if (full) return *reinterpret_cast<const uint32_t*>(row + x);
  uint32_t v = 0;
#pragma unroll
  for (int c = 0; c < 4; c++) v |= (uint32_t)row[min(x + c, w - 1)] << (8 * c);
  return v;
}

__global__ __launch_bounds__(TPB) void k_analysis(const AnArgs a) {
  __shared__ uint32_t bins[16][TPB];
  __shared__ int s_uva[MBS_PER_BLOCK], s_img[MBS_PER_BLOCK];
  const int l = threadIdx.x & (LPM - 1), slot = threadIdx.x / LPM;
  uint32_t* col = &bins[0][threadIdx.x];
#pragma unroll
  for (int k = 0; k < 16; k++) col[k * TPB] = 0;
  const int m_raw = blockIdx.x * MBS_PER_BLOCK + slot;
  const bool valid = m_raw < a.total;
  const int m = valid ? m_raw : a.total - 1;
  const int mbs = a.mbw * a.mbh;
  const int img = m / mbs, idx = m - img * mbs;
  const int mby = idx / a.mbw, mbx = idx - mby * a.mbw;
  const int ys = 16 * a.mbw, uvs = 8 * a.mbw;
  const uint8_t* Y = a.y + img * a.y_pitch;
  const uint8_t* U = a.u + img * a.uv_pitch;
  const uint8_t* V = a.v + img * a.uv_pitch;
  const int x0 = 16 * mbx, y0 = 16 * mby;
  __builtin_amdgcn_wave_barrier();

  // ---- luma (generateI16Prediction :455-552 + collectHistogramAlphaWith :559-600);
  //      source rows / columns are clamped to the real image like the reference.
  //      Lane l: block row by = l, rows y0 + 4l .. + 3 ----
  const bool full_w = x0 + 16 <= a.w;
  const uint8_t* top_row = Y + (int64_t)(y0 - 1) * ys;  // valid only when mby > 0
  uint32_t px[4][4];  // [row][bx]
  int left4[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint8_t* row = Y + (int64_t)min(y0 + 4 * l + r, a.h - 1) * ys;
    if (full_w) {
      const uint4 q = *reinterpret_cast<const uint4*>(row + x0);
      px[r][0] = q.x; px[r][1] = q.y; px[r][2] = q.z; px[r][3] = q.w;
    } else {
#pragma unroll
      for (int bx = 0; bx < 4; bx++) px[r][bx] = row4(row, x0 + 4 * bx, a.w, false);
    }
    left4[r] = mbx > 0 ? row[x0 - 1] : 0;
  }
  int dc = 128;
  {
    int s = 0;
    if (mby > 0) {
      const uint32_t t4 = row4(top_row, x0 + 4 * l, a.w, full_w);
      s += (int)byte_of(t4, 0) + (int)byte_of(t4, 1) + (int)byte_of(t4, 2) + (int)byte_of(t4, 3);
    }
    if (mbx > 0) s += left4[0] + left4[1] + left4[2] + left4[3];
    const int sum = sum4(s);
    const int count = (mby > 0 ? 16 : 0) + (mbx > 0 ? 16 : 0);
    if (count > 0) dc = (sum + count / 2) / count;
  }
#pragma unroll
  for (int bx = 0; bx < 4; bx++) {
    int d[16];
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int c = 0; c < 4; c++) d[4 * r + c] = (int)byte_of(px[r][bx], c) - dc;
    int16_t co[16];
    fdct4x4(d, co);
    histo_add(col, co);
  }
  int best = histo_alpha(bins, slot, l);
  if (mbx > 0 && mby > 0) {  // TM (uniform over the MB's lanes)
    const int tl = top_row[x0 - 1];
#pragma unroll
    for (int bx = 0; bx < 4; bx++) {
      const uint32_t top4 = row4(top_row, x0 + 4 * bx, a.w, full_w);
      int d[16];
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int c = 0; c < 4; c++)
          d[4 * r + c] = (int)byte_of(px[r][bx], c) - clip8((int)byte_of(top4, c) + left4[r] - tl);
      int16_t co[16];
      fdct4x4(d, co);
      histo_add(col, co);
    }
    best = min(best, histo_alpha(bins, slot, l));
  }
  const int lum = min(best, 255);

  // ---- chroma (computeMBUVAlphaDCTWith :613-728), planes are MB-padded;
  //      lane l: plane l >> 1, block row l & 1, both block columns ----
  const int ux0 = 8 * mbx, uy0 = 8 * mby;
  int dcu = 128, dcv = 128;
  {
    int su = 0, sv = 0;
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int k = 2 * l + i;
      if (mby > 0) {
        su += U[(int64_t)(uy0 - 1) * uvs + ux0 + k];
        sv += V[(int64_t)(uy0 - 1) * uvs + ux0 + k];
      }
      if (mbx > 0) {
        su += U[(int64_t)(uy0 + k) * uvs + ux0 - 1];
        sv += V[(int64_t)(uy0 + k) * uvs + ux0 - 1];
      }
    }
    su = sum4(su);
    sv = sum4(sv);
    const int count = (mby > 0 ? 8 : 0) + (mbx > 0 ? 8 : 0);
    if (count > 0) {
      dcu = (su + count / 2) / count;
      dcv = (sv + count / 2) / count;
    }
  }
  {
    const uint8_t* P = (l >> 1) ? V : U;
    const int dcp = (l >> 1) ? dcv : dcu;
    const int cby = l & 1;
#pragma unroll
    for (int cbx = 0; cbx < 2; cbx++) {
      int d[16];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const uint32_t q = *reinterpret_cast<const uint32_t*>(P + (int64_t)(uy0 + 4 * cby + r) * uvs + ux0 + 4 * cbx);
#pragma unroll
        for (int c = 0; c < 4; c++) d[4 * r + c] = (int)byte_of(q, c) - dcp;
      }
      int16_t co[16];
      fdct4x4(d, co);
      histo_add(col, co);
    }
  }
  const int uva = histo_alpha(bins, slot, l);

  int mixed = 255 - ((3 * lum + uva + 2) >> 2);
  mixed = min(max(mixed, 0), 255);
  if (valid && l == 0) {
    a.alphas[m] = mixed;
    if (a.lum) a.lum[m] = lum;
    if (a.uva) a.uva[m] = uva;
  }
  if (a.uv_sum) {
    // one atomic per run of same-image MBs in the block (a per-MB atomic
    // serialised ~8k updates on each image's counter)
    if (l == 0) {
      s_uva[slot] = valid ? uva : 0;
      s_img[slot] = img;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int cur = s_img[0], acc = 0;
      for (int i = 0; i < MBS_PER_BLOCK; i++) {
        if (s_img[i] != cur) {
          atomicAdd(&a.uv_sum[cur], acc);
          cur = s_img[i];
          acc = 0;
        }
        acc += s_uva[i];
      }
      atomicAdd(&a.uv_sum[cur], acc);
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
  WG_REQUIRE((int64_t)n_images * a.mbw * a.mbh < (1ll << 31) - MBS_PER_BLOCK);
  a.total = n_images * a.mbw * a.mbh;
  hipLaunchKernelGGL(k_analysis, dim3(wg::blocks_for(a.total, MBS_PER_BLOCK)), dim3(TPB), 0, s, a);
  return wg::check_launch("k_analysis");
}
