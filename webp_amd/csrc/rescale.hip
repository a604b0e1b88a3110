// rescale.hip -- the row rescaler of internal/dsp/rescale.go (SURVEY.md
// 8(f)#4) as one gather kernel per plane batch.
//
// The Go Rescaler (rescale.go:14-257) is a row state machine: ImportRow
// resamples one source row horizontally into FRow (and, when shrinking
// vertically, adds it to IRow); ExportRow emits a destination row from
// FRow/IRow whenever YAccum <= 0.  Every quantity that carries state between
// pixels or rows depends only on the sizes, never on pixel values, except the
// shrink carry `sum = multFix(frac, FXScale)`, which needs one source pixel.
// So the host walks the state machine once per size (the plan, O(sw + sh)):
//
//   xtab[dw]  shrink: first source pixel, in-range count, out-of-range count,
//                     -accum after the pixel, and the previous pixel's last
//                     source index / -accum (for the carry);
//             expand: left / right source index and int32(accum);
//   ytab[rows] shrink: the source rows imported since the previous export
//                     (IRow is zeroed by every export: FYScale is 0 when
//                     shrinking, rescale.go:91-93, :235-257);
//             expand: the current source row, the source row whose FRow sits
//                     in IRow (copied at the previous export), and the
//                     interpolation weight b (0 = the YAccum == 0 direct path).
//
// and every destination pixel is then independent: one lane computes the
// FRow values of the source rows it needs straight from HBM and combines them
// exactly as ExportRow does.  Each source byte is read once (twice at a
// fractional column/row boundary); the bound is HBM: sw*sh + dw*dh bytes.
#include <string.h>

#include <vector>

#include "wg_common.h"
#include "wg_instr.h"

namespace {

constexpr int kRFix = 32;

struct XEntry {  // 8 x int32 (32 B) per destination column
  int32_t a, b, c;       // shrink: x0, n_in, n_extra   expand: left, right, accum
  uint32_t negacc;       // shrink: uint32(-accum) after the pixel
  int32_t prev_idx;      // shrink: previous pixel's base index (-1: base 0 or none)
  uint32_t prev_negacc;  // shrink: previous pixel's uint32(-accum)
  int32_t pad0, pad1;
};
struct YEntry {  // 4 x int32 per destination row
  int32_t s0, s1;  // shrink: rows s0..s1 inclusive   expand: current row, IRow's row (-1: zeros)
  uint32_t b;      // expand: rescalerFrac(-YAccum, YSub); 0 = direct
  int32_t pad;
};
struct Header {
  int32_t sw, sh, dw, dh, x_expand, y_expand, x_add, x_sub;
  uint32_t fx_scale, fy_scale, fxy_scale;
  int32_t rows;
  int32_t pad[4];
};
static_assert(sizeof(Header) == 64 && sizeof(XEntry) == 32 && sizeof(YEntry) == 16, "plan layout");

__host__ __device__ inline uint32_t mult_fix(uint32_t x, uint32_t y) {
  return (uint32_t)(((uint64_t)x * y + ((uint64_t)1 << (kRFix - 1))) >> kRFix);
}
inline uint32_t frac_of(int64_t x, int64_t y) { return y == 0 ? 0u : (uint32_t)(((uint64_t)x << kRFix) / (uint64_t)y); }

__host__ __device__ inline size_t plan_bytes(int dw, int dh) { return sizeof(Header) + sizeof(XEntry) * (size_t)dw + sizeof(YEntry) * (size_t)dh; }

// Walks RescalerInit / ImportRow / ExportRow (rescale.go:63-257) over sizes only.
void build_plan(int sw, int sh, int dw, int dh, std::vector<uint8_t>& out) {
  out.assign(plan_bytes(dw, dh), 0);
  Header* hd = reinterpret_cast<Header*>(out.data());
  XEntry* xt = reinterpret_cast<XEntry*>(out.data() + sizeof(Header));
  YEntry* yt = reinterpret_cast<YEntry*>(out.data() + sizeof(Header) + sizeof(XEntry) * (size_t)dw);
  hd->sw = sw, hd->sh = sh, hd->dw = dw, hd->dh = dh;
  hd->x_expand = dw > sw;
  hd->y_expand = dh > sh;
  hd->x_add = sw, hd->x_sub = dw;
  if (!hd->x_expand) hd->fx_scale = frac_of(1, dw);
  if (hd->y_expand) hd->fy_scale = frac_of(1, dh);
  if (!hd->y_expand) {
    const uint64_t ratio = ((uint64_t)dh << kRFix) / ((uint64_t)sw * (uint64_t)sh);
    hd->fxy_scale = ratio != (uint64_t)(uint32_t)ratio ? 0u : (uint32_t)ratio;
  }
  if (hd->x_expand) {  // rescalerImportRowExpand (:128-153)
    int x_in = 1, left = 0, right = sw > 1 ? 1 : 0;
    int64_t accum = sw;
    for (int x = 0;;) {
      xt[x].a = left, xt[x].b = right, xt[x].c = (int32_t)accum;
      if (++x >= dw) break;
      accum -= dw;
      if (accum < 0) {
        left = right;
        if (++x_in < sw) right = x_in;
        accum += sw;
      }
    }
  } else {  // rescalerImportRowShrink (:157-181)
    int x_in = 0;
    int64_t accum = 0;
    int32_t prev_idx = -1;
    uint32_t prev_negacc = 0;
    for (int x = 0; x < dw; x++) {
      int32_t base_idx = -1, n_in = 0, n_extra = 0;
      const int x0 = x_in;
      accum += sw;
      while (accum > 0) {
        accum -= dw;
        if (x_in < sw) base_idx = x_in, n_in++;
        else n_extra++;
        x_in++;
      }
      xt[x].a = x0, xt[x].b = n_in, xt[x].c = n_extra;
      xt[x].negacc = (uint32_t)(-accum);
      xt[x].prev_idx = prev_idx, xt[x].prev_negacc = prev_negacc;
      prev_idx = base_idx, prev_negacc = (uint32_t)(-accum);
    }
  }
  // vertical walk with the plane driver of or_rescale_plane: import while
  // YAccum > 0 (and source rows remain), else export.
  int64_t y_accum = hd->y_expand ? dh : sh;
  int src_y = 0, rows = 0, first_unexported = 0, irow_src = -1;
  while (rows < dh) {
    if (y_accum > 0) {
      if (src_y >= sh) break;
      src_y++;
      y_accum -= dh;
    } else {
      YEntry& e = yt[rows];
      if (hd->y_expand) {
        e.s0 = src_y - 1;
        e.s1 = irow_src;
        e.b = y_accum == 0 ? 0u : frac_of(-y_accum, dh);
        irow_src = src_y - 1;
      } else {
        e.s0 = first_unexported;
        e.s1 = src_y - 1;
        first_unexported = src_y;
      }
      y_accum += sh;
      rows++;
    }
  }
  hd->rows = rows;
}

// FRow[x] of one source row (ImportRow's horizontal half)
// (sb / sn: the source buffer and its extent, for WG_BOUNDS builds)
__device__ __forceinline__ uint32_t frow_at(const uint8_t* __restrict__ row, const XEntry& e, int x_expand,
                                            int32_t x_add, int32_t x_sub, uint32_t fx_scale, const uint8_t* sb,
                                            int64_t sn) {
  if (x_expand) {
    const uint32_t left = WG_CHK(row + e.a, 1, sb, sn, "k_rescale src") ? row[e.a] : 0;
    const uint32_t right = WG_CHK(row + e.b, 1, sb, sn, "k_rescale src") ? row[e.b] : 0;
    return right * (uint32_t)x_add + (left - right) * (uint32_t)e.c;
  }
  uint32_t sum = 0;
  if (e.prev_idx >= 0 && e.prev_negacc != 0 && WG_CHK(row + e.prev_idx, 1, sb, sn, "k_rescale src"))
    sum = mult_fix((uint32_t)row[e.prev_idx] * e.prev_negacc, fx_scale);
  uint32_t base = 0;
  const uint8_t* p = row + e.a;
  for (int i = 0; i < e.b; i++) {
    base = WG_CHK(p + i, 1, sb, sn, "k_rescale src") ? p[i] : 0;
    sum += base;
  }
  sum += base * (uint32_t)e.c;
  return sum * (uint32_t)x_sub - base * e.negacc;
}

__global__ void __launch_bounds__(256) k_rescale(const uint8_t* __restrict__ plan, const uint8_t* __restrict__ src,
                                                 int64_t src_stride, int64_t src_pitch, uint8_t* __restrict__ dst,
                                                 int64_t dst_stride, int64_t dst_pitch) {
  const Header hd = *reinterpret_cast<const Header*>(plan);
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= hd.dw || y >= hd.rows) return;
  // (WG_BOUNDS) the extents the entry point's shapes give every buffer
  [[maybe_unused]] const int64_t plan_n = (int64_t)plan_bytes(hd.dw, hd.dh), src_n = (int64_t)gridDim.z * src_pitch,
                                 dst_n = (int64_t)gridDim.z * dst_pitch;
  (void)WG_CHK(plan + sizeof(Header) + sizeof(XEntry) * (size_t)x, sizeof(XEntry), plan, plan_n, "k_rescale xtab");
  (void)WG_CHK(plan + sizeof(Header) + sizeof(XEntry) * (size_t)hd.dw + sizeof(YEntry) * (size_t)y, sizeof(YEntry),
               plan, plan_n, "k_rescale ytab");
  const XEntry e = reinterpret_cast<const XEntry*>(plan + sizeof(Header))[x];
  const YEntry ye = reinterpret_cast<const YEntry*>(plan + sizeof(Header) + sizeof(XEntry) * (size_t)hd.dw)[y];
  const uint8_t* img = src + (int64_t)blockIdx.z * src_pitch;
  uint32_t v;
  if (hd.y_expand) {  // rescalerExportRowExpand (:203-231)
    const uint32_t f = frow_at(img + ye.s0 * src_stride, e, hd.x_expand, hd.x_add, hd.x_sub, hd.fx_scale, src, src_n);
    uint32_t j = f;
    if (ye.b != 0) {
      const uint32_t ir = ye.s1 < 0 ? 0u : frow_at(img + ye.s1 * src_stride, e, hd.x_expand, hd.x_add, hd.x_sub,
                                                  hd.fx_scale, src, src_n);
      const uint32_t a = (uint32_t)((((uint64_t)1) << kRFix) - ye.b);
      const uint64_t i = (uint64_t)a * f + (uint64_t)ye.b * ir;
      j = (uint32_t)((i + ((uint64_t)1 << (kRFix - 1))) >> kRFix);
    }
    v = mult_fix(j, hd.fy_scale);
  } else {  // IRow = sum of FRow since the previous export; rescalerExportRowShrink (:235-257)
    uint32_t acc = 0;
    for (int s = ye.s0; s <= ye.s1; s++)
      acc += frow_at(img + s * src_stride, e, hd.x_expand, hd.x_add, hd.x_sub, hd.fx_scale, src, src_n);
    v = mult_fix(acc, hd.fxy_scale);
  }
  uint8_t* const d = dst + (int64_t)blockIdx.z * dst_pitch + y * dst_stride + x;
  if (WG_CHK(d, 1, dst, dst_n, "k_rescale dst")) *d = (uint8_t)(v > 255u ? 255u : v);
}

}  // namespace

extern "C" size_t wg_rescaler_plan_bytes(int32_t dst_width, int32_t dst_height) {
  return dst_width > 0 && dst_height > 0 ? plan_bytes(dst_width, dst_height) : 0;
}

extern "C" int wg_rescaler_plan_host(int32_t src_width, int32_t src_height, int32_t dst_width, int32_t dst_height,
                                     void* plan_host, int32_t* rows) {
  WG_REQUIRE(plan_host && src_width > 0 && src_height > 0 && dst_width > 0 && dst_height > 0);
  std::vector<uint8_t> host;
  build_plan(src_width, src_height, dst_width, dst_height, host);
  memcpy(plan_host, host.data(), host.size());
  if (rows) *rows = reinterpret_cast<const Header*>(host.data())->rows;
  return WG_OK;
}

extern "C" int wg_rescaler_plan(int32_t src_width, int32_t src_height, int32_t dst_width, int32_t dst_height,
                                void* plan, int32_t* rows, void* stream) {
  WG_REQUIRE(plan && src_width > 0 && src_height > 0 && dst_width > 0 && dst_height > 0);
  std::vector<uint8_t> host;
  build_plan(src_width, src_height, dst_width, dst_height, host);
  hipStream_t s = wg::as_stream(stream);
  if (hipMemcpyAsync(plan, host.data(), host.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return wg::check_launch("wg_rescaler_plan copy");
  if (rows) *rows = reinterpret_cast<const Header*>(host.data())->rows;
  return WG_OK;
}

extern "C" int wg_rescale(const void* plan, int32_t dst_width, int32_t rows, const uint8_t* src, int64_t src_stride,
                          int64_t src_pitch, uint8_t* dst, int64_t dst_stride, int64_t dst_pitch, int32_t n_images,
                          void* stream) {
  WG_REQUIRE(plan && src && dst && dst_width > 0 && rows >= 0 && n_images >= 0 && src_stride > 0 &&
             dst_stride >= dst_width);
  if (rows == 0 || n_images == 0) return WG_OK;
  hipLaunchKernelGGL(k_rescale, dim3(wg::blocks_for(dst_width, 256), rows, n_images), dim3(256), 0,
                     wg::as_stream(stream), static_cast<const uint8_t*>(plan), src, src_stride, src_pitch, dst,
                     dst_stride, dst_pitch);
  return wg::check_launch("k_rescale");
}
