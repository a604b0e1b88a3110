// multi_device.hip -- the multi-device batch variant of the encode DSP path
// (last bullet; 8(e) C4) for a host that drives every GPU from
// one process, as the reference's Go program would through cgo.
//
// Frame i belongs to device devices[i % n_devices] (round-robin, the ownership
// webp_amd/shard.py frames_of uses for the one-process-per-GPU path).  Each
// device runs the whole device encode path over its frames on a stream of
// its own -- import (importImage, internal/lossy/encode.go:671-943) ->
// computeAlphas (encode_analysis.go:245-307) -> analysis() segments
// (encode_analysis.go:29-903) -> Phase A of encodeFrameParallel
// (encode_parallel.go:168-232) -- with no exchange between devices.  The only
// cross-device step is the final gather: every frame's MBEncInfo records,
// reconstruction, segment map and segment header come back to the caller's
// host buffers in frame order, which is where the reference's Phase B
// (recordAllTokens, encode_parallel.go:1497) and the bitstream writer run.
#include <algorithm>
#include <map>
#include <mutex>
#include <vector>

#include "vp8_tables.h"
#include "wg_common.h"

namespace {

struct DevJob {
  int dev = 0;
  hipStream_t stream = nullptr;
  std::vector<int> frames;  // global frame indices, in order
  void* mem = nullptr;      // one allocation, carved below
  uint8_t *rgba = nullptr, *y = nullptr, *u = nullptr, *v = nullptr, *seg_ids = nullptr, *segs = nullptr;
  uint8_t *proba = nullptr, *out = nullptr, *work = nullptr, *ry = nullptr, *ru = nullptr, *rv = nullptr;
  int32_t *alphas = nullptr, *uv_sum = nullptr;
  wg_frame_segs* info = nullptr;
};

inline size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

int fail_hip(hipError_t e, const char* what) {
  wg::set_error(std::string(what) + ": " + hipGetErrorString(e));
  return WG_EHIP;
}

// The caller's host buffers, page-locked for the duration of the call
// (hipHostRegister, portable to every device), so the per-device uploads and
// the gather are DMA transfers that overlap across devices instead of
// copies staged through the runtime's bounce buffers.
//
// Registrations are reference-counted across the process: concurrent calls
// (host threads) may pass the same or overlapping host buffers, and a range
// is unregistered only when the last call holding it returns -- never under
// another call's in-flight DMA.  A range that lies inside one this library
// registered takes a reference on it; one that cannot be registered (pinned
// by the caller, or overlapping a registered range) holds references on every
// registered range it overlaps and is copied as it is.
struct PinRange {
  size_t n;
  int refs;
};
std::mutex g_pin_mu;
std::map<uintptr_t, PinRange> g_pins;  // by start address

struct HostPins {
  std::vector<uintptr_t> held;  // starts of the g_pins ranges this call holds a reference on
  void pin(const void* p, size_t n) {
    if (!p || n == 0) return;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p), e = a + n;
    std::lock_guard<std::mutex> lock(g_pin_mu);
    // registered ranges overlapping [a, e)
    std::vector<uintptr_t> over;
    auto it = g_pins.upper_bound(a);
    if (it != g_pins.begin()) --it;
    for (; it != g_pins.end() && it->first < e; ++it)
      if (it->first + it->second.n > a) over.push_back(it->first);
    if (over.empty() && hipHostRegister(const_cast<void*>(p), n, hipHostRegisterPortable) == hipSuccess) {
      g_pins[a] = PinRange{n, 1};
      held.push_back(a);
      return;
    }
    (void)hipGetLastError();  // not fatal: the copies stay correct
    for (uintptr_t k : over) {
      g_pins[k].refs++;
      held.push_back(k);
    }
  }
  ~HostPins() {
    std::lock_guard<std::mutex> lock(g_pin_mu);
    for (uintptr_t k : held) {
      auto it = g_pins.find(k);
      if (it == g_pins.end()) continue;
      if (--it->second.refs == 0) {
        (void)hipHostUnregister(reinterpret_cast<void*>(k));
        g_pins.erase(it);
      }
    }
  }
};

// A first kernel on a new stream (its hardware queue is created then), issued
// before any persistent kernel runs: creating a queue while wg_encode_mbs runs
// on another one stalled it past its dependency-wait bound (webpgpu.h).
hipError_t bind_stream(void* mem, hipStream_t s) {
  hipError_t e = hipMemsetAsync(mem, 0, 256, s);
  return e == hipSuccess ? hipStreamSynchronize(s) : e;
}

}  // namespace

extern "C" int wg_encode_frames_devices(const int32_t* devices, int32_t n_devices, const uint8_t* rgba, int32_t w,
                                        int32_t h, int32_t n_images, int32_t has_alpha, const wg_enc_config* cfg,
                                        void* mb_out, uint8_t* ry, uint8_t* ru, uint8_t* rv, uint8_t* seg_ids_out,
                                        wg_frame_segs* info_out) {
  WG_REQUIRE(devices && n_devices > 0 && rgba && cfg && mb_out);
  WG_REQUIRE(w > 0 && h > 0 && n_images > 0);
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) return wg::check_launch("hipGetDeviceCount");
  // a device may appear more than once: each entry gets its own stream and
  // buffers (how the tests split work on a one-GPU box)
  for (int k = 0; k < n_devices; k++) WG_REQUIRE(devices[k] >= 0 && devices[k] < count);
  const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4;
  if (mbh < 4) return wg::invalid("mbh >= 4 (encode.go:1356 encodes smaller frames serially)");
  const int64_t n_mb = (int64_t)mbw * mbh;
  const int64_t rgba_b = (int64_t)w * h * 4, y_b = 256 * n_mb, uv_b = 64 * n_mb, seg_pitch = 4 * sizeof(wg_segment);
  int prev_dev = 0;
  if (hipGetDevice(&prev_dev) != hipSuccess) return wg::check_launch("hipGetDevice");
  HostPins pins;
  pins.pin(rgba, (size_t)(rgba_b * n_images));
  pins.pin(mb_out, (size_t)(n_mb * n_images) * sizeof(wg_mb_enc));
  pins.pin(ry, (size_t)(y_b * n_images));
  pins.pin(ru, (size_t)(uv_b * n_images));
  pins.pin(rv, (size_t)(uv_b * n_images));
  pins.pin(seg_ids_out, (size_t)(n_mb * n_images));
  pins.pin(info_out, (size_t)n_images * sizeof(wg_frame_segs));

  std::vector<DevJob> jobs((size_t)n_devices);
  for (int i = 0; i < n_images; i++) jobs[(size_t)(i % n_devices)].frames.push_back(i);
  int rc = WG_OK;
  // every device's stream and buffers first (the streams bound to their
  // queues before any persistent kernel runs), then every device's work, so
  // the devices run at once
  for (auto& j : jobs) {
    j.dev = devices[&j - jobs.data()];
    const int nk = (int)j.frames.size();
    if (nk == 0) continue;
    hipError_t e = hipSetDevice(j.dev);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&j.stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      rc = fail_hip(e, "device setup");
      break;
    }
    const size_t work_b = wg_encode_work_bytes(mbw, mbh, nk);
    size_t sz[15] = {(size_t)(rgba_b * nk), (size_t)(y_b * nk), (size_t)(uv_b * nk), (size_t)(uv_b * nk),
                     (size_t)(n_mb * nk), (size_t)(seg_pitch * nk), sizeof(vp8_coeffs_proba0),
                     (size_t)(n_mb * nk) * sizeof(wg_mb_enc), work_b, (size_t)(y_b * nk), (size_t)(uv_b * nk),
                     (size_t)(uv_b * nk), (size_t)(n_mb * nk) * 4, (size_t)nk * 4, (size_t)nk * sizeof(wg_frame_segs)};
    size_t total = 0;
    for (size_t s : sz) total += align_up(s);
    if ((e = hipMalloc(&j.mem, total)) != hipSuccess) {
      rc = fail_hip(e, "hipMalloc (encode batch)");
      break;
    }
    uint8_t* p = static_cast<uint8_t*>(j.mem);
    uint8_t* parts[15];
    for (int q = 0; q < 15; q++) {
      parts[q] = p;
      p += align_up(sz[q]);
    }
    j.rgba = parts[0], j.y = parts[1], j.u = parts[2], j.v = parts[3], j.seg_ids = parts[4], j.segs = parts[5];
    j.proba = parts[6], j.out = parts[7], j.work = parts[8], j.ry = parts[9], j.ru = parts[10], j.rv = parts[11];
    j.alphas = reinterpret_cast<int32_t*>(parts[12]), j.uv_sum = reinterpret_cast<int32_t*>(parts[13]);
    j.info = reinterpret_cast<wg_frame_segs*>(parts[14]);
    if ((e = bind_stream(j.mem, j.stream)) != hipSuccess) {
      rc = fail_hip(e, "stream setup");
      break;
    }
  }
  for (auto& j : jobs) {
    const int nk = (int)j.frames.size();
    if (nk == 0 || rc != WG_OK) continue;
    hipError_t e = hipSetDevice(j.dev);
    for (int q = 0; q < nk && e == hipSuccess; q++)
      e = hipMemcpyAsync(j.rgba + q * rgba_b, rgba + (int64_t)j.frames[(size_t)q] * rgba_b, (size_t)rgba_b,
                         hipMemcpyHostToDevice, j.stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(j.proba, vp8_coeffs_proba0, sizeof(vp8_coeffs_proba0), hipMemcpyHostToDevice, j.stream);
    if (e != hipSuccess) {
      rc = fail_hip(e, "hipMemcpyAsync (frames to device)");
      break;
    }
    void* st = j.stream;
    if ((rc = wg_import_rgba(j.rgba, w, h, 4 * w, rgba_b, has_alpha, j.y, j.u, j.v, y_b, uv_b, nk, st)) != WG_OK) break;
    if ((rc = wg_analysis_alphas(j.y, j.u, j.v, w, h, y_b, uv_b, nk, j.alphas, nullptr, nullptr, j.uv_sum, st)) != WG_OK)
      break;
    if ((rc = wg_segment_analysis(cfg, j.alphas, j.uv_sum, mbw, mbh, nk, j.seg_ids, j.segs, seg_pitch, j.info, st)) !=
        WG_OK)
      break;
    if ((rc = wg_encode_row_order(j.alphas, mbw, mbh, nk, j.work, st)) != WG_OK) break;
    if ((rc = wg_encode_mbs(j.y, j.u, j.v, y_b, uv_b, w, h, nk, j.seg_ids, j.segs, seg_pitch, j.proba, cfg->method,
                            cfg->quality, j.out, j.ry, j.ru, j.rv, j.work, st)) != WG_OK)
      break;
  }
  // the gather: each device's frames back to their places in the host
  // buffers, enqueued on every device first (the copies of one device overlap
  // the others' kernels and copies), then each stream synchronised and its
  // in-kernel wait status checked (a timed-out launch invalidates the outputs)
  for (auto& j : jobs) {
    if (!j.mem || rc != WG_OK) continue;
    hipError_t e = hipSetDevice(j.dev);
    for (size_t q = 0; q < j.frames.size() && e == hipSuccess; q++) {
      const int64_t i = j.frames[q];
      const int64_t rec_b = n_mb * (int64_t)sizeof(wg_mb_enc);
      e = hipMemcpyAsync(static_cast<uint8_t*>(mb_out) + i * rec_b, j.out + (int64_t)q * rec_b, (size_t)rec_b,
                         hipMemcpyDeviceToHost, j.stream);
      if (e == hipSuccess && ry) e = hipMemcpyAsync(ry + i * y_b, j.ry + q * y_b, (size_t)y_b, hipMemcpyDeviceToHost, j.stream);
      if (e == hipSuccess && ru) e = hipMemcpyAsync(ru + i * uv_b, j.ru + q * uv_b, (size_t)uv_b, hipMemcpyDeviceToHost, j.stream);
      if (e == hipSuccess && rv) e = hipMemcpyAsync(rv + i * uv_b, j.rv + q * uv_b, (size_t)uv_b, hipMemcpyDeviceToHost, j.stream);
      if (e == hipSuccess && seg_ids_out)
        e = hipMemcpyAsync(seg_ids_out + i * n_mb, j.seg_ids + q * n_mb, (size_t)n_mb, hipMemcpyDeviceToHost, j.stream);
      if (e == hipSuccess && info_out)
        e = hipMemcpyAsync(info_out + i, j.info + q, sizeof(wg_frame_segs), hipMemcpyDeviceToHost, j.stream);
    }
    if (e != hipSuccess) rc = fail_hip(e, "gather (device to host)");
  }
  for (auto& j : jobs) {
    if (!j.mem || rc != WG_OK) continue;
    if (hipError_t e = hipSetDevice(j.dev); e != hipSuccess) {
      rc = fail_hip(e, "hipSetDevice (gather)");
      continue;
    }
    const int st = wg_encode_status(j.work, mbw, (int)j.frames.size(), j.stream);  // synchronises the stream
    if (st != WG_OK) rc = st;
  }
  for (auto& j : jobs) {
    if (!j.stream && !j.mem) continue;
    (void)hipSetDevice(j.dev);
    if (j.stream) (void)hipStreamSynchronize(j.stream);
    if (j.mem) (void)hipFree(j.mem);
    if (j.stream) (void)hipStreamDestroy(j.stream);
  }
  (void)hipSetDevice(prev_dev);
  return rc;
}

// ---------------- one large image over several devices: row bands (C5) ----------------
//
// the streaming stages of C5 shard by row bands with a halo --
// VP8L ResidualImage by tile rows (1 pixel row above the band: the
// predictors read the row above), plane SSIM by 16-row tiles (3 rows each
// side).  Device k of n takes the contiguous tile-row band band_of(k) (the
// first tiles % n devices one tile row more, as webp_amd/shard.py band_of),
// computes it through the *_rows entry points from its rows plus the halo,
// and the bands come back to host memory at their places.  The SSIM bands'
// per-tile partial sums are reduced on the first device in the one-device
// order, so the sum is bit-identical to wg_plane_ssim's.
namespace {

void band_of(int tiles, int n, int k, int* b0, int* b1) {
  const int base = tiles / n, rem = tiles % n;
  *b0 = k * base + (k < rem ? k : rem);
  *b1 = *b0 + base + (k < rem ? 1 : 0);
}

int check_devices(const int32_t* devices, int32_t n_devices) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) return wg::check_launch("hipGetDeviceCount");
  for (int k = 0; k < n_devices; k++) WG_REQUIRE(devices[k] >= 0 && devices[k] < count);
  return WG_OK;
}

struct Band {
  int dev = 0, t0 = 0, t1 = 0;
  hipStream_t stream = nullptr;
  void* mem = nullptr;
};

void release(std::vector<Band>& bands, int prev_dev) {
  for (auto& b : bands) {
    if (!b.stream && !b.mem) continue;
    (void)hipSetDevice(b.dev);
    if (b.stream) (void)hipStreamSynchronize(b.stream);
    if (b.mem) (void)hipFree(b.mem);
    if (b.stream) (void)hipStreamDestroy(b.stream);
  }
  (void)hipSetDevice(prev_dev);
}

}  // namespace

extern "C" int wg_vp8l_residual_image_devices(const int32_t* devices, int32_t n_devices, const uint32_t* argb,
                                              int32_t width, int32_t height, int32_t bits, int32_t quality,
                                              uint32_t* modes, uint32_t* residuals) {
  WG_REQUIRE(devices && n_devices > 0 && argb && modes && residuals);
  WG_REQUIRE(width > 0 && height > 0 && bits >= 2 && bits <= 9);
  if (int rc = check_devices(devices, n_devices)) return rc;
  const int ts = 1 << bits, tx = (width + ts - 1) >> bits, ty = (height + ts - 1) >> bits;
  const int64_t px = (int64_t)width * height, row_b = (int64_t)width * 4;
  int prev_dev = 0;
  if (hipGetDevice(&prev_dev) != hipSuccess) return wg::check_launch("hipGetDevice");
  HostPins pins;
  pins.pin(argb, (size_t)(px * 4));
  pins.pin(modes, (size_t)tx * ty * 4);
  pins.pin(residuals, (size_t)(px * 4));
  std::vector<Band> bands((size_t)n_devices);
  int rc = WG_OK;
  for (int k = 0; k < n_devices && rc == WG_OK; k++) {
    Band& b = bands[(size_t)k];
    b.dev = devices[k];
    band_of(ty, n_devices, k, &b.t0, &b.t1);
    if (b.t1 <= b.t0) continue;
    hipError_t e = hipSetDevice(b.dev);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking);
    // the band's rows (+ the row above) and its tile modes only: the *_rows
    // entry points address rows at their image positions, so they get base
    // pointers moved back by the band's first row / tile row (only the band's
    // own rows are ever touched)
    const int r0 = (b.t0 << bits) - (b.t0 > 0 ? 1 : 0), r1 = std::min(b.t1 << bits, (int)height);  // + the row above
    const size_t in_b = align_up((size_t)(r1 - r0) * row_b), modes_b = align_up((size_t)tx * (b.t1 - b.t0) * 4);
    if (e == hipSuccess) e = hipMalloc(&b.mem, 2 * in_b + modes_b);
    if (e != hipSuccess) {
      rc = fail_hip(e, "device setup (residual bands)");
      break;
    }
    uint8_t* base = static_cast<uint8_t*>(b.mem);
    uint32_t* d_argb = reinterpret_cast<uint32_t*>(base) - (int64_t)r0 * width;
    uint32_t* d_res = reinterpret_cast<uint32_t*>(base + in_b) - (int64_t)r0 * width;
    uint32_t* d_modes = reinterpret_cast<uint32_t*>(base + 2 * in_b) - (int64_t)b.t0 * tx;
    e = hipMemcpyAsync(base, argb + (int64_t)r0 * width, (size_t)((r1 - r0) * row_b), hipMemcpyHostToDevice, b.stream);
    if (e != hipSuccess) {
      rc = fail_hip(e, "hipMemcpyAsync (band to device)");
      break;
    }
    rc = wg_vp8l_residual_image_rows(d_argb, width, height, px, bits, quality, b.t0, b.t1, 1, d_modes, d_res, b.stream);
  }
  for (auto& b : bands) {  // gather: the band's tile modes and residual rows at their places
    if (!b.mem || rc != WG_OK) continue;
    if (hipError_t e = hipSetDevice(b.dev); e != hipSuccess) {
      rc = fail_hip(e, "hipSetDevice (residual gather)");
      continue;
    }
    uint8_t* base = static_cast<uint8_t*>(b.mem);
    const int h0 = (b.t0 << bits) - (b.t0 > 0 ? 1 : 0);  // the buffer's first row
    const int r0 = b.t0 << bits, r1 = std::min(b.t1 << bits, (int)height);
    const size_t in_b = align_up((size_t)(r1 - h0) * row_b);
    hipError_t e = hipMemcpyAsync(modes + (int64_t)b.t0 * tx, base + 2 * in_b, (size_t)(b.t1 - b.t0) * tx * 4,
                                  hipMemcpyDeviceToHost, b.stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(residuals + (int64_t)r0 * width, base + in_b + (size_t)(r0 - h0) * row_b,
                         (size_t)((r1 - r0) * row_b), hipMemcpyDeviceToHost, b.stream);
    if (e != hipSuccess) rc = fail_hip(e, "gather (residual bands)");
  }
  for (auto& b : bands) {  // every device's gather is in flight: now wait for each
    if (!b.mem || rc != WG_OK) continue;
    hipError_t e = hipSetDevice(b.dev);
    if (e == hipSuccess) e = hipStreamSynchronize(b.stream);
    if (e != hipSuccess) rc = fail_hip(e, "gather (residual bands)");
  }
  release(bands, prev_dev);
  return rc;
}

extern "C" int wg_plane_ssim_devices(const int32_t* devices, int32_t n_devices, const uint8_t* a, int32_t a_stride,
                                     const uint8_t* b_plane, int32_t b_stride, int32_t w, int32_t h, double* out) {
  WG_REQUIRE(devices && n_devices > 0 && a && b_plane && out);
  WG_REQUIRE(w > 0 && h > 0 && a_stride >= w && b_stride >= w);
  if (int rc = check_devices(devices, n_devices)) return rc;
  constexpr int TILE = 16, HALO = 3;
  const int tx = wg_plane_ssim_row_partials(w), ty = (h + TILE - 1) / TILE;  // partials per tile row, tile rows
  int prev_dev = 0;
  if (hipGetDevice(&prev_dev) != hipSuccess) return wg::check_launch("hipGetDevice");
  std::vector<Band> bands((size_t)n_devices);
  std::vector<double> partial((size_t)tx * ty);
  HostPins pins;  // (declared after `partial`: unpinned before it is freed)
  pins.pin(a, (size_t)a_stride * h);
  pins.pin(b_plane, (size_t)b_stride * h);
  pins.pin(partial.data(), partial.size() * sizeof(double));
  int rc = WG_OK;
  // each band's buffer: its rows + halo of both planes, then its partial sums
  auto rows_of = [&](const Band& b, int* r0, int* r1) {
    *r0 = std::max(TILE * b.t0 - HALO, 0);
    *r1 = std::min(TILE * b.t1 + HALO, (int)h);
  };
  for (int k = 0; k < n_devices && rc == WG_OK; k++) {
    Band& b = bands[(size_t)k];
    b.dev = devices[k];
    band_of(ty, n_devices, k, &b.t0, &b.t1);
    if (b.t1 <= b.t0) continue;
    hipError_t e = hipSetDevice(b.dev);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking);
    int r0, r1;
    rows_of(b, &r0, &r1);
    const size_t a_b = align_up((size_t)(r1 - r0) * a_stride), b_b = align_up((size_t)(r1 - r0) * b_stride);
    const size_t part_b = align_up((size_t)tx * (b.t1 - b.t0) * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&b.mem, a_b + b_b + part_b);
    if (e != hipSuccess) {
      rc = fail_hip(e, "device setup (ssim bands)");
      break;
    }
    uint8_t* base = static_cast<uint8_t*>(b.mem);
    e = hipMemcpyAsync(base, a + (size_t)r0 * a_stride, (size_t)(r1 - r0) * a_stride, hipMemcpyHostToDevice, b.stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(base + a_b, b_plane + (size_t)r0 * b_stride, (size_t)(r1 - r0) * b_stride, hipMemcpyHostToDevice,
                         b.stream);
    if (e != hipSuccess) {
      rc = fail_hip(e, "hipMemcpyAsync (ssim band to device)");
      break;
    }
    // plane bases moved back by r0 rows: the rows entry point addresses rows at their image positions
    rc = wg_plane_ssim_rows(base - (int64_t)r0 * a_stride, a_stride, (int64_t)a_stride * h,
                            base + a_b - (int64_t)r0 * b_stride, b_stride, (int64_t)b_stride * h, w, h, b.t0, b.t1, 1,
                            reinterpret_cast<double*>(base + a_b + b_b), b.stream);
  }
  for (auto& b : bands) {  // gather the per-tile partial sums in tile-row order
    if (!b.mem || rc != WG_OK) continue;
    if (hipError_t e = hipSetDevice(b.dev); e != hipSuccess) {
      rc = fail_hip(e, "hipSetDevice (ssim gather)");
      continue;
    }
    const uint8_t* base = static_cast<const uint8_t*>(b.mem);
    int r0, r1;
    rows_of(b, &r0, &r1);
    const size_t a_b = align_up((size_t)(r1 - r0) * a_stride), b_b = align_up((size_t)(r1 - r0) * b_stride);
    hipError_t e = hipMemcpyAsync(partial.data() + (size_t)b.t0 * tx, base + a_b + b_b,
                                  (size_t)tx * (b.t1 - b.t0) * sizeof(double), hipMemcpyDeviceToHost, b.stream);
    if (e != hipSuccess) rc = fail_hip(e, "gather (ssim bands)");
  }
  for (auto& b : bands) {  // every device's partials are in flight: now wait for each
    if (!b.mem || rc != WG_OK) continue;
    hipError_t e = hipSetDevice(b.dev);
    if (e == hipSuccess) e = hipStreamSynchronize(b.stream);
    if (e != hipSuccess) rc = fail_hip(e, "gather (ssim bands)");
  }
  if (rc == WG_OK) {  // the one-device reduction order, on the first device that holds a band
    for (auto& b : bands) {
      if (!b.mem) continue;
      void* red = nullptr;
      hipError_t e = hipSetDevice(b.dev);
      if (e == hipSuccess) e = hipMalloc(&red, align_up(partial.size() * sizeof(double)) + 256);
      if (e == hipSuccess) {
        double* d_part = static_cast<double*>(red);
        double* d_out = reinterpret_cast<double*>(static_cast<uint8_t*>(red) + align_up(partial.size() * sizeof(double)));
        e = hipMemcpyAsync(d_part, partial.data(), partial.size() * sizeof(double), hipMemcpyHostToDevice, b.stream);
        if (e == hipSuccess) {
          rc = wg_plane_ssim_reduce(d_part, (int64_t)partial.size(), 1, d_out, b.stream);
          if (rc == WG_OK) e = hipMemcpyAsync(out, d_out, sizeof(double), hipMemcpyDeviceToHost, b.stream);
          if (rc == WG_OK && e == hipSuccess) e = hipStreamSynchronize(b.stream);
        }
      }
      if (red) (void)hipFree(red);
      if (e != hipSuccess && rc == WG_OK) rc = fail_hip(e, "ssim reduce");
      break;
    }
  }
  release(bands, prev_dev);
  return rc;
}
