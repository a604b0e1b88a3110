// probe.hip -- measurement kernels, not product code (tools/libprobe.so).
//
//  probe_copy            a streaming device-to-device copy: the measured HBM
//                        copy ceiling bench.py reports beside the 8 TB/s spec
//                        ("also report a measured copy-kernel peak").
//  probe_read_stream     16 B per lane, lane-contiguous reads of a known byte
//                        count: MI355X_MICROARCH.md's gfx950 FETCH_SIZE case (x2).
//  probe_read_rows       k_encode_rows' source-row pattern: a wave owns 16
//                        rows, lanes 0..15 read `piece` bytes (16-B or 8-B
//                        loads) of their own row, walking the row left to right;
//                        with s_sleep between pieces (slow variants) so the sectors of one
//                        128-B line are requested far apart, as they are when a
//                        wave walks its MB row (~70 us per MB).
//  probe_write_rows      the same pattern for stores (the reconstruction rows).
// tools/fetch_calib.py runs each under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
// and divides the counters by the bytes moved; tools/pmc_summary.py applies the
// ratio measured for k_encode_rows' pattern.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_probe_copy(v4u* __restrict__ dst, const v4u* __restrict__ src, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const v4u a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + stride);
    const v4u c = __builtin_nontemporal_load(src + i + 2 * stride), d = __builtin_nontemporal_load(src + i + 3 * stride);
    __builtin_nontemporal_store(a, dst + i);
    __builtin_nontemporal_store(b, dst + i + stride);
    __builtin_nontemporal_store(c, dst + i + 2 * stride);
    __builtin_nontemporal_store(d, dst + i + 3 * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ void __launch_bounds__(256) k_probe_read_stream(const uint4* __restrict__ src, int64_t n16, uint32_t* out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int64_t i = t; i < n16; i += stride) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[t] = acc;
}

// wave w owns rows [16w, 16w + 16); lanes 0..15 read, the others idle (as in
// k_encode_rows' Y import); piece = 32 (two 16-B loads) or 8 (one 8-B load)
template <int PIECE, bool SLOW>
__global__ void __launch_bounds__(64) k_probe_read_rows(const uint8_t* __restrict__ src, int64_t pitch, int row_bytes,
                                                        uint32_t* out) {
  const int lane = threadIdx.x;
  const int64_t row = 16 * (int64_t)blockIdx.x + lane;
  uint32_t acc = 0;
  if (lane < 16) {
    const uint8_t* p = src + row * pitch;
    for (int c = 0; c < row_bytes; c += PIECE) {
      if constexpr (PIECE == 32) {
        const uint4 a = *reinterpret_cast<const uint4*>(p + c), b = *reinterpret_cast<const uint4*>(p + c + 16);
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
      } else {
        const uint2 a = *reinterpret_cast<const uint2*>(p + c);
        acc ^= a.x ^ a.y;
      }
      if constexpr (SLOW) {  // ~14 us between a row's pieces
        for (int s = 0; s < 4; s++) __builtin_amdgcn_s_sleep(127);
      }
    }
  }
  out[(int64_t)blockIdx.x * 64 + lane] = acc;
}

template <int PIECE, bool SLOW>
__global__ void __launch_bounds__(64) k_probe_write_rows(uint8_t* __restrict__ dst, int64_t pitch, int row_bytes) {
  const int lane = threadIdx.x;
  const int64_t row = 16 * (int64_t)blockIdx.x + lane;
  if (lane < 16) {
    uint8_t* p = dst + row * pitch;
    for (int c = 0; c < row_bytes; c += PIECE) {
      const uint32_t v = (uint32_t)(row * 131 + c);
      if constexpr (PIECE == 32) {
        *reinterpret_cast<uint4*>(p + c) = make_uint4(v, v + 1, v + 2, v + 3);
        *reinterpret_cast<uint4*>(p + c + 16) = make_uint4(v + 4, v + 5, v + 6, v + 7);
      } else {
        *reinterpret_cast<uint2*>(p + c) = make_uint2(v, v + 1);
      }
      if constexpr (SLOW) {  // ~14 us between a row's pieces
        for (int s = 0; s < 4; s++) __builtin_amdgcn_s_sleep(127);
      }
    }
  }
}

int status() { return hipGetLastError() == hipSuccess ? 0 : -1; }

}  // namespace

extern "C" int probe_copy(void* dst, const void* src, int64_t bytes, int grid, void* stream) {
  if ((bytes & 15) || (((uintptr_t)dst | (uintptr_t)src) & 15) || grid <= 0) return -2;
  hipLaunchKernelGGL(k_probe_copy, dim3(grid), dim3(256), 0, (hipStream_t)stream, (v4u*)dst, (const v4u*)src,
                     bytes / 16);
  return status();
}

extern "C" int probe_read_stream(const void* src, int64_t bytes, int grid, uint32_t* out, void* stream) {
  if ((bytes & 15) || ((uintptr_t)src & 15) || grid <= 0) return -2;
  hipLaunchKernelGGL(k_probe_read_stream, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint4*)src, bytes / 16,
                     out);
  return status();
}

// rows must be a multiple of 16; out holds rows / 16 * 64 words; slow: s_sleep between pieces
#define PROBE_ROWS(K, ...)                                                                              \
  do {                                                                                                  \
    const dim3 g((unsigned)(rows / 16));                                                                \
    hipStream_t s = (hipStream_t)stream;                                                                \
    if (piece == 32 && slow) hipLaunchKernelGGL((K<32, true>), g, dim3(64), 0, s, __VA_ARGS__);        \
    else if (piece == 32) hipLaunchKernelGGL((K<32, false>), g, dim3(64), 0, s, __VA_ARGS__);           \
    else if (slow) hipLaunchKernelGGL((K<8, true>), g, dim3(64), 0, s, __VA_ARGS__);                   \
    else hipLaunchKernelGGL((K<8, false>), g, dim3(64), 0, s, __VA_ARGS__);                             \
  } while (0)

extern "C" int probe_read_rows(const void* src, int64_t pitch, int64_t rows, int row_bytes, int piece, int slow,
                               uint32_t* out, void* stream) {
  if ((rows & 15) || (piece != 32 && piece != 8) || row_bytes % piece || (((uintptr_t)src | pitch) & 15)) return -2;
  PROBE_ROWS(k_probe_read_rows, (const uint8_t*)src, pitch, row_bytes, out);
  return status();
}

extern "C" int probe_write_rows(void* dst, int64_t pitch, int64_t rows, int row_bytes, int piece, int slow,
                                void* stream) {
  if ((rows & 15) || (piece != 32 && piece != 8) || row_bytes % piece || (((uintptr_t)dst | pitch) & 15)) return -2;
  PROBE_ROWS(k_probe_write_rows, (uint8_t*)dst, pitch, row_bytes);
  return status();
}
