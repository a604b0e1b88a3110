// Measurement kernels (not product code): cycles per step of a dependent
// chain through one cross-lane move, one wave alone on the chip, timed with
// s_memtime inside the kernel.  kind: 0 wave_shr:1 DPP, 1 row_shr:1 DPP,
// 2 no cross-lane move (plain VALU chain), 3 row_bcast:15 + row_shr:1
// (wave_shr composed), 4 ds_bpermute (__shfl_up), 5 wave_shr + a ds_write_b8 a step
#include <hip/hip_runtime.h>
#include <cstdint>

template <int KIND>
__global__ __launch_bounds__(64) void k_chain(int* out, unsigned long long* cyc, int n) {
  __shared__ uint8_t ring[64 * 132];
  int v = threadIdx.x, o = threadIdx.x * 3;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++) {
      int t;
      if constexpr (KIND == 0) t = __builtin_amdgcn_update_dpp(o, v, 0x138, 0xf, 0xf, false);
      else if constexpr (KIND == 1) t = __builtin_amdgcn_update_dpp(o, v, 0x111, 0xf, 0xf, false);
      else if constexpr (KIND == 2) t = v ^ o;
      else if constexpr (KIND == 3) {
        const int b = __builtin_amdgcn_update_dpp(o, v, 0x142, 0xe, 0xf, false);
        t = __builtin_amdgcn_update_dpp(b, v, 0x111, 0xf, 0xf, false);
      } else if constexpr (KIND == 4) t = __shfl_up(v, 1, 64);
      else t = __builtin_amdgcn_update_dpp(o, v, 0x138, 0xf, 0xf, false);
      v = min(max(t + v - o, 0), 255) + (u & 3);
      if constexpr (KIND == 5) ring[threadIdx.x * 132 + ((i * 16 + u) & 127)] = (uint8_t)v;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = v;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

extern "C" int probe_chain(int kind, int n, int* out, unsigned long long* cyc) {
  switch (kind) {
    case 0: hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, out, cyc, n); break;
    case 1: hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, out, cyc, n); break;
    case 2: hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, out, cyc, n); break;
    case 3: hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(64), 0, 0, out, cyc, n); break;
    case 4: hipLaunchKernelGGL(k_chain<4>, dim3(1), dim3(64), 0, 0, out, cyc, n); break;
    default: hipLaunchKernelGGL(k_chain<5>, dim3(1), dim3(64), 0, 0, out, cyc, n); break;
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
