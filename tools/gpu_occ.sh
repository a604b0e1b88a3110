#!/bin/bash
# GPU box: encoder per-phase cycles at the default occupancy (2 workgroups / CU)
# and with dynamic LDS padding forcing one workgroup (one wave per SIMD).
mkdir -p gpurun_out
export TMPDIR=/tmp
export WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so
for pad in 0 80000; do
  for c in mix noise; do
    WEBPGPU_ENC_LDS_PAD=$pad CONTENT=$c timeout -k 10 240 python tools/debug_enc_phases.py 2>&1 | grep -v amdgpu.ids | sed "s/^/pad=$pad /" || exit 1
  done
done
