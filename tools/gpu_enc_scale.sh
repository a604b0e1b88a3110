#!/bin/bash
# GPU box: encoder time vs batch at occupancy 3 (default build) and 2.
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "occ3"; timeout -k 10 300 python tools/enc_scaling.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "occ2"; WEBPGPU_LIB=webp_amd/libwebpgpu_occ2.so timeout -k 10 300 python tools/enc_scaling.py 2>&1 | grep -v amdgpu.ids || exit 1
