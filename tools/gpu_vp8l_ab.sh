#!/bin/bash
# GPU box: VP8L parity (lossless tests + the reference's testdata files), then
# the C5 stage timings with the A build (webp_amd/libwebpgpu_a.so) and the
# current build.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step vp8l 300 python -u -m pytest tests/test_gpu_lossless.py tests/test_reference_testdata.py tests/test_vp8l_color.py -x -q -m gpu --timeout 120 --timeout-method thread
TAILN=1 WEBPGPU_LIB=webp_amd/libwebpgpu_a.so step c5a 300 python tools/bench_c5.py
TAILN=1 step c5b 300 python tools/bench_c5.py
