#!/bin/bash
# GPU box: C5 kernels -- parity of the current build (SharpYUV, SSIM, VP8L,
# shard band tests), then tools/bench_c5.py for the current build and for the
# A/B switches given as env assignments in $AB (e.g. "WG_SHARP_KERNEL=band").
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -30 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step c5tests 600 python -u -m pytest tests/test_sharpyuv.py tests/test_gpu_shard.py tests/test_gpu_multi_device.py tests/test_reference_pins.py tests/test_gpu_lossless.py tests/test_blockops_yuv.py -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=1 step c5_new 300 python tools/bench_c5.py
for ab in $AB; do TAILN=1 step c5_$ab 300 env $ab python tools/bench_c5.py; done
