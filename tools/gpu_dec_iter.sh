#!/bin/bash
# GPU box: decoder parity, C3 timing and the split kernel's phase cycles.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step dec 400 python -u -m pytest tests/test_gpu_frames.py tests/test_reference_testdata.py tests/test_gpu_bench_config.py -x -q -m gpu -k "decode or vp8 or nrgba or bench" --timeout 200 --timeout-method thread
TAILN=3 C3_ONLY=1 step c3 300 python tools/bench_c3.py
TAILN=3 WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so step ph 300 python tools/debug_split_phases.py
