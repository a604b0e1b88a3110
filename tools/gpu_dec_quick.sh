#!/bin/bash
# GPU box: decode parity (frames, bitstreams, reference testdata), then C3 timings.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step dec 600 python -u -m pytest tests/test_gpu_frames.py tests/test_reference_testdata.py tests/test_gpu_bench_config.py -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=6 step c3 300 python tools/bench_c3.py
TAILN=6 step c3b 300 python tools/bench_c3.py
