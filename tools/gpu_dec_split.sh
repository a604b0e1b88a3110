#!/bin/bash
# GPU box: decoder parity with the current default kernel, then C3 / batch
# decode timings for k_decode_bands vs k_decode_split (WG_DECODE_KERNEL).
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step dec 400 python -u -m pytest tests/test_gpu_frames.py tests/test_reference_testdata.py -x -q -m gpu -k "decode or vp8 or nrgba" --timeout 120 --timeout-method thread
TAILN=3 C3_ONLY=1 WG_DECODE_KERNEL=bands step c3_bands 300 python tools/bench_c3.py
TAILN=3 C3_ONLY=1 WG_DECODE_KERNEL=split step c3_split 300 python tools/bench_c3.py
