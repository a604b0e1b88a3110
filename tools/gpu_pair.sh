#!/bin/bash
# GPU box: encoder parity under both row schedules (one wave / a wave pair a
# row), the bench-configuration parity, then C2 / C3 timings with the pair
# schedule (default for one frame) and forced off (A/B), and encoder batch scaling.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step enc 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_bench_config.py tests/test_gpu_segments.py -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=12 step c3_pair 300 python tools/bench_c3.py
WG_ENCODE_PAIR=0 TAILN=12 step c3_single 300 python tools/bench_c3.py
TAILN=8 step scale 300 python tools/enc_scaling.py
