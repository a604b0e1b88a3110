#!/bin/bash
# GPU box: encoder parity (both row schedules, the bench configuration), C2 / C3
# timings, encoder batch scaling, one bench line without the CPU baseline.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step enc 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_bench_config.py tests/test_gpu_segments.py tests/test_gpu_multi_device.py -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=6 step c3 300 python tools/bench_c3.py
TAILN=8 step scale 300 python tools/enc_scaling.py
TAILN=1 step bench 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
python3 -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['stage_ms_isolated'])"
