#!/bin/bash
# GPU box: encoder parity of the current build, then A/B of the encoder against
# webp_amd/libwebpgpu_prev.so (batch scaling, bench line) and the per-phase cycles
# of the stamped build.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step enc 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_bench_config.py -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=6 step scale_new 300 python tools/enc_scaling.py
WEBPGPU_LIB=webp_amd/libwebpgpu_prev.so TAILN=6 step scale_prev 300 python tools/enc_scaling.py
TAILN=1 step bench_new 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
WEBPGPU_LIB=webp_amd/libwebpgpu_prev.so TAILN=1 step bench_prev 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
TAILN=1 step bench_new2 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
for f in bench_new bench_prev bench_new2; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['stage_ms_isolated']['encode'])"; done
WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so CONTENT=mix TAILN=1 step phases 300 python tools/debug_enc_phases.py
