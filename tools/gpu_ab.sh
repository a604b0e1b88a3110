#!/bin/bash
# GPU box: parity first (FULL=1: the whole -m gpu suite + smoke; else the
# encoder tests), then an A/B over library variants: encoder batch scaling and
# alternating bench lines (no CPU baseline), then the row timeline when
# webp_amd/libwebpgpu_rowtimes.so exists.
#   VARIANTS="new=webp_amd/libwebpgpu.so prev=webp_amd/libwebpgpu_prev.so"
#   ROUNDS (2), BATCHES (1,16,64), STEPS (20)
source tools/gpu_step.sh
VARIANTS=${VARIANTS:-"new=webp_amd/libwebpgpu.so prev=webp_amd/libwebpgpu_prev.so"}
if [ -n "$FULL" ]; then
  step gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
else
  step enc 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_bench_config.py -x -q -m gpu --timeout 300 --timeout-method thread
fi
for v in $VARIANTS; do
  BATCHES=${BATCHES:-1,16,64} WEBPGPU_LIB=${v#*=} TAILN=3 step scale_${v%%=*} 300 python tools/enc_scaling.py
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    WEBPGPU_LIB=${v#*=} TAILN=0 step bench_${v%%=*}$r 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline
  done
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    f=bench_${v%%=*}$r
    python3 -c "import json; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', round(d['value']), d['runs']['encode+decode']['median'], d['runs']['encode']['median'], d['ms_per_step'], d['stage_ms_isolated']['encode'])"
  done
done
if [ -f webp_amd/libwebpgpu_rowtimes.so ]; then
  WEBPGPU_LIB=webp_amd/libwebpgpu_rowtimes.so TAILN=8 step timeline 300 python tools/enc_timeline.py
fi
true
