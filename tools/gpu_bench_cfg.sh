#!/bin/bash
# GPU box: bench-line A/B over pipeline configurations (CFGS, each a set of
# bench.py flags), ROUNDS alternations; prints mean / median / encode-only.
source tools/gpu_step.sh
IFS=';' read -ra C <<< "${CFGS:-;--split;--slots 4;--split --slots 4}"
for r in $(seq 1 ${ROUNDS:-3}); do
  i=0
  for c in "${C[@]}"; do
    TAILN=0 step bench_c${i}_$r 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --runs 6 $c
    python3 -c "import json; d=json.loads(open('gpurun_out/bench_c${i}_$r.log').read().strip().splitlines()[-1]); print('cfg[$c] r$r', round(d['value']), d['runs']['encode+decode']['median'], d['runs']['encode']['median'], d['ms_per_step'])"
    i=$((i+1))
  done
done
