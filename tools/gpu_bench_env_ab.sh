#!/bin/bash
# GPU box: alternating bench runs (no CPU baseline) with and without an
# environment setting, e.g. ENV_B="WG_DECODE_KERNEL=bands" bash tools/gpu_bench_env_ab.sh
source tools/gpu_step.sh
for r in 1 2; do
  TAILN=0 step ab_a$r 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
  TAILN=0 step ab_b$r 300 env $ENV_B python bench.py --steps 10 --warmup 3 --no-cpu-baseline
done
for f in gpurun_out/ab_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["runs"]; print(d["value"], r["encode+decode"]["median"], r["encode"]["median"], r["decode"]["median"])')"; done
