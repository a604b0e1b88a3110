#!/bin/bash
# GPU box: kernel trace of a short bench run (which kernels overlap which),
# plus bench variants (--split, --slots 4).
source tools/gpu_step.sh
OUT=gpurun_out/trace; mkdir -p $OUT
step trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --runs 0
TAILN=0 step bench_base 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
TAILN=0 step bench_split 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --split
TAILN=0 step bench_slots4 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --slots 4
for f in bench_base bench_split bench_slots4; do
  python3 -c "import json; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', round(d['value']), d['runs']['encode+decode']['median'], d['runs']['encode']['median'], d['runs']['decode']['median'], d['ms_per_step'])"
done
find $OUT -name "*kernel_trace.csv"
