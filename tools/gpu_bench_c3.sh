#!/bin/bash
# GPU box: the bench line (no CPU baseline) and the C2 / C3 stage timings
source tools/gpu_step.sh
TAILN=1 step bench 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
TAILN=8 step c3 300 python tools/bench_c3.py
true
