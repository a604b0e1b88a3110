#!/bin/bash
# GPU box: alternating bench.py runs of the default build with and without the
# extra arguments in $B (e.g. B="--no-split"), $N rounds each, one line per run.
mkdir -p gpurun_out
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --runs 0 "$@" > gpurun_out/ab_$tag.log 2>&1 || { tail -20 gpurun_out/ab_$tag.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$tag.log').read().splitlines()[-1]); print('$tag', d['value'], {k: round(v, 2) for k, v in d['stage_ms_overlapped'].items()})"
}
for i in $(seq ${N:-2}); do
  run A || exit 1
  run B $B || exit 1
done
