#!/bin/bash
# GPU box: bench.py with 2-5 batches in flight (--slots), alternating; one line per run.
mkdir -p gpurun_out
for s in 3 4 5 2 3 4 5; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --runs 6 --slots $s > gpurun_out/sl_$s.log 2>&1 || { echo "slots $s failed"; tail -5 gpurun_out/sl_$s.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/sl_$s.log') if l.startswith('{')][-1]); print('slots', $s, d['value'], d['runs']['encode+decode']['median'])"
done
