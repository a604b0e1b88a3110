#!/bin/bash
# GPU box: the bench line with 2 / 3 (default) / 4 batches in flight,
# alternating twice (value = contract mean, and the whole-path runs median).
source tools/gpu_step.sh
for i in 1 2; do
  for n in 2 3 4; do
    TAILN=0 step slots_${n}_$i 300 python3 bench.py --slots $n --no-cpu-baseline --iso-steps 1
    echo "$i slots=$n $(python3 -c "import json; d=json.loads(open('gpurun_out/slots_${n}_$i.log').read().strip().splitlines()[-1]); print(d['value'], d['runs']['encode+decode']['median'])")"
  done
done
