#!/bin/bash
# GPU box: the bench line at 1..N batches in flight (SLOTS="1 2 3 4").
mkdir -p gpurun_out
for s in ${SLOTS:-1 2 3}; do
timeout -k 10 300 python bench.py --steps 12 --warmup 3 --slots $s --no-cpu-baseline > gpurun_out/slots$s.log 2>&1 || { echo "bench slots=$s failed"; tail -20 gpurun_out/slots$s.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/slots$s.log').read().strip().splitlines()[-1]);print($s,d['value'],d['ms_per_step'],d['stage_ms_overlapped'])"
done
