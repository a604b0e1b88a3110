#!/bin/bash
# GPU box: VP8L ResidualImage kernels -- parity (tests/test_gpu_lossless.py,
# test_gpu_shard.py) and C5 stage times (tools/bench_c5.py) with the tile
# selection variant WG_VP8L_SELECT = 2 (q2) and 3 (q3, the default), twice.
source tools/gpu_step.sh
TAILN=3 step c5sel_tests 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_lossless.py tests/test_gpu_shard.py
for i in 1 2; do
  for v in 2 3; do
    WG_VP8L_SELECT=$v TAILN=0 step c5sel_${v}_$i 300 python3 tools/bench_c5.py
    echo "$i select=$v $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/c5sel_${v}_$i.log').read().strip().splitlines()[-1]); print(d['stages']['residual_image'])")"
  done
done
