#!/bin/bash
# GPU box: VP8L inverse at 4096^2 (tools/bench_c5.py) for the default build
# (UPD 6) and the look-ahead variants libwebpgpu_upd<N>.so, alternating twice.
source tools/gpu_step.sh
TAILN=2 step invupd_test 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_upd3.so python -u -m pytest tests/test_gpu_lossless.py -x -q -m gpu -k inverse --timeout 200 --timeout-method thread
for i in 1 2; do
  for v in default 3 4 9; do
    lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_upd$v.so
    WEBPGPU_LIB=$lib TAILN=0 step invupd_${v}_$i 300 python3 tools/bench_c5.py
    echo "$i upd=$v $(python3 -c "import json; d=json.loads(open('gpurun_out/invupd_${v}_$i.log').read().strip().splitlines()[-1]); print(d['stages']['inverse_predictor']['ms'])")"
  done
done
