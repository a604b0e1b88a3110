#!/bin/bash
# GPU box: tools/bench_c5.py on the library and the variants $VARIANTS
# (webp_amd/libwebpgpu_<v>.so), alternating twice, after each variant's
# lossless inverse tests; prints the VP8L inverse time of each run.
source tools/gpu_step.sh
for v in $VARIANTS; do
  TAILN=1 step c5ab_test_$v 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_$v.so python -u -m pytest tests/test_gpu_lossless.py -x -q -m gpu -k "inverse or c5" --timeout 200 --timeout-method thread
done
for i in 1 2; do
  for v in default $VARIANTS; do
    lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
    WEBPGPU_LIB=$lib TAILN=0 step c5ab_${v}_$i 300 python3 tools/bench_c5.py
    echo "$i $v $(python3 -c "import json; d=json.loads(open('gpurun_out/c5ab_${v}_$i.log').read().strip().splitlines()[-1]); print(d['stages']['inverse_predictor']['ms'])")"
  done
done
