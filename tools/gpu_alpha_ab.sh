#!/bin/bash
# GPU box: the alpha tests on the library, then tools/bench_aux.py on the
# library and the variant $B (webp_amd/libwebpgpu_$B.so), alternating twice.
source tools/gpu_step.sh
step alpha_tests 300 python -u -m pytest tests/test_alpha.py tests/test_gpu_shard.py -x -q -m gpu --timeout 200 --timeout-method thread
for r in 1 2; do
  for v in default $B; do
    lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
    WEBPGPU_LIB=$lib TAILN=0 step aab_${v}_$r 200 python3 tools/bench_aux.py
    echo "$r $v $(python3 -c "import json; d=json.loads(open('gpurun_out/aab_${v}_$r.log').read().strip().splitlines()[-1])['stages']; print('unfilter_gradient', d['unfilter_gradient']['ms'], 'estimate', d['estimate_filter+colors']['ms'])")"
  done
done
