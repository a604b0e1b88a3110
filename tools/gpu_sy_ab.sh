#!/bin/bash
# GPU box: the SharpYUV GPU tests on the library, the k_sharp_wave timeline
# (libwebpgpu_timelines.so), the lossless inverse tests of the variants
# $VARIANTS (webp_amd/libwebpgpu_<v>.so), then tools/bench_c5.py on the
# library and the variants alternating twice; prints each run's SharpYUV and
# VP8L inverse times.
source tools/gpu_step.sh
step sy_test 300 python -u -m pytest tests/test_sharpyuv.py -x -q -m gpu --timeout 200 --timeout-method thread
WEBPGPU_LIB=webp_amd/libwebpgpu_timelines.so step sy_timeline 120 python3 tools/sharp_timeline.py gpurun_out/sharp_timeline.json
for v in $VARIANTS; do
  TAILN=1 step syab_test_$v 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_$v.so python -u -m pytest tests/test_gpu_lossless.py tests/test_sharpyuv.py -x -q -m gpu -k "inverse or c5 or sharp" --timeout 200 --timeout-method thread
done
for i in 1 2; do
  for v in default $VARIANTS; do
    lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
    WEBPGPU_LIB=$lib TAILN=0 step syab_${v}_$i 300 python3 tools/bench_c5.py
    echo "$i $v $(python3 -c "import json; d=json.loads(open('gpurun_out/syab_${v}_$i.log').read().strip().splitlines()[-1])['stages']; print('sharpyuv', round(d['sharpyuv']['ms'], 3), 'inverse', round(d['inverse_predictor']['ms'], 3))")"
  done
done
