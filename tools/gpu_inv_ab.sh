#!/bin/bash
# GPU box: tools/bench_c5.py on the library and on the variants $VARIANTS
# (webp_amd/libwebpgpu_<v>.so), alternating twice, after each variant's
# lossless tests; then the encoder's row timeline (libwebpgpu_rowtimes.so)
# and SharpYUV's per-wave timeline (libwebpgpu_timelines.so).
source tools/gpu_step.sh
VARIANTS=${VARIANTS:-invA}
for v in $VARIANTS; do
  TAILN=1 step invab_test_$v 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_$v.so python -u -m pytest tests/test_gpu_lossless.py -x -q -m gpu -k "inverse or c5" --timeout 200 --timeout-method thread
done
TAILN=1 step cc_test 300 python -u -m pytest tests/test_vp8l_color.py -x -q -m gpu --timeout 200 --timeout-method thread
for i in 1 2; do
  for v in default $VARIANTS; do
    lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
    WEBPGPU_LIB=$lib TAILN=0 step c5ab_${v}_$i 300 python3 tools/bench_c5.py
    echo "$i $v $(python3 -c "import json; d=json.loads(open('gpurun_out/c5ab_${v}_$i.log').read().strip().splitlines()[-1]); print({k: round(v['ms'], 4) for k, v in d['stages'].items()})")"
  done
done
TAILN=12 step enc_timeline 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_rowtimes.so JSON=gpurun_out/r06_enc_timeline.json python -u tools/enc_timeline.py
TAILN=2 step sharp_timeline 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_timelines.so python -u tools/sharp_timeline.py gpurun_out/r06_sharp_timeline.json
