#!/bin/bash
# GPU box: C3 (tools/bench_c3.py) on the library and the variants $VARIANTS,
# alternating twice, after each variant's decoder tests.
source tools/gpu_step.sh
for v in $VARIANTS; do
  TAILN=1 step c3ab_test_$v 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_$v.so python -u -m pytest tests/test_c3_real.py tests/test_gpu_frames.py -x -q -m gpu --timeout 200 --timeout-method thread
done
for i in 1 2; do
  for v in default $VARIANTS; do
    lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
    WEBPGPU_LIB=$lib TAILN=0 step c3ab_${v}_$i 300 python3 tools/bench_c3.py
    echo "$i $v $(grep -h 'C3 real\|decode 16x' gpurun_out/c3ab_${v}_$i.log | sed 's/.*reconstruct+filter \([0-9.]*\) ms.*/\1/' | tr '\n' ' ')"
  done
done
