#!/bin/bash
# GPU box: the suite, C3's phases on the stamped build, and the VP8L inverse
# against the variant $C5 (alternating twice).
source tools/gpu_step.sh
TAILN=2 step suite 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=2 step dec_phases 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so REAL=1 python -u tools/debug_split_phases.py
TAILN=1 step c5_test_$C5 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_$C5.so python -u -m pytest tests/test_gpu_lossless.py -x -q -m gpu -k "inverse or c5" --timeout 200 --timeout-method thread
for i in 1 2; do
  for v in default $C5; do
    lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
    WEBPGPU_LIB=$lib TAILN=0 step c5ab_${v}_$i 300 python3 tools/bench_c5.py
    echo "$i $v $(python3 -c "import json; d=json.loads(open('gpurun_out/c5ab_${v}_$i.log').read().strip().splitlines()[-1]); print(d['stages']['inverse_predictor']['ms'])")"
  done
done
if [ -n "$C3V" ]; then
  for i in 1 2; do
    for v in default $C3V; do
      lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
      WEBPGPU_LIB=$lib TAILN=0 step c3ab_${v}_$i 300 python3 tools/bench_c3.py
      echo "$i $v $(grep -h 'C3 real\|decode 16x' gpurun_out/c3ab_${v}_$i.log | sed 's/.*reconstruct+filter \([0-9.]*\) ms.*/\1/' | tr '\n' ' ')"
    done
  done
fi
