#!/bin/bash
# GPU box: decode parity on the current build, then tools/bench_dec_shapes.py under library variants.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -x -q -m gpu -k "decode" --timeout 120 --timeout-method thread > gpurun_out/dv_tests.log 2>&1 || { tail -30 gpurun_out/dv_tests.log; exit 1; }
tail -1 gpurun_out/dv_tests.log
for tag in "$@"; do
  for lib in webp_amd/libwebpgpu_$tag.so; do
    WEBPGPU_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_frames.py -x -q -m gpu -k "decode_frames or bitstreams" --timeout 120 --timeout-method thread > gpurun_out/dv_t_$tag.log 2>&1 || { echo "$tag parity failed"; tail -20 gpurun_out/dv_t_$tag.log; exit 1; }
    echo "== $tag $(tail -1 gpurun_out/dv_t_$tag.log)"
    WEBPGPU_LIB=$lib timeout -k 10 200 python tools/bench_dec_shapes.py > gpurun_out/dv_$tag.log 2>&1 || { echo "$tag failed"; tail -20 gpurun_out/dv_$tag.log; exit 1; }
    grep MBs gpurun_out/dv_$tag.log | tr '\n' ';'; echo
  done
done
