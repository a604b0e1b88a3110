#!/bin/bash
# GPU box: time a tool under several library builds (webp_amd/libwebpgpu_<tag>.so):
#   bash tools/gpu_lib_ab.sh "<tool.py>" tag1 tag2 ...
# Parity of the current build runs first (TESTS, default the VP8L tests).
mkdir -p gpurun_out
export TMPDIR=/tmp
TOOL=$1; shift
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_lossless.py tests/test_reference_testdata.py} -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for tag in "$@"; do
  WEBPGPU_LIB=webp_amd/libwebpgpu_$tag.so timeout -k 10 300 python $TOOL > gpurun_out/ab_$tag.log 2>&1 || { echo "$tag failed"; tail -20 gpurun_out/ab_$tag.log; exit 1; }
  echo "== $tag"; tail -${TAILN:-1} gpurun_out/ab_$tag.log
done
