#!/bin/bash
# GPU box: VP8L parity, then k_vp8l_inverse timing by shape for the current
# build and the variant libraries named in $LIBS (webp_amd/libwebpgpu_<tag>.so)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lossless.py tests/test_reference_testdata.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ll.log 2>&1 || { tail -30 gpurun_out/ll.log; exit 1; }
tail -1 gpurun_out/ll.log
for t in cur $LIBS; do
  lib=webp_amd/libwebpgpu.so; [ "$t" != cur ] && lib=webp_amd/libwebpgpu_$t.so
  echo "== $t"; WEBPGPU_LIB=$lib timeout -k 10 120 python tools/bench_inv.py 2>&1 | grep -v amdgpu.ids || exit 1
done
