#!/bin/bash
# GPU box: decode parity of the current build (frames, C3 real bitstream,
# reference testdata, bench config), then C3 timing (tools/bench_c3.py) of
# the current build and of webp_amd/libwebpgpu_prev.so, alternating.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -30 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step dec 600 python -u -m pytest tests/test_gpu_frames.py tests/test_c3_real.py tests/test_reference_testdata.py tests/test_gpu_bench_config.py -x -q -m gpu --timeout 300 --timeout-method thread
step dec_bands 300 env WG_DECODE_KERNEL=bands python -u -m pytest tests/test_gpu_frames.py tests/test_reference_testdata.py -x -q -m gpu -k "decode" --timeout 200 --timeout-method thread
for i in 1 2; do
  TAILN=4 step c3_new_$i 300 env C3_ONLY=1 python tools/bench_c3.py
  # other builds to compare: webp_amd/libwebpgpu_prev.so (the last commit) and libwebpgpu_v*.so
  for lib in webp_amd/libwebpgpu_prev.so webp_amd/libwebpgpu_v*.so; do
    [ -f $lib ] || continue
    n=$(basename $lib .so); n=${n#libwebpgpu_}
    WEBPGPU_LIB=$lib TAILN=4 step c3_${n}_$i 300 env C3_ONLY=1 python tools/bench_c3.py
  done
done
