#!/bin/bash
# GPU box: C3 (one 4096^2 decode) and 4 / 16-image decode timings for decode
# builds with other band sizes / R->F ring depths (webp_amd/libwebpgpu_swXrY.so,
# -DWG_DEC_SW / -DWG_DEC_RING_M), alternating with the default build.
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in ${VARIANTS:-default sw4r16 sw4r4 default sw4r16 sw4r4}; do
  if [ $n = default ]; then L=webp_amd/libwebpgpu.so; else L=webp_amd/libwebpgpu_$n.so; fi
  WEBPGPU_LIB=$L C3_ONLY=${C3_ONLY:-1} REPS=9 timeout -k 10 120 python tools/bench_c3.py > gpurun_out/dec_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/dec_$n.log; exit 1; }
  grep 'decode ' gpurun_out/dec_$n.log | sed "s/^/$n /"
done
