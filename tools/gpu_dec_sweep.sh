#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in default sw2r8 sw8r8 sw4r4 sw4r16 sw8r4 default; do
  if [ $n = default ]; then L=webp_amd/libwebpgpu.so; else L=webp_amd/libwebpgpu_$n.so; fi
  WEBPGPU_LIB=$L C3_ONLY=1 REPS=9 timeout -k 10 120 python tools/bench_c3.py > gpurun_out/dec_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/dec_$n.log; exit 1; }
  echo "$n $(grep 'decode 1x' gpurun_out/dec_$n.log)"
done
