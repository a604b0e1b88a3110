#!/bin/bash
# GPU box: encoder batch time (64 mixed 1080p frames, tools/enc_scaling.py B=64)
# for builds with other row-schedule head starts (webp_amd/libwebpgpu_sN.so,
# -DWG_ENC_SLACK_DIV=N), alternating with the default build.
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in ${VARIANTS:-default s2 s3 s6 default s2 s3 s6}; do
  if [ $n = default ]; then L=webp_amd/libwebpgpu.so; else L=webp_amd/libwebpgpu_$n.so; fi
  WEBPGPU_LIB=$L BATCHES=64 timeout -k 10 120 python tools/enc_scaling.py > gpurun_out/enc_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/enc_$n.log; exit 1; }
  grep 'B=' gpurun_out/enc_$n.log | sed "s/^/$n /"
done
