#!/bin/bash
# GPU box: encoder experiment A/B.  For each tag: webp_amd/libwebpgpu_<tag>.so
# (plain) and webp_amd/libwebpgpu_<tag>_stamps.so (phase stamps, optional).
#   bash tools/gpu_enc_exp.sh base new ...
# Parity of the LAST tag's plain build runs first (encoder + bench-config
# tests); then per tag: one-frame noise / gradient RD launch, the 64-frame mix
# launch, and the stamped per-phase cycles on noise and mix.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -30 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
last=${@: -1}
if [ -z "$NOTEST" ]; then
  WEBPGPU_LIB=webp_amd/libwebpgpu_$last.so step parity 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_bench_config.py -x -q -m gpu --timeout 300 --timeout-method thread
fi
for tag in "$@"; do
  echo "== $tag"
  WEBPGPU_LIB=webp_amd/libwebpgpu_$tag.so TAILN=3 step time_$tag 300 python tools/enc_exp_time.py
  if [ -f webp_amd/libwebpgpu_${tag}_stamps.so ] && [ -z "$NOSTAMP" ]; then
    for c in noise mix; do
      WEBPGPU_LIB=webp_amd/libwebpgpu_${tag}_stamps.so CONTENT=$c TAILN=1 step ph_${tag}_$c 300 python tools/debug_enc_phases.py
    done
  fi
done
