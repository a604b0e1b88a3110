#!/bin/bash
source tools/gpu_step.sh
for v in "" _upd10 _upd14; do
  WEBPGPU_LIB=webp_amd/libwebpgpu$v.so TAILN=1 step c5$v 300 python tools/bench_c5.py
done
true
