#!/bin/bash
# GPU box: tools/bench_c5.py against library variants (webp_amd/libwebpgpu_<name>.so,
# built with `make -C webp_amd variant NAME=<name> DEFS=...`), e.g.
# VARIANTS="probe1 probe2" bash tools/gpu_variants_c5.sh
source tools/gpu_step.sh
for v in "" ${VARIANTS:-}; do
  WEBPGPU_LIB=webp_amd/libwebpgpu${v:+_$v}.so TAILN=1 step c5${v:+_$v} 300 python tools/bench_c5.py
done
true
