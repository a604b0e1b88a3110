#!/bin/bash
# GPU box: per-phase cycles of k_encode_rows (stamped build) for the given
# contents at the bench batch, plus C2 / C3 stage timings (tools/bench_c3.py).
source tools/gpu_step.sh
for c in ${CONTENTS:-mix noise}; do
  WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so CONTENT=$c TAILN=20 step phases_$c 300 python tools/debug_enc_phases.py
done
[ -n "$NOC3" ] || TAILN=8 step c3 300 python tools/bench_c3.py
true
