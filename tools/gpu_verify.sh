#!/bin/bash
# GPU box: the whole -m gpu suite on the default build, then the C5 and aux
# stage times, then the split decoder's per-phase cycles on C3's real stream
# (stamped build).
source tools/gpu_step.sh
TAILN=2 step suite 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=1 step c5 300 python3 tools/bench_c5.py
TAILN=3 step aux 300 python3 tools/bench_aux.py
TAILN=2 step c3 300 python3 tools/bench_c3.py
TAILN=2 step dec_phases 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so REAL=1 python -u tools/debug_split_phases.py
