#!/bin/bash
# Encoder iteration on the GPU box: parity tests, then timing on the bench's
# frame mix (plain build) and per-phase cycles (stamped build).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_lossless.py -x -q -m gpu --timeout 120 --timeout-method thread -k "encode" > gpurun_out/enc_t.log 2>&1 || { echo FAIL; tail -40 gpurun_out/enc_t.log; exit 1; }
tail -1 gpurun_out/enc_t.log
CONTENT=mix timeout -k 10 200 python tools/debug_enc_phases.py 
CONTENT=mix WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so timeout -k 10 200 python tools/debug_enc_phases.py
