#!/bin/bash
# Decode parity tests, then per-stage timings at several resident-workgroup counts.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -q -m gpu -k "decode or filter" > gpurun_out/pytest_decode.log 2>&1 || { echo "decode tests failed rc=$?"; tail -30 gpurun_out/pytest_decode.log; exit 1; }
tail -2 gpurun_out/pytest_decode.log
timeout -k 10 180 python tools/bench_stages.py
for n in ${WGS:-8 12 16}; do echo "== WG_DECODE_WG_PER_CU=$n"; WG_DECODE_WG_PER_CU=$n DECODE_ONLY=1 timeout -k 10 120 python tools/bench_stages.py; done
