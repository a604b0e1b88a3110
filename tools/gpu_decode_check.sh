#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 180 python -m pytest tests -q -m gpu -k decode > gpurun_out/pytest_decode.log 2>&1 || { echo "decode tests failed rc=$?"; tail -30 gpurun_out/pytest_decode.log; exit 1; }
tail -2 gpurun_out/pytest_decode.log
timeout -k 10 180 python tools/bench_stages.py
