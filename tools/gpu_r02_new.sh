#!/bin/bash
# GPU box: this round's new GPU tests (dithered import, shard bands, C5 sizes).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dither.py tests/test_gpu_shard.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/new2.log 2>&1 || { echo "new2 failed rc=$?"; tail -60 gpurun_out/new2.log; exit 1; }
tail -20 gpurun_out/new2.log
