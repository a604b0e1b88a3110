#!/bin/bash
# GPU box: the multi-device batch entry point and the C-API / encode tests.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi_device.py tests/test_capi.py -x -q -m "gpu or not gpu" --timeout 120 --timeout-method thread > gpurun_out/md.log 2>&1 || { echo "md failed rc=$?"; tail -40 gpurun_out/md.log; exit 1; }
tail -3 gpurun_out/md.log
