#!/bin/bash
# GPU box: alpha-plane + rescaler parity tests, then the aux stage bench.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_alpha.py tests/test_rescale.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/alpha.log 2>&1 || { echo "alpha tests failed"; tail -40 gpurun_out/alpha.log; exit 1; }
tail -3 gpurun_out/alpha.log
timeout -k 10 300 python tools/bench_aux.py > gpurun_out/aux.log 2>&1 || { echo "aux bench failed"; tail -20 gpurun_out/aux.log; exit 1; }
tail -1 gpurun_out/aux.log
