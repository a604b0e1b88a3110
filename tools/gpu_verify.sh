#!/bin/bash
# GPU-box check of the current tree: parity tests, smoke, one bench line.
# Each GPU step has its own time limit; the first failure ends the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
