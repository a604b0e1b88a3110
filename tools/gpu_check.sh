#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel stats.
# Every GPU step has its own time limit; any failure ends the script.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
cat gpurun_out/bench.log
timeout -k 10 1500 bash tools/profile.sh > gpurun_out/profile.log 2>&1 && tail -30 gpurun_out/profile.log
