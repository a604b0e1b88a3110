#!/bin/bash
# GPU box: one bench line (with the CPU baseline) then the rocprofv3 passes of
# tools/profile.sh.  Each GPU step has its own limit; the first failure ends it.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 1500 bash tools/profile.sh > gpurun_out/profile.log 2>&1 || { echo "profile failed"; tail -30 gpurun_out/profile.log; exit 1; }
tail -60 gpurun_out/profile.log
