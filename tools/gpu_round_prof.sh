#!/bin/bash
# GPU box: rocprofv3 passes of tools/profile.sh (kernel trace + FETCH/WRITE +
# SQ), their per-kernel JSON summaries put where bench.py reads them, then the
# bench line itself (with the CPU baseline).  First failure ends it.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 bash tools/profile.sh > gpurun_out/profile.log 2>&1 || { echo "profile failed"; tail -30 gpurun_out/profile.log; exit 1; }
cp gpurun_out/prof/pmc_traffic.json profiles/pmc_traffic.json
cp gpurun_out/prof/pmc_valu.json profiles/pmc_valu.json
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
grep -h "k_" $(find gpurun_out/prof/trace -name "*kernel_stats.csv") | cut -c1-150
