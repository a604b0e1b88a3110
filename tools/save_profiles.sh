#!/bin/bash
# Copy the judged summaries out of gpurun_out/ (scratch) into profiles/ (tracked).
# usage: tools/save_profiles.sh <tag>   e.g. r01
set -e
TAG=${1:?tag}
P=gpurun_out/prof
cp $P/trace/run_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
[ -f $P/trace_iso/run_kernel_stats.csv ] && cp $P/trace_iso/run_kernel_stats.csv profiles/${TAG}_kernel_stats_isolated.csv
cp $P/pmc_traffic.json profiles/${TAG}_pmc_traffic.json
cp $P/pmc_traffic.json profiles/pmc_traffic.json
[ -f $P/pmc_valu.json ] && cp $P/pmc_valu.json profiles/${TAG}_pmc_valu.json && cp $P/pmc_valu.json profiles/pmc_valu.json
python3 tools/pmc_summary.py $(find $P/fetch $P/write -name "*counter_collection.csv") > profiles/${TAG}_pmc_summary.txt
[ -f gpurun_out/bench.log ] && tail -1 gpurun_out/bench.log > profiles/${TAG}_bench.json
ls -la profiles
