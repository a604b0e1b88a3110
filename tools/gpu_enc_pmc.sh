#!/bin/bash
# GPU box: instruction-cache and wait counters of k_encode_rows (B=64 mixed, one launch set).
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
export BATCHES=64
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc/ic -o run -- python3 tools/enc_scaling.py > gpurun_out/pmc/ic.log 2>&1 || { echo "ic pass failed"; tail -20 gpurun_out/pmc/ic.log; exit 1; }
python3 tools/pmc_summary.py $(find gpurun_out/pmc/ic -name "*counter_collection.csv") | grep -i "k_encode\|Kernel\|counter" | head -20
