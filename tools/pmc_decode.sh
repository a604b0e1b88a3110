#!/bin/bash
# Instruction-mix counters for the decode kernel (separate --pmc passes, kernel trace only).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_dec
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $OUT/a -o run -- python3 tools/decode_once.py > $OUT/a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/b -o run -- python3 tools/decode_once.py > $OUT/b.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD --output-format csv -d $OUT/c -o run -- python3 tools/decode_once.py > $OUT/c.log 2>&1
find $OUT -name "*counter_collection.csv" | while read f; do python3 tools/pmc_summary.py "$f"; done
