#!/bin/bash
# Streaming kernels (import / analysis / upsample) alone: kernel trace + SQ and traffic PMC passes.
export TMPDIR=/tmp
OUT=gpurun_out/sprof
mkdir -p $OUT
export STREAM_ONLY=1 REPS=${REPS:-5}
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/bench_stages.py > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 tools/bench_stages.py > $OUT/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 tools/bench_stages.py > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 tools/bench_stages.py > $OUT/write.log 2>&1 || exit 1
python3 tools/pmc_summary.py $(find $OUT/sq $OUT/fetch $OUT/write -name "*counter_collection.csv")
grep -h "k_" $(find $OUT/trace -name "*kernel_stats.csv") | cut -c1-160
