#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the bench.
# Results land in gpurun_out/prof; copy the summaries into profiles/ (tools/save_profiles.sh).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="--steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${EXTRA:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
# isolated launches (one batch at a time, as the bench line's stage_ms_isolated /
# roofline.achieved time them): AverageNs of k_encode_rows is the roofline's launch
BATCHES=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_iso -o run -- python3 tools/enc_scaling.py > $OUT/trace_iso.log 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
python3 tools/pmc_summary.py --json $OUT/pmc_traffic.json $(find $OUT/fetch $OUT/write -name "*counter_collection.csv")
# SQ / GRBM pass (8 SQ + 1 GRBM counters, within the per-pass slots): VALU issue
# rate of the latency-bound kernels against the SIMD issue peak.
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
python3 tools/pmc_summary.py --valu-json $OUT/pmc_valu.json $(find $OUT/sq -name "*counter_collection.csv")
# counter calibration on known byte counts (tools/fetch_calib.py; MI355X_MICROARCH.md:
# other access widths than 16-B streams are uncalibrated)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_fetch -o run -- python3 tools/fetch_calib.py > $OUT/cal_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cal_write -o run -- python3 tools/fetch_calib.py > $OUT/cal_write.log 2>&1
python3 tools/fetch_calib.py --summarize $OUT/fetch_calibration.json $(find $OUT/cal_fetch $OUT/cal_write -name "*counter_collection.csv")
find $OUT -name "*.csv"
