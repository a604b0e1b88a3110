#!/bin/bash
# GPU box: the -m gpu suite, smoke, one bench line (no CPU baseline unless CPU=1)
# and the counter calibration passes.  Each step has its own limit; the first
# failure ends the call.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 step bench 600 python bench.py --steps 20 --warmup 5 ${BENCH_EXTRA:---no-cpu-baseline}
if [ -n "$CAL" ]; then
  OUT=gpurun_out/prof; mkdir -p $OUT
  step cal_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_fetch -o run -- python3 tools/fetch_calib.py
  step cal_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cal_write -o run -- python3 tools/fetch_calib.py
  TAILN=60 step cal_sum 60 python3 tools/fetch_calib.py --summarize $OUT/fetch_calibration.json $(find $OUT/cal_fetch $OUT/cal_write -name "*counter_collection.csv")
fi
if [ -n "$C3" ]; then TAILN=8 step c3 300 python tools/bench_c3.py; fi
