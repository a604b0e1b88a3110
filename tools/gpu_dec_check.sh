#!/bin/bash
# GPU box: decode-path parity (frames, real C3 bitstream, reference testdata,
# bench configuration), C3 timing, and the k_decode_split WRITE_SIZE pass.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step dec_tests 600 python -u -m pytest tests/test_gpu_frames.py tests/test_c3_real.py tests/test_reference_testdata.py tests/test_capi.py tests/test_gpu_bench_config.py -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=4 step c3 300 python tools/bench_c3.py
OUT=gpurun_out/prof_dec; mkdir -p $OUT
step write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
TAILN=12 step wsum 60 python3 tools/pmc_summary.py $(find $OUT/write -name "*counter_collection.csv")
