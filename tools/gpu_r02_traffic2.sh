#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log; }
step dec 600 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_bench_config.py -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=1 step c3 300 python tools/bench_c3.py
step fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/tr2/fetch -o run -- python3 bench.py --steps 2 --warmup 1 --slots 1 --no-cpu-baseline --iso-steps 1
step write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/tr2/write -o run -- python3 bench.py --steps 2 --warmup 1 --slots 1 --no-cpu-baseline --iso-steps 1
python3 tools/pmc_summary.py $(find gpurun_out/tr2 -name "*counter_collection.csv") | tee gpurun_out/tr2_summary.txt
bash tools/gpu_exp_write.sh
