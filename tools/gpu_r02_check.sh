#!/bin/bash
# GPU box, round 2: the new encode-path parity (segments, pipeline, bench
# configuration), the full -m gpu suite, smoke, one bench line and a kernel
# trace of the bench.  Each GPU step has its own limit; the first failure ends it.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -60 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-3} gpurun_out/$name.log
}
step new 400 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_encode.py tests/test_gpu_bench_config.py -x -q -m gpu --timeout 300 --timeout-method thread
step gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 step bench 600 python bench.py --steps 10 --warmup 3
TAILN=30 step trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
find gpurun_out/prof_r02 -name "*kernel_stats.csv" | head -3
