#!/bin/bash
# GPU box: decode + alpha/rescaler parity, smoke, then C3 / aux / main bench.
# Each GPU step has its own limit; the first failure ends the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-3} gpurun_out/$name.log
}
step decode 300 python -u -m pytest tests/test_gpu_frames.py -x -q -m gpu -k decode --timeout 120 --timeout-method thread
step alpha 300 python -u -m pytest tests/test_alpha.py tests/test_rescale.py -x -q -m gpu --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 step c3 300 python tools/bench_c3.py
TAILN=1 step aux 300 python tools/bench_aux.py
TAILN=1 step bench 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
