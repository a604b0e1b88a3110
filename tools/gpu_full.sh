#!/bin/bash
# GPU box, round 2 evidence: the full -m gpu suite, smoke, the bench line (with
# the CPU baseline), C3 / C5 / aux stage timings, encoder batch scaling, and
# the rocprofv3 passes of tools/profile.sh (kernel trace + FETCH / WRITE + SQ).
# Each GPU step has its own limit; the first failure ends it.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log
}
# PART=a: everything but the profiler passes; PART=b: the profiler passes only
# (each fits one gpurun call)
if [ "${PART:-a}" != b ]; then
step gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 step bench 600 python bench.py --steps 10 --warmup 3
TAILN=4 step c3 300 python tools/bench_c3.py
TAILN=1 step c5 300 python tools/bench_c5.py
TAILN=1 step aux 300 python tools/bench_aux.py
TAILN=6 step scale 300 python tools/enc_scaling.py
fi
[ "${PART:-ab}" != a ] && step profile 1500 bash tools/profile.sh
true
