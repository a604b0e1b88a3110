#!/bin/bash
# Sourced by gpurun commands: step NAME LIMIT CMD... runs CMD under its own
# time limit with output in gpurun_out/NAME.log, prints the log's tail
# (TAILN lines), and ends the whole call on the first failure.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 gpurun_out/$name.log; exit 1; }
  tail -${TAILN:-2} gpurun_out/$name.log
}
