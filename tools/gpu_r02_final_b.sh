#!/bin/bash
# GPU box, round 2 final evidence (part B): encoder batch scaling and the
# rocprofv3 passes of tools/profile.sh (kernel trace + FETCH / WRITE + SQ).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/enc_scaling.py > gpurun_out/scale.log 2>&1 || { echo "scale failed"; tail -30 gpurun_out/scale.log; exit 1; }
tail -6 gpurun_out/scale.log
timeout -k 10 900 bash tools/profile.sh > gpurun_out/profile.log 2>&1 || { echo "profile failed"; tail -30 gpurun_out/profile.log; exit 1; }
tail -5 gpurun_out/profile.log
