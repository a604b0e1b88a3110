#!/bin/bash
# encoder parity tests + per-content phase cycles (stamped build) on the GPU box
set -e
timeout -k 10 300 python -m pytest tests/test_gpu_encode.py -x -q -m gpu > gpurun_out/pytest_enc.log 2>&1 || { tail -30 gpurun_out/pytest_enc.log; exit 1; }
tail -2 gpurun_out/pytest_enc.log
bash tools/gpu_enc_phases.sh > gpurun_out/phases.log 2>&1
grep -v amdgpu.ids gpurun_out/phases.log
