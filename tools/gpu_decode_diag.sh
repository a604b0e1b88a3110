#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so SIZE=4096 BATCH=1 python tools/debug_phases.py > gpurun_out/ph4096.log 2>&1 || { tail -20 gpurun_out/ph4096.log; exit 1; }
cat gpurun_out/ph4096.log | grep -v amdgpu.ids
timeout -k 10 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so BATCH=64 python tools/debug_phases.py > gpurun_out/ph1080.log 2>&1 || { tail -20 gpurun_out/ph1080.log; exit 1; }
cat gpurun_out/ph1080.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --slots 1 --no-cpu-baseline > gpurun_out/b1.log 2>&1 || { tail -20 gpurun_out/b1.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/b1.log').read().strip().splitlines()[-1]);print(d['value'],d['stage_ms'])"
