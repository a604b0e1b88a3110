#!/bin/bash
# GPU box: an encoder variant $B (webp_amd/libwebpgpu_$B.so) against the
# library: the encoder's GPU tests on the variant, the isolated 64 x 1080p
# launch and the bench (alternating twice), and the variant's stamped phases
# ($ST build) beside the library's.
source tools/gpu_step.sh
TAILN=1 step encab_tests 600 env WEBPGPU_LIB=webp_amd/libwebpgpu_$B.so python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_bench_config.py tests/test_encode_quality.py -x -q -m gpu --timeout 300 --timeout-method thread
for r in 1 2; do
  TAILN=0 step ab_a$r 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c3c5
  WEBPGPU_LIB=webp_amd/libwebpgpu_$B.so TAILN=0 step ab_b$r 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c3c5
done
for f in gpurun_out/ab_[ab][12].log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["runs"]; print(d["value"], r["encode+decode"]["median"], r["encode"]["median"], r["decode"]["median"], d["stage_ms_isolated"]["encode"])')"; done
if [ -n "$ST" ]; then
  TAILN=2 step encab_stamps_default 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so CONTENT=bench python -u tools/debug_enc_phases.py
  TAILN=2 step encab_stamps_$B 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_$ST.so CONTENT=bench python -u tools/debug_enc_phases.py
fi
true
