#!/bin/bash
# GPU box: the encoder's GPU tests on the library, then alternating bench runs
# (no CPU baseline) of the library and of a variant build
# (webp_amd/libwebpgpu_$B.so), e.g. B=prev TESTS="tests/test_gpu_encode.py" bash tools/gpu_lib_ab.sh
source tools/gpu_step.sh
[ -n "$TESTS" ] && TAILN=2 step ab_tests 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $TESTS
for r in 1 2; do
  TAILN=0 step ab_a$r 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
  WEBPGPU_LIB=webp_amd/libwebpgpu_$B.so TAILN=0 step ab_b$r 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
done
for f in gpurun_out/ab_[ab]*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["runs"]; print(d["value"], r["encode+decode"]["median"], r["encode"]["median"], r["decode"]["median"], d["stage_ms_isolated"]["encode"])')"; done
