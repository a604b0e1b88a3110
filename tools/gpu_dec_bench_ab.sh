#!/bin/bash
# GPU box: the decoder tests on the library, then bench.py on the library and
# the variant $B (webp_amd/libwebpgpu_$B.so), alternating twice; prints the
# bench value, the whole-path / decode-side medians and the isolated decode.
source tools/gpu_step.sh
step decb_tests 400 python -u -m pytest tests/test_c3_real.py tests/test_gpu_frames.py tests/test_reference_testdata.py tests/test_gpu_bench_config.py -x -q -m gpu --timeout 200 --timeout-method thread
for r in 1 2; do
  for v in default $B; do
    lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
    WEBPGPU_LIB=$lib TAILN=0 step decb_${v}_$r 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c3c5
    echo "$r $v $(tail -1 gpurun_out/decb_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["runs"]; print(d["value"], r["encode+decode"]["median"], r["decode"]["median"], d["stage_ms_isolated"]["decode"])')"
  done
done
