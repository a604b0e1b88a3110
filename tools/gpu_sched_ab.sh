#!/bin/bash
# GPU box: A/B of a library variant $B (webp_amd/libwebpgpu_$B.so) against the
# library on the bench (whole path, alternating twice, after the variant's
# encoder tests), the variant's row timeline ($B_RT build, tools/enc_timeline.py),
# and tools/bench_c5.py default vs $C5 alternating twice.
source tools/gpu_step.sh
B=${B:-slk}
TAILN=1 step sched_tests 600 env WEBPGPU_LIB=webp_amd/libwebpgpu_$B.so python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_bench_config.py -x -q -m gpu -k "not row_schedule_table" --timeout 300 --timeout-method thread
for r in 1 2; do
  TAILN=0 step ab_a$r 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c3c5
  WEBPGPU_LIB=webp_amd/libwebpgpu_$B.so TAILN=0 step ab_b$r 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c3c5
done
for f in gpurun_out/ab_[ab][12].log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["runs"]; print(d["value"], r["encode+decode"]["median"], r["encode"]["median"], r["decode"]["median"], d["stage_ms_isolated"]["encode"])')"; done
[ -n "$RT" ] && TAILN=12 step enc_timeline_$B 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_$RT.so JSON=gpurun_out/r06_enc_timeline_$B.json python -u tools/enc_timeline.py
if [ -n "$C5" ]; then
  TAILN=1 step c5_test_$C5 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_$C5.so python -u -m pytest tests/test_gpu_lossless.py -x -q -m gpu -k "inverse or c5" --timeout 200 --timeout-method thread
  for i in 1 2; do
    for v in default $C5; do
      lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
      WEBPGPU_LIB=$lib TAILN=0 step c5ab_${v}_$i 300 python3 tools/bench_c5.py
      echo "$i $v $(python3 -c "import json; d=json.loads(open('gpurun_out/c5ab_${v}_$i.log').read().strip().splitlines()[-1]); print(d['stages']['inverse_predictor']['ms'])")"
    done
  done
fi
true
