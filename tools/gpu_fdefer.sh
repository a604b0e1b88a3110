#!/bin/bash
# GPU box: the decoder tests on the library, the whole suite, then C3 on the
# library against webp_amd/libwebpgpu_fprev.so (alternating twice) and one
# short bench run.
source tools/gpu_step.sh
TAILN=2 step dec_tests 300 python -u -m pytest tests/test_c3_real.py tests/test_gpu_frames.py tests/test_reference_testdata.py -x -q -m gpu --timeout 200 --timeout-method thread
TAILN=2 step suite 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
for i in 1 2; do
  for v in default fprev; do
    lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
    WEBPGPU_LIB=$lib TAILN=0 step c3ab_${v}_$i 300 python3 tools/bench_c3.py
    echo "$i $v $(grep -h 'C3 real\|decode 16x' gpurun_out/c3ab_${v}_$i.log | sed 's/.*reconstruct+filter \([0-9.]*\) ms.*/\1/' | tr '\n' ' ')"
  done
done
TAILN=1 step bench_short 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
python3 -c "import json; d=json.loads(open('gpurun_out/bench_short.log').read().strip().splitlines()[-1]); r=d['runs']; print(d['value'], r['encode+decode']['median'], r['encode']['median'], d['stage_ms_isolated']['encode'], d.get('c3'))"
