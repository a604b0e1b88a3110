#!/bin/bash
# GPU box: the C5 / aux walks' parity tests, then their stage timings
# (tools/bench_c5.py, tools/bench_aux.py).
source tools/gpu_step.sh
TAILN=3 step c5_tests 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_sharpyuv.py tests/test_gpu_lossless.py tests/test_vp8l_color.py tests/test_alpha.py
TAILN=1 step c5 300 python tools/bench_c5.py
true
