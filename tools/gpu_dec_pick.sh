source tools/gpu_step.sh
TAILN=2 step gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=1 step bench 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
TAILN=6 step c3 300 python tools/bench_c3.py
WG_DECODE_KERNEL=split TAILN=6 step c3_split 300 python tools/bench_c3.py
true
