#!/bin/bash
# GPU box: the whole -m gpu suite, C3, and one short bench run (no CPU baseline).
source tools/gpu_step.sh
TAILN=2 step suite 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=2 step c3 300 python3 tools/bench_c3.py
TAILN=1 step bench_short 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
python3 -c "import json; d=json.loads(open('gpurun_out/bench_short.log').read().strip().splitlines()[-1]); r=d['runs']; print(d['value'], r['encode+decode']['median'], r['encode']['median'], d['stage_ms_isolated']['encode'], {k: v.get('ms') for k, v in d.get('c3', {}).items() if isinstance(v, dict)})"
