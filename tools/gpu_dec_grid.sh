mkdir -p gpurun_out
for i in 1 2; do for g in 0 512 256 128; do
  WG_DECODE_MAX_WG=$g timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --runs 0 > gpurun_out/dg_$g.log 2>&1 || { tail -5 gpurun_out/dg_$g.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/dg_$g.log').read().splitlines()[-1]); print('grid $g', d['value'], d['stage_ms_isolated']['decode'], {k: round(v, 2) for k, v in d['stage_ms_overlapped'].items()})"
done; done
