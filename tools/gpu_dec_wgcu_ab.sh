source tools/gpu_step.sh
for r in 1 2; do
  for e in "X=0" "WG_DECODE_WG_PER_CU=1" "WG_DECODE_WG_PER_CU=2"; do
    n=$(echo $e | tr '=' '_')
    TAILN=0 step ab_${n}_$r 300 env $e python bench.py --steps 10 --warmup 3 --no-cpu-baseline
  done
done
for f in gpurun_out/ab_*_[12].log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["runs"]; print(d["value"], r["encode+decode"]["median"], r["encode"]["median"], r["decode"]["median"])')"; done
