#!/bin/bash
# GPU box: the whole -m gpu suite on the library, then the library against
# the variant $B (webp_amd/libwebpgpu_$B.so), alternating twice: C5 stages
# (VP8L inverse, SharpYUV), C3, the alpha unfilter / estimate stages and the
# bench's encoder (isolated launch, medians).
source tools/gpu_step.sh
step suite 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  for v in default $B; do
    lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
    WEBPGPU_LIB=$lib TAILN=0 step all_c5_${v}_$r 200 python3 tools/bench_c5.py
    WEBPGPU_LIB=$lib TAILN=0 step all_c3_${v}_$r 200 python3 tools/bench_c3.py
    WEBPGPU_LIB=$lib TAILN=0 step all_aux_${v}_$r 200 python3 tools/bench_aux.py
    WEBPGPU_LIB=$lib TAILN=0 step all_enc_${v}_$r 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c3c5
    python3 - $v $r <<'PY'
import json, sys
v, r = sys.argv[1], sys.argv[2]
last = lambda n: json.loads(open(f"gpurun_out/all_{n}_{v}_{r}.log").read().strip().splitlines()[-1])
c5 = last("c5")["stages"]; aux = last("aux")["stages"]; e = last("enc")
c3 = [l for l in open(f"gpurun_out/all_c3_{v}_{r}.log") if "C3 real" in l][0].split("reconstruct+filter ")[1].split(" ms")[0]
print(r, v, "inverse", round(c5["inverse_predictor"]["ms"], 3), "sharpyuv", round(c5["sharpyuv"]["ms"], 3), "c3", c3,
      "unfilter_gradient", aux["unfilter_gradient"]["ms"], "estimate", aux["estimate_filter+colors"]["ms"],
      "bench", e["value"], e["runs"]["encode+decode"]["median"], "enc_iso", e["stage_ms_isolated"]["encode"])
PY
  done
done
