#!/bin/bash
# GPU box: WRITE_SIZE of k_decode_bands per store site.
# One WRITE_SIZE pass of tools/dec_write_sites.py (the bench batch's decode,
# alone) per build: the default library and libwebpgpu_skipw<mask>.so with
# store sites dropped (decode.hip WG_DEC_SKIPW).  Summary:
# gpurun_out/decwrite/summary.json.
source tools/gpu_step.sh
OUT=gpurun_out/decwrite; mkdir -p $OUT
for m in 0 ${MASKS:-1 2 4 8 16 32 63}; do
  if [ $m = 0 ]; then lib=webp_amd/libwebpgpu.so; else lib=webp_amd/libwebpgpu_skipw$m.so; fi
  WEBPGPU_LIB=$lib step dw_$m 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/m$m -o run -- python3 tools/dec_write_sites.py
  python3 tools/pmc_summary.py --any-json $OUT/m$m.json $(find $OUT/m$m -name "*counter_collection.csv") > /dev/null || exit 1
done
python3 - <<'PY'
import json, glob, os
res = {}
for f in glob.glob("gpurun_out/decwrite/m*.json"):
    d = json.load(open(f)).get("k_decode_bands")
    if d:
        res[os.path.basename(f)[1:-5]] = d["WRITE_SIZE"] * 1024
json.dump(res, open("gpurun_out/decwrite/raw.json", "w"), indent=1)
PY
python3 tools/dec_write_sites.py --summarize $OUT/raw.json $OUT/summary.json
