#!/bin/bash
# GPU box: two SQ counter passes over C3 (tools/bench_c3.py) (tools/bench_c3.py),
# each its own rocprofv3 run, summarised for the split decoder (k_decode_split)
# into gpurun_out/c3_pmc/summary.json (tools/pmc_summary.py).
OUT=gpurun_out/c3_pmc; mkdir -p $OUT && export TMPDIR=/tmp
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 tools/bench_c3.py > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  python3 tools/pmc_summary.py --any-json $OUT/$name.json $(find $OUT/$name -name "*counter_collection.csv") > /dev/null || exit 1
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY
pass sq2 SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY
python3 - <<'PY'
import json
out = {}
for n in ("sq1", "sq2"):
    for k, v in json.load(open(f"gpurun_out/c3_pmc/{n}.json")).items():
        if "k_decode_split" in k:
            out.setdefault(k, {}).update(v)
json.dump(out, open("gpurun_out/c3_pmc/summary.json", "w"), indent=1)
for k, v in out.items():
    print(k, json.dumps(v))
PY
