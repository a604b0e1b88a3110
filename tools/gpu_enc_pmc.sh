#!/bin/bash
# GPU box: SQ counter passes over one 64 x 1080p k_encode_rows launch
# (tools/enc_scaling.py, BATCHES=64): LDS array cycles and bank conflicts,
# instruction mix, waits.  Each pass its own run (<= 8 SQ counters).
source tools/gpu_step.sh
OUT=gpurun_out/encpmc; mkdir -p $OUT
export BATCHES=64
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
run_pass() { local name=$1; shift
  step pmc_$name 180 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 tools/enc_scaling.py
}
run_pass lds SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY
run_pass mix SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES
python3 tools/pmc_summary.py --any-json $OUT/enc_sq.json $(find $OUT/lds $OUT/mix -name "*counter_collection.csv") > $OUT/summary.log
python3 -c "import json; d=json.load(open('$OUT/enc_sq.json'))['k_encode_rows']; print(json.dumps(d, indent=0))"
