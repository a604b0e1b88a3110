#!/bin/bash
# GPU box: VALU lane utilisation of one 64 x 1080p k_encode_rows launch
# (active lanes): SQ_THREAD_CYCLES_VALU (thread-cycles of VALU
# work) over SQ_ACTIVE_INST_VALU (VALU instruction-cycles) = the mean active
# lanes per VALU cycle, beside the instruction counts.  One pass, 5 SQ counters.
source tools/gpu_step.sh
OUT=gpurun_out/enclanes; mkdir -p $OUT
export BATCHES=64
step pmc_lanes 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d $OUT/lanes -o run -- python3 tools/enc_scaling.py
python3 tools/pmc_summary.py --any-json $OUT/enc_lanes.json $(find $OUT/lanes -name "*counter_collection.csv") > $OUT/summary.log
python3 -c "import json; d=json.load(open('$OUT/enc_lanes.json')); [print(k, json.dumps(v)) for k, v in d.items() if 'encode' in k]"
