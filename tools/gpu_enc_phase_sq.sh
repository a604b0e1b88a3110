#!/bin/bash
# GPU box: per-phase SQ counters of k_encode_rows.  One
# pass of 8 SQ counters over one 64 x 1080p launch series (tools/enc_scaling.py,
# BATCHES=64) for the default library and for each phase-repeat build
# (webp_amd/libwebpgpu_rep<PHASE>.so, -DWG_EXP_REP_<PHASE>=2: that phase runs
# twice per macroblock, outputs unchanged); tools/enc_phase_sq.py differences
# them into per-phase cycles, VALU instructions, active lanes, LDS bank
# conflicts and waits.  Build the variants first (make -C webp_amd variant ...,
# see tools/enc_phase_sq.py --build).
source tools/gpu_step.sh
OUT=gpurun_out/encphase; mkdir -p $OUT
export BATCHES=64
CTRS="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY"
for v in base ${PHASES:-RD I4 PRE CAND PREP DP FIN}; do
  if [ $v = base ]; then lib=webp_amd/libwebpgpu.so; else lib=webp_amd/libwebpgpu_rep$v.so; fi
  WEBPGPU_LIB=$lib TAILN=1 step sq_$v 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/$v -o run -- python3 tools/enc_scaling.py
  WEBPGPU_LIB=$lib timeout -k 10 120 python3 tools/enc_phase_sq.py --hash >> $OUT/hashes.txt || exit 1
  python3 tools/pmc_summary.py --any-json $OUT/sq_$v.json $(find $OUT/$v -name "*counter_collection.csv") > /dev/null
done
cat $OUT/hashes.txt
python3 tools/enc_phase_sq.py $OUT $OUT/enc_phase_sq.json
