#!/bin/bash
# GPU box: plane SSIM parity tests, C5 timing of plane SSIM for the wave
# group sizes in $SSIM_GROUPS (WG_SSIM_GROUP), and one SQ counter pass.
mkdir -p gpurun_out/sp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_multi_device.py tests/test_gpu_frames.py -x -q -m gpu --timeout 300 --timeout-method thread -k "ssim" > gpurun_out/ssimt.log 2>&1 || { tail -30 gpurun_out/ssimt.log; exit 1; }
tail -1 gpurun_out/ssimt.log
for g in ${SSIM_GROUPS:-2}; do
  WG_SSIM_GROUP=$g timeout -k 10 300 python tools/bench_c5.py > gpurun_out/c5_$g.log 2>&1 || exit 1
  echo "group $g: $(tail -1 gpurun_out/c5_$g.log | python3 -c "import json,sys; print(json.load(sys.stdin)['stages']['plane_ssim'])")"
done
if [ -n "$PMC" ]; then
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sp/sq -o run -- python3 tools/bench_c5.py > gpurun_out/sp/sq.log 2>&1
python3 tools/pmc_summary.py $(find gpurun_out/sp/sq -name "*counter_collection.csv") | grep "k_plane_ssim"
fi
