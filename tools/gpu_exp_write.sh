#!/bin/bash
# GPU box: WRITE_SIZE of k_encode_rows with the product lib and two experiment libs.
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" _exp_NO_RECON _exp_NO_MBENC; do
  export WEBPGPU_LIB=webp_amd/libwebpgpu$v.so
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/exp$v -o run -- python3 tools/debug_enc_phases.py > gpurun_out/exp$v.log 2>&1 || { echo "fail $v"; tail -20 gpurun_out/exp$v.log; exit 1; }
  echo "== $v"; python3 tools/pmc_summary.py $(find gpurun_out/exp$v -name "*counter_collection.csv") | grep k_encode
done
