#!/bin/bash
# GPU box (round 5 experiments): the one-round I16 trellis (encoder parity
# tests + isolated-launch A/B against libwebpgpu_i16r3.so, the three-round
# build), then k_decode_bands with non-temporal frame stores
# (libwebpgpu_ntst.so): WRITE_SIZE and the bench batch's decode time, A/B.
source tools/gpu_step.sh
TESTS="tests/test_gpu_encode.py tests/test_gpu_bench_config.py" VARS=i16r3 ROUNDS=3 bash tools/gpu_enc_ab.sh > gpurun_out/ab_i16.log 2>&1 || { tail -20 gpurun_out/ab_i16.log; exit 1; }
cat gpurun_out/ab_i16.log
WEBPGPU_LIB=webp_amd/libwebpgpu_ntst.so step dec_nt_w 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/decnt -o run -- python3 tools/dec_write_sites.py
python3 tools/pmc_summary.py --any-json gpurun_out/decnt.json $(find gpurun_out/decnt -name "*counter_collection.csv") | grep -A2 k_decode_bands
for i in 1 2; do
  LAUNCHES=9 step dec_t_def_$i 120 python3 tools/dec_write_sites.py
  WEBPGPU_LIB=webp_amd/libwebpgpu_ntst.so LAUNCHES=9 step dec_t_nt_$i 120 python3 tools/dec_write_sites.py
done
