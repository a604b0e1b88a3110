#!/bin/bash
# GPU box: k_decode_bands HBM bytes (separate FETCH_SIZE / WRITE_SIZE passes over
# the 64 x 1080p decode batch) and C3 time, for the default build and the
# variants named in $LIBS (webp_amd/libwebpgpu_<name>.so).
mkdir -p gpurun_out/dec
export TMPDIR=/tmp
for v in default ${LIBS:-}; do
  if [ $v = default ]; then L=webp_amd/libwebpgpu.so; else L=webp_amd/libwebpgpu_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    WEBPGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/dec/$v/$c -o run -- python3 tools/decode_once.py > gpurun_out/dec/$v_$c.log 2>&1 || { echo "$v $c failed"; exit 1; }
  done
  echo "== $v"; python3 tools/pmc_summary.py $(find gpurun_out/dec/$v -name "*counter_collection.csv") | grep k_decode
  WEBPGPU_LIB=$L timeout -k 10 120 python3 tools/bench_c3.py 2>&1 | grep "^decode" || exit 1
done
