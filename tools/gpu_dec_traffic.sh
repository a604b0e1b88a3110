#!/bin/bash
# GPU box: HBM traffic of the decode kernels (separate FETCH_SIZE / WRITE_SIZE
# passes, MI355X_MICROARCH.md's recipe) over the bench batch (k_decode_bands)
# and C3 real (k_decode_split); summaries in gpurun_out/dectraffic/*.json.
source tools/gpu_step.sh
OUT=gpurun_out/dectraffic
mkdir -p $OUT
B="--steps 3 --warmup 1 --runs 0 --iso-steps 1 --no-cpu-baseline --no-gather"
step dt_bw 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/bw -o run -- python3 bench.py $B
step dt_bf 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/bf -o run -- python3 bench.py $B
step dt_cw 300 env C3_ONLY=1 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cw -o run -- python3 tools/bench_c3.py
step dt_cf 300 env C3_ONLY=1 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cf -o run -- python3 tools/bench_c3.py
python3 tools/pmc_summary.py --json $OUT/bench.json $(find $OUT/bw $OUT/bf -name "*counter_collection.csv") > $OUT/bench.txt
python3 tools/pmc_summary.py --json $OUT/c3.json $(find $OUT/cw $OUT/cf -name "*counter_collection.csv") > $OUT/c3.txt
grep -h -E "decode|upsample" $OUT/bench.txt $OUT/c3.txt
