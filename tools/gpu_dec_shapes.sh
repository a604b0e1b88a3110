#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
for k in split bands; do echo "== $k"; WG_DECODE_KERNEL=$k timeout -k 10 200 python tools/bench_dec_shapes.py > gpurun_out/shapes_$k.log 2>&1 || { tail -20 gpurun_out/shapes_$k.log; exit 1; }; grep MBs gpurun_out/shapes_$k.log; done
