#!/bin/bash
# GPU box: encoder A/B -- the encoder's parity tests on the default library,
# then the isolated 64 x 1080p k_encode_rows launch (tools/enc_scaling.py,
# median of 5) for the default library and each variant in $VARS
# (webp_amd/libwebpgpu_<v>.so), alternating, $ROUNDS rounds.
source tools/gpu_step.sh
[ -n "$TESTS" ] && TAILN=2 step enc_ab_tests 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $TESTS
export BATCHES=${BATCHES:-64}
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in default $VARS; do
    lib=webp_amd/libwebpgpu.so; [ $v != default ] && lib=webp_amd/libwebpgpu_$v.so
    WEBPGPU_LIB=$lib TAILN=0 step enc_ab_${v}_$r 120 python tools/enc_scaling.py
    echo "$r $v $(tail -1 gpurun_out/enc_ab_${v}_$r.log)"
  done
done
