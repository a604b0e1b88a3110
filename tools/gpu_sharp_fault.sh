#!/bin/bash
# GPU box: the sharpyuv tests on the default build (with the cross-colour
# tests), then on the WG_BOUNDS build with every launch serialised
# (AMD_SERIALIZE_KERNEL=3: a fault is reported by the launch that made it)
source tools/gpu_step.sh
TAILN=3 step default_sharp 300 python -u -m pytest tests/test_sharpyuv.py tests/test_vp8l_color.py -m gpu -x -q --timeout 120 --timeout-method thread
TAILN=30 step bounds_sharp_serial 300 env AMD_SERIALIZE_KERNEL=3 WEBPGPU_LIB=webp_amd/libwebpgpu_bounds.so python -u -m pytest tests/test_sharpyuv.py -m gpu -x -s -v --timeout 120 --timeout-method thread
