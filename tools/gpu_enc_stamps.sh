#!/bin/bash
# GPU box: the encoder's per-phase cycles on the bench's frames (the stamped
# build, tools/debug_enc_phases.py CONTENT=bench), then the VP8L / cross-colour
# counter passes (tools/gpu_vp8l_pmc.sh).
source tools/gpu_step.sh
TAILN=4 step enc_stamps 300 env WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so CONTENT=bench python -u tools/debug_enc_phases.py
bash tools/gpu_vp8l_pmc.sh
