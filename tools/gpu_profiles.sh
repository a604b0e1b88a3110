#!/bin/bash
# GPU box: the rocprofv3 passes of tools/profile.sh and the encoder SQ passes
# (tools/gpu_enc_pmc.sh), without the suite and bench (tools/gpu_round.sh
# PROFILE=0 runs those).
source tools/gpu_step.sh
step profile 900 bash tools/profile.sh
bash tools/gpu_enc_pmc.sh
