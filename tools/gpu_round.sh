#!/bin/bash
# GPU box, one call: the -m gpu suite, the bench line (with C3 / C5), then the
# rocprofv3 passes of tools/profile.sh and the encoder SQ passes
# (tools/gpu_enc_pmc.sh).  Every step under its own limit; the first failure
# ends the call.
source tools/gpu_step.sh
step suite 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 420 python bench.py
[ "${PROFILE:-1}" = 1 ] || exit 0
step profile 1000 bash tools/profile.sh
bash tools/gpu_enc_pmc.sh
