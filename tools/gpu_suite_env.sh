#!/bin/bash
# GPU box: the whole -m gpu suite under an environment setting, e.g.
# ENV_S="WG_DECODE_KERNEL=split" bash tools/gpu_suite_env.sh
source tools/gpu_step.sh
TAILN=3 step gpu_env 900 env $ENV_S python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
true
