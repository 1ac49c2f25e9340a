#!/bin/bash
# Round-6 evidence in one box: the bounds-checked indel run, then the c3 / c5 group sweeps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_indel_ichk.sh && bash tools/gpu_sweep_r06.sh
