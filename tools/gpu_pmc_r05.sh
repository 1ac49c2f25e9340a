#!/bin/bash
# Round-5 PMC step summaries: c2 and c2id (configs[1] with indel CIGARs: the multi-segment fused
# plan and the indel tally inside the step) through tools/gpu_pmc_step.sh, then tools/pmc_step.py.
# The chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--no-e2e --no-side-configs --no-fastq --no-pcie"
TAG=r05c2id BENCH_ARGS="--config c2id $A" bash tools/gpu_pmc_step.sh && \
python3 tools/pmc_step.py r05c2id c2id 10000000 gpurun_out/pmc_step_c2id.json && \
TAG=r05c2 BENCH_ARGS="$A" bash tools/gpu_pmc_step.sh && \
python3 tools/pmc_step.py r05c2 c2 10000000 gpurun_out/pmc_step_c2.json && echo ALLDONE
