#!/bin/bash
# Round-4 PMC step summaries: c2, c3, c5 through tools/gpu_pmc_step.sh (kernel trace + three PMC
# passes each), then tools/pmc_step.py per config. The chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--no-e2e --no-side-configs --no-fastq --no-pcie"
TAG=r04c2 BENCH_ARGS="$A" bash tools/gpu_pmc_step.sh && \
python3 tools/pmc_step.py r04c2 c2 10000000 gpurun_out/pmc_step_c2.json && \
TAG=r04c3 BENCH_ARGS="--config c3 --reads 10000000 --genome 25000000 --windows 2500 --germline 25000 $A" bash tools/gpu_pmc_step.sh && \
python3 tools/pmc_step.py r04c3 c3 10000000 gpurun_out/pmc_step_c3.json && \
TAG=r04c5 BENCH_ARGS="--config c5 --reads 10000 --genome 100000000 $A" bash tools/gpu_pmc_step.sh && \
python3 tools/pmc_step.py r04c5 c5 10000 gpurun_out/pmc_step_c5.json && echo ALLDONE
