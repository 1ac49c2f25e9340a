#!/bin/bash
# Round-6 PMC summaries on the current kernel sources (verdict r05 item 3): the FASTQ formatter, then
# the c3 / c5 side-config steps and the c2 / c2id steps, each through tools/gpu_pmc_step.sh (or
# gpu_pmc_fastq.sh) and tools/pmc_step.py, which records the sources' digest (bench.py cites a summary
# only while it matches). CONFIGS selects a subset. The chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--no-e2e --no-side-configs --no-fastq --no-pcie"
R=${ROUND_TAG:-r06}
for c in ${CONFIGS:-fastq c3 c5 c2 c2id}; do
  case $c in
    fastq) TAG=${R}fq bash tools/gpu_pmc_fastq.sh && python3 tools/pmc_step.py ${R}fq fastq 9800000 gpurun_out/pmc_fastq.json || exit 1 ;;
    c3) TAG=${R}c3 BENCH_ARGS="--config c3 --reads 10000000 --genome 25000000 --windows 2500 --germline 25000 $A" bash tools/gpu_pmc_step.sh \
          && python3 tools/pmc_step.py ${R}c3 c3 10000000 gpurun_out/pmc_step_c3.json || exit 1 ;;
    c5) TAG=${R}c5 BENCH_ARGS="--config c5 --reads 10000 --genome 100000000 $A" bash tools/gpu_pmc_step.sh \
          && python3 tools/pmc_step.py ${R}c5 c5 10000 gpurun_out/pmc_step_c5.json || exit 1 ;;
    c2) TAG=${R}c2 BENCH_ARGS="$A" bash tools/gpu_pmc_step.sh \
          && python3 tools/pmc_step.py ${R}c2 c2 10000000 gpurun_out/pmc_step_c2.json || exit 1 ;;
    c2id) TAG=${R}c2id BENCH_ARGS="--config c2id $A" bash tools/gpu_pmc_step.sh \
          && python3 tools/pmc_step.py ${R}c2id c2id 10000000 gpurun_out/pmc_step_c2id.json || exit 1 ;;
  esac
  echo "== $c done"
done
echo ALLDONE
