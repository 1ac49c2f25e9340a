#!/bin/bash
# SQ instruction / wait counters of the FASTQ formatter kernels (tools/fq_run.py), one
# rocprofv3 --pmc pass per counter (no tracing domains in a PMC pass). Each pass has its own
# time limit; the chain stops at the first failure. Output: gpurun_out/fqpmc_$TAG_<counter>.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$REPO"
mkdir -p gpurun_out
TAG=${TAG:-fq}
ARGS="--reads ${READS:-2000000} --runs 2 --configs ${CONFIGS:-2:0}"
timeout -k 10 300 python3 tools/fq_run.py $ARGS > gpurun_out/fqrun_$TAG.json 2> gpurun_out/fqrun_$TAG.err || exit $?
for C in ${COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH GRBM_GUI_ACTIVE}; do
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/fqpmc_${TAG}_$C -o run --output-format csv -- \
      python3 tools/fq_run.py $ARGS > /dev/null 2> gpurun_out/fqpmc_${TAG}_$C.err || exit $?
done
echo "exit=0"
