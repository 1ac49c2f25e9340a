#!/bin/bash
# Indel tally on the box: the indel GPU tests, then the c2id and c5 bench lines (kernel phases).
# Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A="--steps 10 --warmup 3 --no-cpu-baseline --no-pcie --no-fastq --no-e2e --no-side-configs"
timeout -k 10 600 python -u -m pytest tests/test_indels.py tests/test_adapter.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/indel_tests.log 2>&1 || { tail -30 gpurun_out/indel_tests.log; exit 1; }
tail -2 gpurun_out/indel_tests.log
timeout -k 10 300 python bench.py --config c2id $A > gpurun_out/ind_c2id.json 2> gpurun_out/ind_c2id.err || exit 1
timeout -k 10 300 python bench.py --config c5 --reads 10000 --genome 100000000 $A > gpurun_out/ind_c5.json 2> gpurun_out/ind_c5.err || exit 1
echo "exit=0"
