#!/bin/bash
# Verdict r05 item 2: the indel tally under the bounds-checked build (GANON_INDEL_CHECK=1: every index
# the tally kernels dereference is checked against its buffer's capacity; a failing check is reported
# by ganon_indel_download with its source line) — the indel GPU tests in every sort / walk mode, the
# full-size c2id oracle test in the default and the global-sort mode, and the c2id / c5 bench lines.
# Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ichk
export GANON_HIP_LIB=genomeanonymizer_amd/variants/libganon_hip_ichk.so
A="--steps 5 --warmup 2 --no-cpu-baseline --no-pcie --no-fastq --no-e2e --no-side-configs"
timeout -k 10 600 python -u -m pytest tests/test_indels.py -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/ichk/indel_tests.log 2>&1 || { tail -40 gpurun_out/ichk/indel_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/ichk/indel_tests.log | tail -1
for mode in default global; do
  if [ $mode = global ]; then export GANON_INDEL_SORTMODE=global; fi
  timeout -k 10 600 python -u -m pytest tests/test_gpu.py::test_hip_config2_indel_cigars_full_size_matches_oracle -m gpu -v \
    --timeout 500 --timeout-method thread > gpurun_out/ichk/c2id_full_$mode.log 2>&1 || { tail -40 gpurun_out/ichk/c2id_full_$mode.log; exit 1; }
  echo "c2id full-size ($mode): $(grep -E 'passed|failed' gpurun_out/ichk/c2id_full_$mode.log | tail -1)"
done
unset GANON_INDEL_SORTMODE
timeout -k 10 300 python bench.py --config c2id $A > gpurun_out/ichk/c2id.json 2> gpurun_out/ichk/c2id.err || { tail -20 gpurun_out/ichk/c2id.err; exit 1; }
timeout -k 10 300 python bench.py --config c5 --reads 10000 --genome 100000000 $A > gpurun_out/ichk/c5.json 2> gpurun_out/ichk/c5.err || { tail -20 gpurun_out/ichk/c5.err; exit 1; }
echo "exit=0"
