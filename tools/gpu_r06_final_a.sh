#!/bin/bash
# Round-6 final evidence, part A: smoke and every GPU test on the final tree, then the formatter / c3 /
# c5 PMC summaries (tools/gpu_pmc_r06.sh). The chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fin
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 || { tail -20 gpurun_out/fin/smoke.log; exit 1; }
tail -1 gpurun_out/fin/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/fin/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/fin/pytest_gpu.log
CONFIGS="${CONFIGS:-fastq c3 c5}" bash tools/gpu_pmc_r06.sh > gpurun_out/fin/pmc.log 2>&1 || { tail -20 gpurun_out/fin/pmc.log; exit 1; }
grep -E "step_hbm|== " gpurun_out/fin/pmc.log
echo "exit=0"
