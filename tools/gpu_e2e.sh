#!/bin/bash
# GPU tests, then the end-to-end pipeline (streamed and whole-sample) on a tiled synthetic pair.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${PYTEST_TARGET:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python tools/e2e_data.py /tmp/e2e_data ${COPIES:-24} > gpurun_out/e2e_data.log 2>&1 \
 && timeout -k 10 600 python tools/e2e_bench.py /tmp/e2e_data /tmp/e2e_out ${E2E_MODES:-stream,whole} > gpurun_out/e2e.json 2> gpurun_out/e2e.err
rc=$?
echo "exit=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -n 12
cat gpurun_out/e2e.json 2>/dev/null
tail -n 5 gpurun_out/e2e.err 2>/dev/null
exit $rc
