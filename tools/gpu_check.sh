#!/bin/bash
# GPU-box sequence: smoke, GPU tests, short bench. Each GPU step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/gpu_info.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 900 python -u -m pytest ${PYTEST_TARGET:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "exit=$rc"
tail -n 3 gpurun_out/smoke.log 2>/dev/null
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -n 40
cat gpurun_out/bench.json 2>/dev/null | head -c 3000
tail -n 20 gpurun_out/bench.err 2>/dev/null
exit $rc
