#!/bin/bash
# Round-end GPU sequence: smoke, every GPU test, the default bench (driver's command), the same
# bench under rocprofv3 --kernel-trace --stats, and the chromosome-scale end-to-end check. Each GPU
# step has its own time limit; the chain stops at the first failure.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$REPO"
mkdir -p gpurun_out
TAG=${TAG:-final}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_$TAG -o run --output-format csv -- \
      python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --no-side-configs > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err \
 && E2E_WORKERS=2 timeout -k 10 900 bash tools/gpu_e2e_big.sh > gpurun_out/e2e_big.log 2>&1
rc=$?
echo "exit=$rc"
tail -n 2 gpurun_out/smoke.log
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -n 2
head -c 1200 gpurun_out/bench.json
exit $rc
