#!/bin/bash
# Round-6 validation on the final tree: smoke, every GPU test, the default bench (the driver's
# command). Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 \
 && timeout -k 10 700 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
rc=$?
echo "exit=$rc"
tail -n 2 gpurun_out/final/smoke.log
tail -n 3 gpurun_out/final/pytest_gpu.log
python3 -c "import json; d=json.loads(open('gpurun_out/final/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['summary']))" 2>/dev/null
exit $rc
