#!/bin/bash
# Round-6 final evidence, part B: the c2 / c2id PMC summaries (tools/gpu_pmc_r06.sh), then the default
# bench (the driver's command) citing them. The chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fin
CONFIGS="${CONFIGS:-c2 c2id}" bash tools/gpu_pmc_r06.sh > gpurun_out/fin/pmc_b.log 2>&1 || { tail -20 gpurun_out/fin/pmc_b.log; exit 1; }
grep -E "step_hbm|== " gpurun_out/fin/pmc_b.log
mkdir -p profiles/r06 && cp gpurun_out/pmc_step_c2.json gpurun_out/pmc_step_c2id.json profiles/r06/ 2>/dev/null
[ -f gpurun_out/pmc_step_c3.json ] && cp gpurun_out/pmc_step_c3.json profiles/r06/
timeout -k 10 700 python bench.py > gpurun_out/fin/bench.json 2> gpurun_out/fin/bench.err || { tail -20 gpurun_out/fin/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/fin/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['summary']))"
echo "exit=0"
