#!/bin/bash
# GPU inflate on the box: its tests, the throughput bench (tools/inflate_bench.py) and a rocprofv3
# kernel-trace summary of the bench. Each step has its own time limit; the chain stops at the first
# failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_inflate.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/inflate_tests.log 2>&1 || { tail -30 gpurun_out/inflate_tests.log; exit 1; }
tail -3 gpurun_out/inflate_tests.log
timeout -k 10 300 python tools/inflate_bench.py ${INF_ARGS:-} > gpurun_out/inflate_bench.json 2> gpurun_out/inflate_bench.err \
  || { tail -20 gpurun_out/inflate_bench.err; exit 1; }
cat gpurun_out/inflate_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/inf_prof -o inf -- python3 tools/inflate_bench.py --no-cpu \
  > gpurun_out/inflate_prof.log 2>&1 || { tail -20 gpurun_out/inflate_prof.log; exit 1; }
find gpurun_out/inf_prof -name '*kernel_stats.csv' -exec cat {} \;
# PMC passes (INF_PMC=1): wave cycles / waits, then instruction mix, one pass each
if [ -n "$INF_PMC" ]; then
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    -d gpurun_out/inf_pmc_a -o run --output-format csv -- python3 tools/inflate_bench.py --no-cpu --iters 1 \
    > gpurun_out/inf_pmc_a.log 2>&1 || { tail -5 gpurun_out/inf_pmc_a.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES \
    -d gpurun_out/inf_pmc_b -o run --output-format csv -- python3 tools/inflate_bench.py --no-cpu --iters 1 \
    > gpurun_out/inf_pmc_b.log 2>&1 || { tail -5 gpurun_out/inf_pmc_b.log; exit 1; }
  find gpurun_out/inf_pmc_a gpurun_out/inf_pmc_b -name '*counter_collection.csv' | while read f; do
    python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_inflate" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(dict(acc))
PY
  done
fi
echo "exit=0"
