#!/bin/bash
# PMC passes over tools/inflate_bench.py --no-cpu --iters 1 (one pass per counter group, each under
# its own kill timer), summed over the k_inflate dispatches. GANON_INFLATE_ROUNDS passes through.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/inf_pmc_$i -o run --output-format csv -- python3 tools/inflate_bench.py --no-cpu --iters 1 \
    > gpurun_out/inf_pmc_$i.log 2>&1 || { tail -5 gpurun_out/inf_pmc_$i.log; exit 1; }
done
find gpurun_out/inf_pmc_1 gpurun_out/inf_pmc_2 -name '*counter_collection.csv' | while read f; do
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
n = 0
for r in csv.DictReader(open(sys.argv[1])):
    if "k_inflate" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
print({k: v for k, v in acc.items()})
PY
done
echo "exit=0"
