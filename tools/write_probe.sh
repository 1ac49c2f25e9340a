#!/bin/bash
# Write/read traffic of the fused group kernel by phase: copy only (skip scan + classify) with
# non-temporal and plain stores, and the full kernel. One rocprofv3 --pmc pass per counter.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$REPO"
mkdir -p gpurun_out/probe
for CFG in ${CFGS:-0:2:3:256:1 0:2:3:256:0 0:2:5:256:1}; do
  for C in ${CTRS:-TCC_EA0_WRREQ_64B TCC_EA0_RDREQ_128B}; do
    T=$(echo "$CFG" | tr ':' '_')
    timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/probe/${T}_$C -o run --output-format csv -- \
      python3 tools/phase_timing.py --rounds 1 --steps 2 --configs $CFG > gpurun_out/probe/${T}_$C.json 2> gpurun_out/probe/${T}_$C.err || exit $?
  done
done
python3 - <<'PY'
import csv, glob, collections, json
out = {}
for d in sorted(glob.glob("gpurun_out/probe/*_TCC*")):
    if not d.endswith(tuple("0123456789BQ")) and "." in d: continue
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f: continue
    tot, n = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(f[0])):
        if "k_group" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    cfg = d.split("/")[-1]
    out[cfg] = {k: tot[k] / n[k] for k in tot}
print(json.dumps(out, indent=1))
PY
