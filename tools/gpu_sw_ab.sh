#!/bin/bash
# Scan-store A/B (round 6): the mask GPU tests, then c2 / c3 / c2id bench lines with the scan store on
# (default) and off (GANON_SCAN_STORE=0), alternated. Each step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sw_ab
A="--steps ${STEPS:-50} --warmup 5 --no-cpu-baseline --no-pcie --no-fastq --no-e2e --no-side-configs"
C3="--config c3 --reads 10000000 --genome 25000000 --windows 2500 --germline 25000"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${PYTEST_TARGET:-tests/test_gpu.py} -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/sw_ab/tests.log 2>&1 || { tail -40 gpurun_out/sw_ab/tests.log; exit 1; }
  tail -3 gpurun_out/sw_ab/tests.log
fi
for rep in 1 2; do
  for sw in 1 0; do
    for cfg in c2 c3 c2id; do
      case $cfg in c3) X="$C3" ;; c2id) X="--config c2id" ;; *) X="" ;; esac
      GANON_SCAN_STORE=$sw timeout -k 10 300 python bench.py $A $X > gpurun_out/sw_ab/${cfg}_sw${sw}_$rep.json \
        2> gpurun_out/sw_ab/${cfg}_sw${sw}_$rep.err || { tail -20 gpurun_out/sw_ab/${cfg}_sw${sw}_$rep.err; exit 1; }
      python3 - "$cfg" "$sw" "$rep" <<'EOF'
import json, sys
cfg, sw, rep = sys.argv[1:]
d = json.loads(open(f"gpurun_out/sw_ab/{cfg}_sw{sw}_{rep}.json").read().strip().splitlines()[-1])
k = d["pass"]["kernels"]
print(cfg, "sw", sw, "rep", rep, "ms/step", d["ms_per_step"], "one_stream", d.get("one_stream_ms_per_step"),
      "k_group", round(k.get("k_group_fused", {}).get("avg_ms", 0), 4), flush=True)
EOF
    done
  done
done
echo "exit=0"
