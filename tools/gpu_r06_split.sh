#!/bin/bash
# Main tree: every GPU test. Then the deep-scope split build (variants/libganon_hip_split.so, branch
# split-wip): the mask GPU tests, and c3 / c2 bench lines against the main build, alternated. Each step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06s
V=genomeanonymizer_amd/variants/libganon_hip_split.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06s/main_tests.log 2>&1
echo "main tests rc=$? $(tail -1 gpurun_out/r06s/main_tests.log)"
GANON_HIP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06s/split_tests.log 2>&1
echo "split tests rc=$? $(tail -1 gpurun_out/r06s/split_tests.log)"
grep FAILED gpurun_out/r06s/split_tests.log | head
A="--steps 30 --warmup 5 --no-cpu-baseline --no-pcie --no-fastq --no-e2e --no-side-configs"
C3="--config c3 --reads 10000000 --genome 25000000 --windows 2500 --germline 25000"
for rep in 1 2; do
  for lib in split main; do
    for cfg in c3 c2; do
      case $cfg in c3) X="$C3" ;; *) X="" ;; esac
      E=""; [ $lib = split ] && E="GANON_HIP_LIB=$V"
      env $E timeout -k 10 300 python bench.py $A $X > gpurun_out/r06s/${cfg}_${lib}_$rep.json 2> gpurun_out/r06s/${cfg}_${lib}_$rep.err || { tail -5 gpurun_out/r06s/${cfg}_${lib}_$rep.err; exit 1; }
      python3 - "$cfg" "$lib" "$rep" <<'PY'
import json, sys
cfg, lib, rep = sys.argv[1:]
d = json.loads(open(f"gpurun_out/r06s/{cfg}_{lib}_{rep}.json").read().strip().splitlines()[-1])
k = d["pass"]["kernels"]
print(cfg, lib, rep, "ms/step", d["ms_per_step"], "one_stream", d.get("one_stream_ms_per_step"),
      {n: round(v["avg_ms"], 4) for n, v in k.items()}, flush=True)
PY
    done
  done
done
echo "exit=0"
