#!/bin/bash
# A/B of compile-time variants (tools/build_variant.py) and bench flags on the configs[1] line:
#   bash tools/gpu_variants.sh "tag|ENV=..|bench flags" ...
# after the masking GPU tests of the default build. Each step has its own time limit; the chain
# stops at the first failure. Results: gpurun_out/var_<tag>.json and a summary line per variant.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_var.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_var.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-e2e --no-side-configs --no-cpu-baseline --no-pcie --no-fastq --steps 100 --warmup 10"
for spec in "$@"; do
  IFS='|' read -r tag envs flags <<< "$spec"
  timeout -k 10 300 env $envs $B $flags > gpurun_out/var_$tag.json 2> gpurun_out/var_$tag.err
  rc=$?; [ $rc -eq 0 ] || { tail -c 600 gpurun_out/var_$tag.err; exit $rc; }
  python - "$tag" <<'EOF'
import json, sys
t = sys.argv[1]
d = json.load(open(f"gpurun_out/var_{t}.json"))
k = {n: v["avg_ms"] for n, v in d["pass"]["kernels"].items()}
print(t, d["ms_per_step"], d.get("one_stream_ms_per_step"), d.get("sync_plan_ms_per_step"), k, flush=True)
EOF
done
