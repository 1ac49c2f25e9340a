#!/bin/bash
# c5 line A/B over compile-time variants: bash tools/gpu_c5_variants.sh "tag|ENV=.." ...
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for spec in "$@"; do
  IFS='|' read -r tag envs flags <<< "$spec"
  timeout -k 10 400 env $envs python bench.py --config c5 --reads 10000 --genome 100000000 --steps 5 --warmup 2 --no-e2e --no-side-configs --no-cpu-baseline --no-pcie --no-fastq $flags > gpurun_out/c5_$tag.json 2> gpurun_out/c5_$tag.err
  rc=$?; [ $rc -eq 0 ] || { tail -c 600 gpurun_out/c5_$tag.err; exit $rc; }
  python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
d = json.load(open(f"gpurun_out/c5_{t}.json"))
print(t, d["ms_per_step"], {n: v["avg_ms"] for n, v in d["pass"]["kernels"].items()}, flush=True)
PY
done
