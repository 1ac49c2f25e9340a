#!/bin/bash
# Long-read / indel GPU tests, then the c5 line with and without a flag set given as arguments.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_indels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c5.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_c5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config c5 --reads 10000 --genome 100000000 --steps 5 --warmup 2 --no-e2e --no-side-configs --no-cpu-baseline --no-pcie --no-fastq > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
rc=$?; tail -c 300 gpurun_out/bench_c5.err; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_c5.json"))
print("c5", d["ms_per_step"], d.get("run_only_ms_per_step"), {n: v["avg_ms"] for n, v in d["pass"]["kernels"].items()})
PY
