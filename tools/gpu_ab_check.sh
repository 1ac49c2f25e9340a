#!/bin/bash
# GPU check of a kernel change: the masking GPU tests, then the configs[1] bench line with the
# default build settings and with the extra bench flags given as arguments (an A/B pair).
# Each step has its own time limit; the chain stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-e2e --no-side-configs --no-cpu-baseline --no-pcie --no-fastq --steps 100 --warmup 10"
timeout -k 10 300 $B > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err
rc=$?; tail -c 300 gpurun_out/bench_a.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B "$@" > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err
rc=$?; tail -c 300 gpurun_out/bench_b.err; [ $rc -eq 0 ] || exit $rc
python - <<'EOF'
import json
for t in "ab":
    d = json.load(open(f"gpurun_out/bench_{t}.json"))
    k = {n: v["avg_ms"] for n, v in d["pass"]["kernels"].items()}
    print(t, d["ms_per_step"], d.get("one_stream_ms_per_step"), d.get("sync_plan_ms_per_step"), k)
EOF
