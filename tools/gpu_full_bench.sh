#!/bin/bash
# The full default bench (every line, as the driver runs it). Its own time limit; the JSON line goes
# to gpurun_out/bench_full.json, stderr (progress, child lines) to bench_full.err.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
start=$(date +%s)
timeout -k 10 1100 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - start ))s"; tail -c 800 gpurun_out/bench_full.err; exit $rc
