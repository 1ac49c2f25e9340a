#!/bin/bash
# Full default bench (every line, as the driver runs it), then a rocprofv3 kernel-trace summary of
# the configs[1] step. Each step has its own time limit; the chain stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
start=$(date +%s)
timeout -k 10 1000 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - start ))s"; tail -c 600 gpurun_out/bench_full.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run -- python3 bench.py --no-e2e --no-side-configs --no-cpu-baseline --no-pcie --no-fastq --steps 50 --warmup 5 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
rc=$?; echo "prof rc=$rc"; exit $rc
