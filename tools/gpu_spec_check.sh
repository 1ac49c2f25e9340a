#!/bin/bash
# GPU check of a build: every GPU test, then the configs[1] bench without its child lines.
# Each step has its own time limit; the chain stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-e2e --no-side-configs --no-cpu-baseline --no-pcie --no-fastq --steps 100 --warmup 10 > gpurun_out/bench_spec.json 2> gpurun_out/bench_spec.err
rc=$?; tail -c 400 gpurun_out/bench_spec.err; head -c 1500 gpurun_out/bench_spec.json; exit $rc
