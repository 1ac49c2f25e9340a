#!/bin/bash
# Group-target / unroll sweeps on the c3 and c5 side-line shapes (tools/sweep_group.py; the target
# applies at upload, results must not change: "same"). Each step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
SWEEP_SHAPE="reads=10000000,genome=25000000,windows=2500,germline=25000" SWEEP_TARGETS="704,1408,2816,5632" SWEEP_UNROLL="2" \
  timeout -k 10 400 python tools/sweep_group.py c3 20 > gpurun_out/sweep/c3.jsonl 2> gpurun_out/sweep/c3.err || { tail -5 gpurun_out/sweep/c3.err; exit 1; }
cut -c1-200 gpurun_out/sweep/c3.jsonl
SWEEP_SHAPE="reads=10000,genome=100000000" SWEEP_TARGETS="704,1408,2816,5632" SWEEP_UNROLL="1,2" \
  timeout -k 10 400 python tools/sweep_group.py c5 10 > gpurun_out/sweep/c5.jsonl 2> gpurun_out/sweep/c5.err || { tail -5 gpurun_out/sweep/c5.err; exit 1; }
cut -c1-200 gpurun_out/sweep/c5.jsonl
echo "exit=0"
