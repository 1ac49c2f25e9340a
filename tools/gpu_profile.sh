#!/bin/bash
# rocprofv3 kernel trace + stats of the bench, then one PMC pass per counter (never combined
# with tracing domains): L2-to-fabric read requests by size and write requests, from which
# tools/pmc_summary.py derives HBM bytes per launch. Each step has its own time limit; the
# chain stops at the first failure.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$REPO"
mkdir -p gpurun_out
TAG=${TAG:-r01}
ARGS="--steps ${STEPS:-10} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-}"
PMC_ARGS="--steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err || exit $?
for C in TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_WRREQ TCC_EA0_WRREQ_64B FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C -d gpurun_out/pmc_${TAG}_$C -o run --output-format csv -- \
      python3 bench.py $PMC_ARGS > /dev/null 2> gpurun_out/pmc_${TAG}_$C.err || exit $?
done
echo "exit=0"
find gpurun_out/prof_$TAG -type f | head -20
