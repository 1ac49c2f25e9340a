#!/bin/bash
# rocprofv3 kernel-trace/stats of the bench, then one PMC pass per counter (never combined
# with tracing domains). Each step has its own time limit; the chain stops on failure.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$REPO"
mkdir -p gpurun_out
TAG=${TAG:-r01}
ARGS="--steps ${STEPS:-10} --warmup 3 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err \
 && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc_fetch_$TAG.err \
 && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc_write_$TAG.err
rc=$?
echo "exit=$rc"
find gpurun_out/prof_$TAG gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG -type f 2>/dev/null | head -20
exit $rc
