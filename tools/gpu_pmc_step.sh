#!/bin/bash
# One bench configuration under rocprofv3: kernel trace + stats, then three PMC passes (never
# combined with tracing domains; at most 4 TCC counters each): L2-to-fabric read requests by size
# and write requests, FETCH_SIZE / WRITE_SIZE beside them. tools/pmc_step.py turns them into HBM
# bytes per launch of every kernel of the step. Each step has its own time limit; the chain stops at
# the first failure.
#   TAG=r02c3 BENCH_ARGS="--config c3 --no-fastq --no-pcie" tools/gpu_pmc_step.sh
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$REPO"
mkdir -p gpurun_out
TAG=${TAG:-r02}
ARGS="--steps ${STEPS:-10} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-}"
PMC_ARGS="--steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err || exit $?
echo "trace done"
P1="TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_WRREQ"
P2="TCC_EA0_WRREQ_64B FETCH_SIZE"
P3="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -k 10 -s KILL 500 rocprofv3 --pmc $P -d gpurun_out/pmc_${TAG}_p$i -o run --output-format csv -- \
      python3 bench.py $PMC_ARGS > /dev/null 2> gpurun_out/pmc_${TAG}_p$i.err || exit $?
  echo "pmc pass $i done"
done
echo "exit=0"
