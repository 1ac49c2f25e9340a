#!/bin/bash
# C3 (deep coverage) and C5 (long reads) lines, rocprofv3 kernel stats of both, and one PMC pass per
# counter (no tracing domains in a PMC pass) for the HBM traffic of their kernels. Each GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$REPO"
mkdir -p gpurun_out
TAG=${TAG:-r02}
C3="--config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-fastq --no-pcie"
C5="--config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-fastq --no-pcie"
timeout -k 10 300 python3 bench.py $C3 > gpurun_out/c3_$TAG.json 2> gpurun_out/c3_$TAG.err \
 && timeout -k 10 300 python3 bench.py $C5 > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_$TAG -o run --output-format csv -- \
      python3 bench.py $C3 > /dev/null 2> gpurun_out/prof_c3_$TAG.err \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o run --output-format csv -- \
      python3 bench.py $C5 > /dev/null 2> gpurun_out/prof_c5_$TAG.err || exit $?
for C in TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_WRREQ TCC_EA0_WRREQ_64B; do
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/pmc_c5${TAG}_$C -o run --output-format csv -- \
      python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-fastq --no-pcie > /dev/null 2> gpurun_out/pmc_c5${TAG}_$C.err || exit $?
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/pmc_c3${TAG}_$C -o run --output-format csv -- \
      python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-fastq --no-pcie > /dev/null 2> gpurun_out/pmc_c3${TAG}_$C.err || exit $?
done
echo "exit=0"
