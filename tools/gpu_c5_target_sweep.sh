#!/bin/bash
# Long-read group-target sweep (GANON_PARAM_GROUP_TARGET in cost units; long-read default 1408) on the
# c5 side-config shape (10 k reads of 10-100 kb).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
C5="--config c5 --reads 10000 --genome 100000000 --steps 5 --warmup 2 --no-cpu-baseline --no-fastq --no-pcie --no-e2e --no-side-configs"
for T in 704 1408 2816 5632; do
  timeout -k 10 200 python bench.py $C5 --target $T > gpurun_out/c5_t$T.json 2> gpurun_out/c5_t$T.err || exit 1
  echo "c5 $T done"
done
echo "exit=0"
