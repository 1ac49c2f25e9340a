#!/bin/bash
# Group-target sweep (GANON_PARAM_GROUP_TARGET, cost units per group) on the c3 side-config shape and c2.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
C3="--config c3 --reads 10000000 --genome 25000000 --windows 2500 --germline 25000 --steps 20 --warmup 3 --no-cpu-baseline --no-fastq --no-pcie --no-e2e --no-side-configs"
C2="--steps 50 --warmup 5 --no-cpu-baseline --no-fastq --no-pcie --no-e2e --no-side-configs"
for T in 512 704 1024 1408; do
  timeout -k 10 200 python bench.py $C3 --target $T > gpurun_out/c3_t$T.json 2> gpurun_out/c3_t$T.err || exit 1
  echo "c3 $T done"
done
for T in 512 1024; do
  timeout -k 10 200 python bench.py $C2 --target $T > gpurun_out/c2_t$T.json 2> gpurun_out/c2_t$T.err || exit 1
  echo "c2 $T done"
done
timeout -k 10 200 python bench.py $C2 > gpurun_out/c2_t704.json 2> gpurun_out/c2_t704.err || exit 1
echo "exit=0"
