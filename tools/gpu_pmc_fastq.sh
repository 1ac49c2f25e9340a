#!/bin/bash
# HBM bytes of the FASTQ formatter's kernels (9.8 M configs[1] records, tools/fq_run.py): kernel trace +
# stats, then the three PMC passes of tools/gpu_pmc_step.sh (never combined with tracing domains; at
# most 4 TCC counters each); tools/pmc_step.py TAG fastq 9800000 OUT.json summarizes them with the
# formatter sources' digest (bench.py cites the summary while the digest matches). Each step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$REPO"
mkdir -p gpurun_out
TAG=${TAG:-fq}
ARGS="--reads ${READS:-9800000} --runs 3"   # (the bench formats its first batch: 9.8 M records)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 tools/fq_run.py $ARGS > gpurun_out/fqrun_$TAG.json 2> gpurun_out/prof_$TAG.err || exit $?
echo "trace done"
P1="TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_WRREQ"
P2="TCC_EA0_WRREQ_64B FETCH_SIZE"
P3="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $P -d gpurun_out/pmc_${TAG}_p$i -o run --output-format csv -- \
      python3 tools/fq_run.py $ARGS > /dev/null 2> gpurun_out/pmc_${TAG}_p$i.err || exit $?
  echo "pmc pass $i done"
done
echo "exit=0"
