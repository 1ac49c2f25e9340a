#!/bin/bash
# One GPU call: default bench (c2, BASELINE configs[1]), C3/C5 lines, rocprofv3 kernel stats of
# the c2 and c5 benches. Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$REPO"
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 400 python3 bench.py > gpurun_out/m_c2.json 2> gpurun_out/m_c2.err \
 && timeout -k 10 300 python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-fastq > gpurun_out/m_c3.json 2> gpurun_out/m_c3.err \
 && timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-fastq > gpurun_out/m_c5.json 2> gpurun_out/m_c5.err \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_$TAG -o run --output-format csv -- \
      python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/m_prof_c2.json 2> gpurun_out/m_prof_c2.err \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o run --output-format csv -- \
      python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-fastq > gpurun_out/m_prof_c5.json 2> gpurun_out/m_prof_c5.err
rc=$?
echo "exit=$rc"
find gpurun_out -name "*kernel_stats.csv" | head
exit $rc
