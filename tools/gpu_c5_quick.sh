#!/bin/bash
# Quick long-read check after a change to the wave walks: the long-read / indel / prep GPU tests, then
# the C5 line (bench.py --config c5) and its rocprofv3 kernel stats. Each GPU step has its own time
# limit; the chain stops at the first failure.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$REPO"
mkdir -p gpurun_out
TAG=${TAG:-quick}
C5="--config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-fastq --no-pcie"
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_indels.py -m gpu -x -q --timeout 120 --timeout-method thread \
      -k "long or indel or two_pass or prep or edge or pipeline" > gpurun_out/pytest_$TAG.log 2>&1 \
 && timeout -k 10 300 python3 bench.py $C5 > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o run --output-format csv -- \
      python3 bench.py $C5 > /dev/null 2> gpurun_out/prof_c5_$TAG.err
rc=$?
echo "exit=$rc"
tail -n 3 gpurun_out/pytest_$TAG.log
head -c 1500 gpurun_out/c5_$TAG.json
exit $rc
