#!/bin/bash
# GPU inflate A/B on the box: the inflate tests, then tools/inflate_bench.py with the token-round
# decoder (default) and with the scalar symbol loop alone (GANON_INFLATE_ROUNDS=0), then a rocprofv3
# kernel-trace summary of the default. Each step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_inflate.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/inflate_tests.log 2>&1 || { tail -30 gpurun_out/inflate_tests.log; exit 1; }
tail -3 gpurun_out/inflate_tests.log
timeout -k 10 300 python tools/inflate_bench.py --no-cpu > gpurun_out/inflate_bench_rounds.json 2> gpurun_out/inflate_bench.err \
  || { tail -20 gpurun_out/inflate_bench.err; exit 1; }
cat gpurun_out/inflate_bench_rounds.json
GANON_INFLATE_ROUNDS=0 timeout -k 10 300 python tools/inflate_bench.py --no-cpu > gpurun_out/inflate_bench_scalar.json 2>> gpurun_out/inflate_bench.err \
  || { tail -20 gpurun_out/inflate_bench.err; exit 1; }
cat gpurun_out/inflate_bench_scalar.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/inf_prof -o inf -- python3 tools/inflate_bench.py --no-cpu \
  > gpurun_out/inflate_prof.log 2>&1 || { tail -20 gpurun_out/inflate_prof.log; exit 1; }
find gpurun_out/inf_prof -name '*kernel_stats.csv' -exec cat {} \;
echo "exit=0"
