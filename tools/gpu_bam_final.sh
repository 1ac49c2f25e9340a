#!/bin/bash
# The device BAM / region parity tests and one bam_cols_bench run on the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bam_final
timeout -k 10 600 python -u -m pytest tests/test_bam_device.py tests/test_region_device.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/bam_final/tests.log 2>&1 || { tail -40 gpurun_out/bam_final/tests.log; exit 1; }
tail -3 gpurun_out/bam_final/tests.log
timeout -k 10 300 python tools/bam_cols_bench.py --reps 5 > gpurun_out/bam_final/bench.json 2> gpurun_out/bam_final/bench.err \
  || { tail -20 gpurun_out/bam_final/bench.err; exit 1; }
cut -c1-700 gpurun_out/bam_final/bench.json
echo "exit=0"
