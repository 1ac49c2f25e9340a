#!/bin/bash
# GPU-box sequence after a group-kernel change: the masking parity tests, then the c3 (deep
# coverage) and c5 (long reads) bench lines. Each step has its own time limit; the chain stops at
# the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_distributed.py tests/test_indels.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/grp_tests.log 2>&1 \
 && timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-pcie --no-fastq \
    > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err \
 && timeout -k 10 250 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-fastq \
    > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
rc=$?
tail -n 1 gpurun_out/grp_tests.log
for f in gpurun_out/bench_c3.json gpurun_out/bench_c5.json; do
  python -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], d['roofline']['frac'], d['pass']['kernels'].get('k_group_fused'))" "$f" 2>/dev/null
done
exit $rc
