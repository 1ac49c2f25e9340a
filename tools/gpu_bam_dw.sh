#!/bin/bash
# k_bam_scatter by dwords (round 6): the device BAM / region parity tests, then tools/bam_cols_bench.py
# on the default build (dword blobs) and on the byte-path build (tools/build_variant.py bam0
# -DGANON_BAM_DW=0), alternated. Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bam_dw
timeout -k 10 600 python -u -m pytest tests/test_bam_device.py tests/test_region_device.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/bam_dw/tests.log 2>&1 || { tail -40 gpurun_out/bam_dw/tests.log; exit 1; }
tail -3 gpurun_out/bam_dw/tests.log
for rep in 1 2; do
  for v in dw byte; do
    if [ "$v" = dw ]; then LIB=""; else LIB="genomeanonymizer_amd/variants/libganon_hip_bam0.so"; fi
    GANON_HIP_LIB=$LIB timeout -k 10 300 python tools/bam_cols_bench.py --reps 5 > gpurun_out/bam_dw/${v}_$rep.json \
      2> gpurun_out/bam_dw/${v}_$rep.err || { tail -20 gpurun_out/bam_dw/${v}_$rep.err; exit 1; }
    echo "$v rep $rep: $(cut -c1-900 gpurun_out/bam_dw/${v}_$rep.json)"
  done
done
echo "exit=0"
