#!/bin/bash
# k_bam_scatter records per workgroup A/B (round 6): tools/bam_cols_bench.py on the default build
# (16 records, 16 KiB staged) and variant builds (tools/build_variant.py srN -DGANON_SCAT_RECS=N
# -DGANON_SCAT_STAGE=B), alternated. Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bam_sr
for rep in 1 2; do
  for v in 16 8 32 64; do
    if [ "$v" = 16 ]; then LIB=""; else LIB="genomeanonymizer_amd/variants/libganon_hip_sr$v.so"; fi
    GANON_HIP_LIB=$LIB timeout -k 10 300 python tools/bam_cols_bench.py --reps 5 > gpurun_out/bam_sr/sr${v}_$rep.json \
      2> gpurun_out/bam_sr/sr${v}_$rep.err || { tail -20 gpurun_out/bam_sr/sr${v}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['device_ms'], d['device_kernels_ms']['k_bam_scatter'], d['columns_equal_host_decoder'])" gpurun_out/bam_sr/sr${v}_$rep.json "recs $v rep $rep"
  done
done
echo "exit=0"
