#!/bin/bash
# Chromosome-scale end-to-end at configs[2] density on the GPU box: 2 x 20 Mb at 30x per sample
# (16 M reads), the streamed product in E2E_WORKERS (8) processes sharing the GPU, once per value of
# GANON_JOBS_PER_RANK given as arguments (default: 6). One JSON line per run under gpurun_out/.
# E2E_INFLATE_AB=1: each run again with GANON_GPU_INFLATE=1 (*_gi.json); E2E_BASE_INFLATE sets the
# first run's GANON_GPU_INFLATE (default auto: on with the GPU engine).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
D=$(mktemp -d /tmp/ganon_chrom.XXXXXX)
trap 'rm -rf $D' EXIT
timeout -k 10 400 python -c "import sys; sys.path.insert(0, '.'); from genomeanonymizer_amd.synth.fastpair import make_pair; make_pair('$D/in', n_contigs=2, contig_len=20_000_000, pairs_per_contig=2_000_000, window_every=20_000, seed=9)" || exit 1
echo "generated"
for jpr in ${@:-6}; do
  GANON_GPU_INFLATE=${E2E_BASE_INFLATE:-auto} GANON_JOBS_PER_RANK=$jpr E2E_RUNS=1 E2E_WORKERS=${E2E_WORKERS:-8} timeout -k 10 400 python tools/e2e_bench.py $D/in $D/out stream > gpurun_out/e2e_chrom_j$jpr.json 2> gpurun_out/e2e_chrom_j$jpr.err || { tail -5 gpurun_out/e2e_chrom_j$jpr.err; exit 1; }
  echo "jobs per rank $jpr: $(head -c 300 gpurun_out/e2e_chrom_j$jpr.json)"
  if [ "${E2E_INFLATE_AB:-0}" = 1 ]; then   # the same run with BGZF inflate on the GPU
    GANON_GPU_INFLATE=1 GANON_JOBS_PER_RANK=$jpr E2E_RUNS=1 E2E_WORKERS=${E2E_WORKERS:-8} timeout -k 10 400 python tools/e2e_bench.py $D/in $D/out stream > gpurun_out/e2e_chrom_j${jpr}_gi.json 2> gpurun_out/e2e_chrom_j${jpr}_gi.err || { tail -5 gpurun_out/e2e_chrom_j${jpr}_gi.err; exit 1; }
  fi
done
echo "exit=0"
