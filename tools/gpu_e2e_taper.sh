#!/bin/bash
# The 30x chromosome-scale end-to-end line (tools/gpu_e2e_chrom.sh's input) once per GANON_JOB_TAPER
# value given as arguments (default: 1 0.5): first/last-job taper A/B. One JSON line per run under
# gpurun_out/. Each run has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
D=$(mktemp -d /tmp/ganon_chrom.XXXXXX)
trap 'rm -rf $D' EXIT
timeout -k 10 400 python -c "import sys; sys.path.insert(0, '.'); from genomeanonymizer_amd.synth.fastpair import make_pair; make_pair('$D/in', n_contigs=2, contig_len=20_000_000, pairs_per_contig=2_000_000, window_every=20_000, seed=9)" || exit 1
echo "generated"
for tp in ${@:-1 0.5}; do
  GANON_JOB_TAPER=$tp E2E_RUNS=${E2E_RUNS:-2} E2E_WORKERS=${E2E_WORKERS:-8} timeout -k 10 400 python tools/e2e_bench.py $D/in $D/out stream > gpurun_out/e2e_taper_$tp.json 2> gpurun_out/e2e_taper_$tp.err || { tail -5 gpurun_out/e2e_taper_$tp.err; exit 1; }
  echo "taper $tp: $(head -c 200 gpurun_out/e2e_taper_$tp.json)"
done
echo "exit=0"
