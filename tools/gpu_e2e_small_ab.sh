#!/bin/bash
# The bench's 24-contig end-to-end pair (synth/fastpair.py defaults of bench.py), 8 processes on the
# GPU, A/B of the secondary exchange (GANON_SEC_EXCHANGE=0 / default) and of E2E_RUNS timed runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
D=$(mktemp -d /tmp/ganon_small.XXXXXX)
trap 'rm -rf $D' EXIT
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '.'); from genomeanonymizer_amd.synth.fastpair import make_pair; make_pair('$D/in', n_contigs=24, pairs_per_contig=23000)" || exit 1
for x in 1 0; do
  GANON_SEC_EXCHANGE=$x E2E_RUNS=3 E2E_WORKERS=8 timeout -k 10 300 python tools/e2e_bench.py $D/in $D/out stream > gpurun_out/e2e_small_x$x.json 2> gpurun_out/e2e_small_x$x.err || { tail -5 gpurun_out/e2e_small_x$x.err; exit 1; }
done
echo "exit=0"
