#!/bin/bash
# End-to-end profile on the GPU box: a synthetic pair (synth/fastpair.py, $E2E_CONTIGS contigs),
# the streamed product timed (tools/e2e_bench.py) with a cProfile of the main thread; each step
# under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
D=$(mktemp -d /tmp/ganon_e2e.XXXXXX)
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '.'); from genomeanonymizer_amd.synth.fastpair import make_pair; make_pair('$D/in', n_contigs=${E2E_CONTIGS:-24})" \
 && E2E_PROFILE=gpurun_out/e2e_prof E2E_RUNS=${E2E_RUNS:-2} timeout -k 10 600 python tools/e2e_bench.py $D/in $D/out ${E2E_MODES:-stream} > gpurun_out/e2e.json 2> gpurun_out/e2e.err
rc=$?
rm -rf $D
cat gpurun_out/e2e.json
tail -5 gpurun_out/e2e.err
exit $rc
