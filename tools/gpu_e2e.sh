#!/bin/bash
# End-to-end runs on the GPU box: one synthetic pair (synth/fastpair.py, $E2E_CONTIGS contigs), then
# the product timed (tools/e2e_bench.py, modes $E2E_MODES) once per line "TAG|ENV" of $E2E_SPEC
# (default: one run, tag "base"), each with a cProfile of its main thread
# (gpurun_out/e2e_prof_TAG_<mode>.txt) and its JSON in gpurun_out/e2e_TAG.json. Each step has its
# own time limit; the chain stops at the first failure. DECODE_SCALING=1 first runs
# tools/decode_scaling.py on the same pair.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
D=$(mktemp -d /tmp/ganon_e2e.XXXXXX)
trap 'rm -rf $D' EXIT
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '.'); from genomeanonymizer_amd.synth.fastpair import make_pair; make_pair('$D/in', n_contigs=${E2E_CONTIGS:-24}, pairs_per_contig=${E2E_PAIRS:-23000})" || exit 1
if [ -n "$DECODE_SCALING" ]; then
  timeout -k 10 300 python tools/decode_scaling.py $D/in > gpurun_out/decode_scaling.json 2> gpurun_out/decode_scaling.err || exit 1
  cat gpurun_out/decode_scaling.json
fi
while IFS='|' read -r TAG ENVS; do
  [ -z "$TAG" ] && continue
  echo "== $TAG"
  env $ENVS E2E_PROFILE=gpurun_out/e2e_prof_$TAG E2E_RUNS=${E2E_RUNS:-2} timeout -k 10 600 \
    python tools/e2e_bench.py $D/in $D/out ${E2E_MODES:-stream} > gpurun_out/e2e_$TAG.json 2> gpurun_out/e2e_$TAG.err \
    || { echo "fail $TAG"; tail -5 gpurun_out/e2e_$TAG.err; exit 1; }
  cat gpurun_out/e2e_$TAG.json
done <<< "${E2E_SPEC:-base|}"
echo "exit=0"
