#!/bin/bash
# The 30x chromosome-scale end-to-end line (tools/gpu_e2e_chrom.sh's input) once per "NAME=VALUE"
# environment setting given as arguments ("-" = none): A/B of a switch. One JSON line per run under
# gpurun_out/e2e_ab_<i>.json. Each run has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
D=$(mktemp -d /tmp/ganon_chrom.XXXXXX)
trap 'rm -rf $D' EXIT
timeout -k 10 400 python -c "import sys; sys.path.insert(0, '.'); from genomeanonymizer_amd.synth.fastpair import make_pair; make_pair('$D/in', n_contigs=2, contig_len=20_000_000, pairs_per_contig=2_000_000, window_every=20_000, seed=9)" || exit 1
echo "generated"
i=0
for kv in "$@"; do
  i=$((i + 1))
  if [ "$kv" = "-" ]; then ENVSET=""; else ENVSET="$kv"; fi
  env $ENVSET E2E_DIGEST=${E2E_DIGEST:-1} E2E_RUNS=${E2E_RUNS:-2} E2E_WORKERS=${E2E_WORKERS:-8} timeout -k 10 400 python tools/e2e_bench.py $D/in $D/out stream > gpurun_out/e2e_ab_$i.json 2> gpurun_out/e2e_ab_$i.err || { tail -5 gpurun_out/e2e_ab_$i.err; exit 1; }
  echo "$kv: $(python -c "import json,sys; s=json.loads(open('gpurun_out/e2e_ab_$i.json').read().strip().splitlines()[-1])['stream']; d=json.loads(open('gpurun_out/e2e_ab_$i.json').read().strip().splitlines()[-1]); print(s['reads_per_s'], s['wall_s_runs'], s['cpu_s'], s['cores_busy'], d.get('output_sha1', '')[:12], (s.get('decode_phases_rank0') or {}).get('device_regions'), (s.get('decode_phases_rank0') or {}).get('device_fallbacks'))")"
done
echo "exit=0"
