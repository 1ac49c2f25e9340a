#!/bin/bash
# GPU-box A/B of bench configurations: each line "TAG|ENV|ARGS" of $AB_SPEC runs
# `env ENV python bench.py ARGS` into gpurun_out/ab_TAG.json, under its own time limit; the chain
# stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
while IFS='|' read -r TAG ENVS ARGS; do
  [ -z "$TAG" ] && continue
  echo "== $TAG"
  env $ENVS timeout -k 10 400 python bench.py $ARGS > gpurun_out/ab_$TAG.json 2> gpurun_out/ab_$TAG.err || { echo "fail $TAG"; tail -5 gpurun_out/ab_$TAG.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$TAG.json')); print('$TAG', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['pass']['kernels'].items()})"
done <<< "$AB_SPEC"
echo "exit=0"
