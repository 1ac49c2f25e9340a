#!/bin/bash
# Formatter A/B on a GPU box: every formatter GPU test (all kernel variants), then the 10 M-record
# configs[1] record set formatted by each variant, interleaved (tools/fq_run.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fastq.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fq.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fq.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fq_run.py --runs 7 --configs ${FQ_CONFIGS:-0:0,13:0,14:0,15:0} > gpurun_out/fq_ab.json 2> gpurun_out/fq_ab.err
rc=$?; tail -c 600 gpurun_out/fq_ab.err; cat gpurun_out/fq_ab.json; exit $rc
