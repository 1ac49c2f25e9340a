#!/bin/bash
# Phase timing of the group kernel, then PMC passes (one counter set per pass, no tracing
# domains) over a short phase_timing run. Each GPU step has its own time limit.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$REPO"
mkdir -p gpurun_out
TAG=${TAG:-r01}
CFG=${CFG:-4:1:0}
timeout -k 10 300 python3 tools/phase_timing.py ${PHASE_ARGS:-} > gpurun_out/phase_$TAG.json 2> gpurun_out/phase_$TAG.err \
 && timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    -d gpurun_out/pmc_sq_$TAG -o run --output-format csv -- \
    python3 tools/phase_timing.py --rounds 1 --steps 2 --configs $CFG > /dev/null 2> gpurun_out/pmc_sq_$TAG.err \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- \
    python3 tools/phase_timing.py --rounds 1 --steps 2 --configs $CFG > /dev/null 2> gpurun_out/pmc_fetch_$TAG.err \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- \
    python3 tools/phase_timing.py --rounds 1 --steps 2 --configs $CFG > /dev/null 2> gpurun_out/pmc_write_$TAG.err
rc=$?
echo "exit=$rc"
cat gpurun_out/phase_$TAG.json
exit $rc
