#!/bin/bash
# A/B of GANON_INDEL_FORK (the indel tally on a side stream beside the group kernel) on the c2id and
# c5 lines: the indel GPU tests with the fork on, then child bench runs of each setting.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fork_ab
GANON_INDEL_FORK=1 timeout -k 10 400 python -u -m pytest tests/test_indels.py tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "indel or c2id or full_size or long" > gpurun_out/fork_ab/tests.log 2>&1 || { tail -20 gpurun_out/fork_ab/tests.log; exit 1; }
tail -1 gpurun_out/fork_ab/tests.log
B="--no-e2e --no-pcie --no-fastq --no-cpu-baseline --no-side-configs --no-bam-decode"
for cfg in c2id c5; do
  if [ $cfg = c5 ]; then X="--reads 10000 --genome 100000000 --steps 5 --warmup 2"; else X="--steps 20 --warmup 5"; fi
  for f in 0 1 0 1; do
    GANON_INDEL_FORK=$f timeout -k 10 300 python bench.py --config $cfg $B $X > gpurun_out/fork_ab/${cfg}_fork$f.json 2> gpurun_out/fork_ab/${cfg}_fork$f.err || { tail -5 gpurun_out/fork_ab/${cfg}_fork$f.err; exit 1; }
    echo "$cfg fork=$f: $(python -c "import json; d=json.loads(open('gpurun_out/fork_ab/${cfg}_fork$f.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('one_stream_ms_per_step'))")"
  done
done
echo "exit=0"
