cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for p in 3 4 2 3; do
  timeout -k 10 400 python bench.py --no-e2e --no-side-configs --no-cpu-baseline --no-pcie --no-fastq --steps 100 --warmup 10 --pipeline $p > gpurun_out/pipe_$p.json 2> gpurun_out/pipe_$p.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/pipe_$p.json').read().strip().splitlines()[-1]); print($p, d['ms_per_step'], d['one_stream_ms_per_step'], d['sync_plan_ms_per_step'])"
done
