#!/bin/bash
# Large-contig end-to-end check on the GPU box: two 40 Mb contigs with 1.5 M pairs each per sample
# (12 M reads, chromosome-scale jobs: one device batch of ~3 M reads per contig and sample pair),
# streamed product in one process (contig mode) and in E2E_WORKERS processes (job mode); files
# compared between the two.
# Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
D=$(mktemp -d /tmp/ganon_big.XXXXXX)
trap 'rm -rf $D' EXIT
timeout -k 10 400 python -c "import sys; sys.path.insert(0, '.'); from genomeanonymizer_amd.synth.fastpair import make_pair; make_pair('$D/in', n_contigs=2, contig_len=40_000_000, pairs_per_contig=1_500_000, window_every=20_000)" || exit 1
echo "generated"; ls -la $D/in
# (the one-process leg: E2E_WORKERS unset whatever the caller exported, and contig mode — one job
# per contig, GANON_JOB_BP=0 — an independent plan of the same files)
env -u E2E_WORKERS GANON_JOB_BP=0 E2E_RUNS=1 timeout -k 10 400 python tools/e2e_bench.py $D/in $D/out1 stream > gpurun_out/e2e_big_w1.json 2> gpurun_out/e2e_big_w1.err || { tail -5 gpurun_out/e2e_big_w1.err; exit 1; }
cat gpurun_out/e2e_big_w1.json
E2E_RUNS=1 E2E_WORKERS=${E2E_WORKERS:-2} timeout -k 10 400 python tools/e2e_bench.py $D/in $D/outw stream > gpurun_out/e2e_big_w.json 2> gpurun_out/e2e_big_w.err || { tail -5 gpurun_out/e2e_big_w.err; exit 1; }
cat gpurun_out/e2e_big_w.json
for f in tumor_stream.1.fastq tumor_stream.2.fastq normal_stream.1.fastq normal_stream.2.fastq tumor_stream.single_end.fastq normal_stream.single_end.fastq; do
  cmp -s $D/out1/$f $D/outw/$f && echo "same $f" || { echo "DIFF $f"; exit 1; }
done
echo "exit=0"
