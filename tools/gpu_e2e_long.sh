#!/bin/bash
# The long-read end-to-end line (synth/longpair.py: 10-100 kb paired reads, soft clips, sequencing and
# germline indels; BASELINE configs[4] shape) file to file on the GPU in E2E_WORKERS processes, then the
# same input through the CPU pipeline (the C oracle masking): the files must be equal. One JSON line
# per leg under gpurun_out/e2e_long_{hip,oracle}.json. Each leg has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
D=$(mktemp -d /tmp/ganon_long.XXXXXX)
trap 'rm -rf $D' EXIT
PAIRS=${LONG_PAIRS:-1500}
timeout -k 10 400 python -c "import sys; sys.path.insert(0, '.'); from genomeanonymizer_amd.synth.longpair import make_long_pair; make_long_pair('$D/in', n_contigs=2, contig_len=10_000_000, pairs_per_contig=$PAIRS, seed=11)" || exit 1
echo "generated"
env E2E_RUNS=${E2E_RUNS:-2} E2E_WORKERS=${E2E_WORKERS:-8} timeout -k 10 400 python tools/e2e_bench.py $D/in $D/hip stream > gpurun_out/e2e_long_hip.json 2> gpurun_out/e2e_long_hip.err || { tail -5 gpurun_out/e2e_long_hip.err; exit 1; }
env E2E_ENGINE=oracle E2E_RUNS=0 E2E_WORKERS=${E2E_WORKERS:-8} E2E_THREADS=2 timeout -k 10 600 python tools/e2e_bench.py $D/in $D/oracle stream > gpurun_out/e2e_long_oracle.json 2> gpurun_out/e2e_long_oracle.err || { tail -5 gpurun_out/e2e_long_oracle.err; exit 1; }
python - "$D" <<'PY'
import json, os, sys
d = sys.argv[1]
def last(p):
    return json.loads(open(p).read().strip().splitlines()[-1])["stream"]
h, o = last("gpurun_out/e2e_long_hip.json"), last("gpurun_out/e2e_long_oracle.json")
def rd(p):
    return open(p, "rb").read() if os.path.exists(p) else None
same = all(rd(f"{d}/hip/{x}_stream{s}") == rd(f"{d}/oracle/{x}_stream{s}") for x in ("tumor", "normal")
           for s in (".1.fastq", ".2.fastq", ".single_end.fastq"))
print(json.dumps({"reads": h["reads"], "bases": h["bases"], "reads_per_s": h["reads_per_s"], "bases_per_s": h["bases_per_s"],
                  "wall_s_runs": h["wall_s_runs"], "cpu_s": h["cpu_s"], "oracle_bases_per_s": o["bases_per_s"],
                  "oracle_wall_s": o["stages_s"]["wall_s"], "files_equal_oracle": same}))
PY
echo "exit=0"
