#!/bin/bash
# k_prep_scan reads-per-thread A/B (round 6): c2 and c2id bench lines on the default build (U = 4)
# and on variant builds (tools/build_variant.py suN -DGANON_SCAN_U=N), alternated. Each step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/scanu_ab
A="--steps ${STEPS:-50} --warmup 5 --no-cpu-baseline --no-pcie --no-fastq --no-e2e --no-side-configs"
V=genomeanonymizer_amd/variants
for rep in 1 2; do
  for u in 4 ${VARIANTS:-2 6 8}; do
    for cfg in c2 c2id; do
      case $cfg in c2id) X="--config c2id" ;; *) X="" ;; esac
      if [ "$u" = 4 ]; then LIB=""; else LIB="$V/libganon_hip_su$u.so"; fi
      GANON_HIP_LIB=$LIB timeout -k 10 300 python bench.py $A $X > gpurun_out/scanu_ab/${cfg}_u${u}_$rep.json \
        2> gpurun_out/scanu_ab/${cfg}_u${u}_$rep.err || { tail -20 gpurun_out/scanu_ab/${cfg}_u${u}_$rep.err; exit 1; }
      python3 - "$cfg" "$u" "$rep" <<'EOF'
import json, sys
cfg, u, rep = sys.argv[1:]
d = json.loads(open(f"gpurun_out/scanu_ab/{cfg}_u{u}_{rep}.json").read().strip().splitlines()[-1])
k = d["pass"]["kernels"]
print(cfg, "U", u, "rep", rep, "ms/step", d["ms_per_step"], "one_stream", d.get("one_stream_ms_per_step"),
      "prep_scan", round(k.get("prep_scan", {}).get("avg_ms", 0), 4),
      "k_group", round(k.get("k_group_fused", {}).get("avg_ms", 0), 4), flush=True)
EOF
    done
  done
done
echo "exit=0"
