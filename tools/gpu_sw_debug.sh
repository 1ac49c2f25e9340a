#!/bin/bash
# Scan-store debugging: the key-range-split dense test under bisect builds (tools/build_variant.py
# bisN -DGANON_SW_BISECT=N) and the current build. Each run has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sw_dbg
T="tests/test_gpu.py::test_dense_scopes_match_oracle"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u -m pytest "$T" -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/sw_dbg/$name.log 2>&1
  echo "$name rc=$? $(grep -E 'passed|failed' gpurun_out/sw_dbg/$name.log | tail -1) $(grep -E 'array\(\[' gpurun_out/sw_dbg/$name.log | head -1 | cut -c1-160)"
}
for i in 1 2; do
  for v in ${VARIANTS:-bis1 bis2 bis4 bis7}; do
    run ${v}_$i GANON_HIP_LIB=genomeanonymizer_amd/variants/libganon_hip_$v.so
    run ${v}_off_$i GANON_SCAN_STORE=0 GANON_HIP_LIB=genomeanonymizer_amd/variants/libganon_hip_$v.so
  done
done
run cur GANON_SCAN_STORE=1
echo done
