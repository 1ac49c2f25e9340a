#!/usr/bin/env python3
"""Per-kernel HBM traffic from the PMC passes of tools/gpu_profile.sh.

Read bytes = 32 * RDREQ_32B + 64 * RDREQ_64B + 128 * RDREQ_128B (L2-to-fabric read requests by
size, summed over the L2 channels); write bytes = 64 * WRREQ_64B + 32 * (WRREQ - WRREQ_64B).
FETCH_SIZE / WRITE_SIZE (KB) are reported beside them: on gfx950 FETCH_SIZE tallies 128-B
requests at 64 B (MI355X_MICROARCH.md, HBM/rocprofv3), which the request-size split avoids.
Infinity-Cache hits are counted as fabric traffic by these counters.

usage: pmc_summary.py TAG KERNEL_SUBSTRING BENCH_KERNEL_NAME READS OUT.json
"""
import collections
import csv
import glob
import json
import sys


def per_kernel(path):
    rows = list(csv.DictReader(open(path)))
    tot, n = collections.defaultdict(float), collections.Counter()
    for r in rows:
        key = (r["Kernel_Name"], r["Counter_Name"])
        tot[key] += float(r["Counter_Value"])
        n[key] += 1
    return {k: tot[k] / n[k] for k in tot}


def main():
    tag, sub, bench_name, reads, out = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
    vals = {}
    for d in glob.glob(f"gpurun_out/pmc_{tag}_*"):
        f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
        if not f:
            continue
        for (kname, cname), v in per_kernel(f[0]).items():
            if sub in kname:
                vals[cname] = v
    rd = 32 * vals.get("TCC_EA0_RDREQ_32B", 0) + 64 * vals.get("TCC_EA0_RDREQ_64B", 0) + \
        128 * vals.get("TCC_EA0_RDREQ_128B", 0)
    wr64 = vals.get("TCC_EA0_WRREQ_64B", 0)
    wr = 64 * wr64 + 32 * (vals.get("TCC_EA0_WRREQ", 0) - wr64)
    res = {"kernel": bench_name, "rocprof_kernel_substring": sub, "reads": reads,
           "hbm_read_bytes_per_launch": int(rd), "hbm_write_bytes_per_launch": int(wr),
           "hbm_bytes_per_launch": int(rd + wr),
           "fetch_size_kb": vals.get("FETCH_SIZE"), "write_size_kb": vals.get("WRITE_SIZE"),
           "counters_per_launch": vals,
           "method": "TCC_EA0_RDREQ_{32B,64B,128B} x size + TCC_EA0_WRREQ{,_64B}; one rocprofv3 --pmc pass "
                     "per counter over bench.py --steps 3 (tools/gpu_profile.sh), mean over dispatches"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
