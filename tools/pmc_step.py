#!/usr/bin/env python3
"""HBM bytes per launch of every kernel of one bench step, from tools/gpu_pmc_step.sh's passes.

Read bytes = 32 * RDREQ_32B + 64 * RDREQ_64B + 128 * RDREQ_128B (L2-to-fabric read requests by size,
summed over the L2 channels); write bytes = 64 * WRREQ_64B + 32 * (WRREQ - WRREQ_64B); FETCH_SIZE /
WRITE_SIZE (KB) beside them (on gfx950 FETCH_SIZE tallies 128-B requests at 64 B,
MI355X_MICROARCH.md). Kernels are matched to bench.py's names by substring. ``step_hbm_bytes`` (the
bench's ``roofline.traffic``) sums the kernels of one step: device prep, group kernel, finish and the
indel tally, each at its launches per step.

usage: pmc_step.py TAG CONFIG READS OUT.json      (CONFIG fastq: the formatter's kernels, READS = records)
"""
import collections
import csv
import glob
import json
import os
import re
import sys

# kernels of one fresh-batch step: ganon_batch_replan + ganon_batch_run + ganon_indel_run (the
# reference copies and the record download run at upload / download only)
STEP_KERNELS = {"k_prep_scan", "k_prep_cands", "k_prep_order_count", "k_prep_order_scatter", "k_prep_scan_long", "k_prep_reduce", "k_prep_nseg", "k_prep_scope_cost", "k_prep_groups", "k_prep_emit", "k_prep_emit_flat", "k_prep_emit_waves", "k_prep_long_groups",
                "k_prep_long_mid", "k_prep_read_recs", "k_prep_linemap", "k_prep_pieces", "k_group", "k_finish", "k_tile_large",
                "k_mask_large", "k_indel_mark", "k_indel_count", "k_indel_emit", "k_indel_segs", "k_indel_runs",
                "k_indel_rcount", "k_indel_remit", "k_indel_icount", "k_indel_expand", "k_indel_mark_t",
                "k_indel_rlist_t", "k_indel_icount_t", "k_indel_expand_t", "k_indel_tsort",
                "k_indel_classify", "rocprim_sort", "rocprim_scan", "rocprim_other"}


def short(name: str) -> str:
    m = re.search(r"\b(k_[A-Za-z0-9_]+)", name)
    if m:
        return m.group(1)
    if "rocprim" in name:
        return "rocprim_sort" if ("sort" in name or "radix" in name) else "rocprim_scan" if "scan" in name \
            else "rocprim_other"
    return name[:60]


def main():
    tag, config, reads, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    tot = collections.defaultdict(float)
    n = collections.Counter()
    # per-dispatch WRITE_SIZE of the memsets (hipMemsetAsync -> fillBufferAligned) and the group
    # kernel's dispatch count: the step's memsets (plan flags, candidates, line map) per step
    fills, n_group = [], 0
    for d in glob.glob(f"gpurun_out/pmc_{tag}_p*"):
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                key = (short(r["Kernel_Name"]), r["Counter_Name"])
                tot[key] += float(r["Counter_Value"])
                n[key] += 1
                if r["Counter_Name"] == "WRITE_SIZE":
                    if "fillBuffer" in r["Kernel_Name"]:
                        fills.append(float(r["Counter_Value"]) * 1024)
                    elif key[0] == "k_group":
                        n_group += 1
    kern = collections.defaultdict(dict)
    for (k, c), v in tot.items():
        kern[k][c] = v / n[(k, c)]
    # launches per step from the kernel trace (the PMC runs use --steps 3 --warmup 1 = 4 runs + 1 for
    # the profiled pass, so counts per launch are means; launches per step from the stats run)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from genomeanonymizer_amd.build import sources_digest
    # the kernels these counters describe: bench.py cites the summary only while the digest matches
    kind = "fastq" if config == "fastq" else "mask"   # (fastq: tools/gpu_pmc_fastq.sh, the formatter's kernels)
    res = {"config": config, "reads": reads, "sources_digest": sources_digest(kind), "kernels": {}}
    step = 0.0
    for k, vals in sorted(kern.items()):
        rd = 32 * vals.get("TCC_EA0_RDREQ_32B", 0) + 64 * vals.get("TCC_EA0_RDREQ_64B", 0) + \
            128 * vals.get("TCC_EA0_RDREQ_128B", 0)
        wr64 = vals.get("TCC_EA0_WRREQ_64B", 0)
        wr = 64 * wr64 + 32 * (vals.get("TCC_EA0_WRREQ", 0) - wr64)
        res["kernels"][k] = {"hbm_read_bytes_per_launch": int(rd), "hbm_write_bytes_per_launch": int(wr),
                             "hbm_bytes_per_launch": int(rd + wr), "fetch_size_kb": vals.get("FETCH_SIZE"),
                             "write_size_kb": vals.get("WRITE_SIZE"), "counters_per_launch": vals}
        if (k.startswith("k_fq") if kind == "fastq" else k in STEP_KERNELS):
            step += rd + wr
    # the step's memsets: fills under 64 MB (the upload's output-buffer clear is ~0.75 GB) over the
    # group kernel's dispatches (one per step); the upload's small clears are counted too (an upper bound)
    memset = sum(b for b in fills if b < 64 * 2 ** 20) / n_group if n_group else 0.0
    res["memset_bytes_per_step"] = int(memset)
    step += memset
    res["step_hbm_bytes"] = int(step)
    res["step_kernels"] = sorted(k for k in res["kernels"]
                                 if (k.startswith("k_fq") if kind == "fastq" else k in STEP_KERNELS))
    res["method"] = ("TCC_EA0_RDREQ_{32B,64B,128B} x size + TCC_EA0_WRREQ{,_64B}; three rocprofv3 --pmc passes "
                     "(tools/gpu_pmc_step.sh) over bench.py --steps 3, mean over dispatches; step = the kernels of "
                     "one fresh-batch step, replan + run + indel tally (step_kernels), one launch each, plus "
                     "memset_bytes_per_step (WRITE_SIZE of the fills under 64 MB per group-kernel dispatch)")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v["hbm_bytes_per_launch"] for k, v in res["kernels"].items()}))
    print("step_hbm_bytes", res["step_hbm_bytes"])


if __name__ == "__main__":
    main()
