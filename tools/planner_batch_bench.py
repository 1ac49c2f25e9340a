#!/usr/bin/env python3
"""The masking step on a batch the product planner derived from BAMs (the
headline's config2_batch synthesises its scopes directly).

DIR holds tumor.bam normal.bam ref.fa variants.vcf (tools/e2e_data.py). The whole sample is decoded
and planned by the native planner, laid out by anonymizer_methods.build_batch exactly as the product
does, uploaded once with the genome resident, and one step (ganon_batch_run: device prep + masking)
is timed over K runs with per-kernel HIP-event times; the same is done for a config2_batch of the same
read count for comparison. One JSON line.

    python tools/planner_batch_bench.py DIR [K]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def step(m, arr, k):
    ref = m.upload_reference(arr["ref_nt16"])
    db = m.upload({x: v for x, v in arr.items() if x != "ref_nt16"}, ref=ref)
    for _ in range(3):
        db.run()
    db.sync()
    t0 = time.perf_counter()
    for _ in range(k):
        db.run()
    db.sync()
    ms = (time.perf_counter() - t0) * 1e3 / k
    m.set_profiling(True)
    kt = {}
    for _ in range(5):
        db.run()
        db.sync()
        for name, n, k_ms in db.kernel_times():
            kt[name] = kt.get(name, 0.0) + k_ms / 5
    m.set_profiling(False)
    info = db.info()
    db.free()
    ref.free()
    return ms, kt, info


def main():
    import numpy as np
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.anonymizer_methods import build_batch
    from genomeanonymizer_amd.io.bam import ReadTable
    from genomeanonymizer_amd.io.fasta import FastaRef
    from genomeanonymizer_amd.io.vcf import read_vcf
    from genomeanonymizer_amd.planner import NativeSamplePlanner, get_windows
    from genomeanonymizer_amd.synth.batch import config2_batch
    d = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    fasta = FastaRef(os.path.join(d, "ref.fa"))
    windows = get_windows(read_vcf(os.path.join(d, "variants.vcf")), dict(fasta.index))
    T, N = ReadTable(os.path.join(d, "tumor.bam")), ReadTable(os.path.join(d, "normal.bam"))
    t0 = time.time()
    planner = NativeSamplePlanner(T, N, fasta, windows)
    plan = planner.run()
    arr, meta = build_batch(plan, (T, N), fasta)
    t_plan = time.time() - t0
    m = native.HipMasker(0)
    n_reads = len(arr["read_len"])
    ms, kt, info = step(m, arr, k)
    written = int((arr["write_scope"] >= 0).sum())
    out = {"planner_batch": {"reads": n_reads, "bam_reads": int(T.n + N.n), "scopes": len(plan.scopes),
                             "incidences": int(len(arr["incid_read"])), "written_reads": written,
                             "genome_bp": int(sum(fasta.lengths)), "plan_and_layout_s": round(t_plan, 2),
                             "ms_per_step": round(ms, 4), "reads_per_s": round(n_reads / ms * 1e3, 1),
                             "kernels_ms": {x: round(v, 4) for x, v in kt.items()}, "batch": info}}
    syn, sinfo = config2_batch(n_reads=n_reads, genome=int(sum(fasta.lengths)),
                               n_windows=len(windows), n_germline=len(windows), seed=2)
    ms2, kt2, info2 = step(m, syn, k)
    out["config2_batch_same_size"] = {"reads": len(syn["read_len"]), "scopes": len(syn["scope_span_len"]),
                                      "incidences": int(len(syn["incid_read"])),
                                      "written_reads": int((syn["write_scope"] >= 0).sum()),
                                      "ms_per_step": round(ms2, 4), "reads_per_s": round(len(syn["read_len"]) / ms2 * 1e3, 1),
                                      "kernels_ms": {x: round(v, 4) for x, v in kt2.items()}, "batch": info2}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
