#!/usr/bin/env python3
"""Profiling driver for the FASTQ formatter alone: config-2 record set (10 M reads, names of
30-45 characters, half reverse), uploaded from host buffers, formatted RUNS times, the
kernel times printed as one JSON line. Usage: python3 tools/fq_run.py [--reads N] [--runs R]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--configs", default="0:0",
                    help="comma list of kd:skip (GANON_PARAM_FASTQ_KD / _SKIP), timed interleaved")
    a = ap.parse_args()
    import numpy as np
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch
    from genomeanonymizer_amd.synth.fastq import fastq_records
    arr, _ = config2_batch(n_reads=a.reads, genome=max(60_000_000, a.reads * 300), seed=2)
    recs = fastq_records(arr, seed=11, name_len=(30, 45), check_bad=False)
    m = native.HipMasker(0)
    f = m.fastq_upload(recs)
    f.run()
    f.sync()
    cfgs = [tuple(int(x) for x in c.split(":")) for c in a.configs.split(",")]
    m.set_profiling(True)
    per = {c: [] for c in cfgs}
    for _ in range(a.runs):
        for c in cfgs:
            m.set_param(native.PARAM_FASTQ_KD, c[0])
            m.set_param(native.PARAM_FASTQ_SKIP, c[1])
            f.run()
            f.sync()
            per[c].append({k: ms for k, _, ms in f.kernel_times()})
    m.set_profiling(False)
    m.set_param(native.PARAM_FASTQ_KD, cfgs[0][0])
    m.set_param(native.PARAM_FASTQ_SKIP, 0)
    times = per[cfgs[0]]
    t = time.perf_counter()
    for _ in range(a.runs):
        f.run()
    f.sync()
    wall = (time.perf_counter() - t) / a.runs * 1e3
    out = f.download()
    ok = len(out) == native.fastq_bytes(recs)
    f.free()
    print(json.dumps({"reads": a.reads, "bytes": len(out), "ok": ok, "wall_ms": round(wall, 4),
                      "kernel_ms": {f"{c[0]}:{c[1]}": {k: round(float(np.median([t[k] for t in ts])), 4)
                                                       for k in ts[0]} for c, ts in per.items()}}))


if __name__ == "__main__":
    main()
