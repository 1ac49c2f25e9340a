#!/usr/bin/env python3
"""Masking kernel time on the bench's interleaved synthetic layout against the product path's
dataset-major sequence buffer (every tumor read, then every normal read: build_batch), and the
masked outputs compared read by read. Usage: python3 tools/layout_ab.py [--reads N] [--config c2]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reads", type=int, default=None)
    ap.add_argument("--genome", type=int, default=None)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import bench
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import dataset_major
    a.windows = a.germline = None
    for k, v in bench.CONFIGS[a.config]["defaults"].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    a.batches = a.pipeline = 1   # (one batch of the configured size)
    arr, _ = bench.make_batch(a, 0, 0)
    dm = dataset_major(arr)
    m = native.HipMasker(0)
    res = {}
    outs = {}
    for name, x in (("interleaved", arr), ("dataset_major", dm)):
        db = m.upload(x)
        m.set_profiling(True)
        times = []
        for _ in range(a.steps):
            db.run()
            db.sync()
            times.append({n: ms / l for n, l, ms in db.kernel_times()})
        m.set_profiling(False)
        res[name] = {k: round(float(np.median([t[k] for t in times])), 5) for k in times[0]}
        o, calls, bases, tot = db.download()
        res[name]["totals"] = tot.tolist()
        nb = (x["read_len"].astype(np.int64) + 1) // 2
        outs[name] = (o, x["seq_off"].astype(np.int64), nb)
        db.free()
    (o1, s1, n1), (o2, s2, n2) = outs["interleaved"], outs["dataset_major"]
    same = all(np.array_equal(o1[s1[i]:s1[i] + n1[i]], o2[s2[i]:s2[i] + n2[i]])
               for i in np.random.default_rng(0).choice(len(n1), size=min(len(n1), 20000), replace=False))
    res["same_reads_sample"] = bool(same)
    res["same_totals"] = res["interleaved"].pop("totals") == res["dataset_major"].pop("totals")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
