#!/usr/bin/env python3
"""A/B of the indel tally's strategies on one batch (GPU): the default (short reads: thread walks,
hashed map, in-place segment sort) against GANON_INDEL_SORTMODE=seg|global / GANON_INDEL_WAVE_WALK=1 /
GANON_INDEL_DENSE_MAP=1 (read at indel upload). Prints the record counts and the first differences.

    python tools/indel_ab.py [READS=10000000]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    arr, info = config2_batch(n_reads=n, genome=3_000_000_000 * n // 10_000_000, n_windows=n // 10,
                              n_germline=n // 10, seed=2, read_seed=2000, germline_del_per_kb=0.1,
                              seq_indel_per_base=1.5e-4)
    m = native.HipMasker(0)
    db = m.upload(arr)
    out = {}
    for name, env in (("default", {}), ("segsort", {"GANON_INDEL_SORTMODE": "seg"}),
                      ("globalsort", {"GANON_INDEL_SORTMODE": "global"}),
                      ("wave_walk", {"GANON_INDEL_WAVE_WALK": "1"}), ("dense_map", {"GANON_INDEL_DENSE_MAP": "1"})):
        for k in ("GANON_INDEL_SORTMODE", "GANON_INDEL_WAVE_WALK", "GANON_INDEL_DENSE_MAP"):
            os.environ.pop(k, None)
        os.environ.update(env)
        t = db.indel_tally(arr)
        for _ in range(2):
            t.run()
        out[name] = t.download()
        t.free()
    base = out["default"]
    res = {"reads": info["reads"], "indel_reads": info.get("indel_reads")}
    for name, rec in out.items():
        same = len(rec) == len(base) and np.array_equal(rec, base)
        res[name] = {"records": len(rec), "equal_default": bool(same)}
        if not same:
            a = set(map(tuple, base.tolist())) if base.dtype.names is None else set(base.tolist())
            b = set(rec.tolist())
            res[name]["only_default"] = sorted(a - b)[:5]
            res[name]["only_this"] = sorted(b - a)[:5]
    print(json.dumps(res, default=str))
    db.free()
    m.close()


if __name__ == "__main__":
    main()
