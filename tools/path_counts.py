#!/usr/bin/env python3
"""The group kernel's rarer paths on a bench configuration (ganon_batch_path_counts): lists of more
than 256 observations sorted in LDS, lists classified from the group's global overflow region, key
range splits — with the group count and the distribution of incidences per group.

    python tools/path_counts.py c3 [reads genome windows germline]
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
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    a = [int(x) for x in sys.argv[2:6]] if len(sys.argv) > 5 else (
        [10_000_000, 25_000_000, 2500, 25000] if cfg == "c3" else [10_000_000, 3_000_000_000, 1_000_000, 1_000_000])
    kw = dict(n_reads=a[0], genome=a[1], n_windows=a[2], n_germline=a[3], seed=3 if cfg == "c3" else 2)
    if cfg == "c3":
        kw.update(n_contigs=4, window_spacing=10_000)
    arr, info = config2_batch(**kw)
    inc = np.diff(arr["scope_incid_off"])
    m = native.HipMasker(0)
    db = m.upload(arr)
    db.run()
    db.download()
    out = {"config": cfg, "reads": a[0], "groups": db.info()["groups"], "paths": db.path_counts(),
           "scopes": int(len(inc)), "incidences_per_scope_pct": {str(p): float(np.percentile(inc, p)) for p in (50, 90, 99, 100)},
           "scopes_over_1000_incidences": int((inc > 1000).sum())}
    db.free()
    m.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
