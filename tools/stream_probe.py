#!/usr/bin/env python3
"""Fresh-batch steps of S resident configs[1] batches, each in its own context on its own HIP
stream, issued round-robin (speculative replans: no host synchronization): how much of one batch's
plan overlaps another's group kernel. Prints ms per batch for S = 1..max.

    python tools/stream_probe.py [max_streams] [steps]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch
    smax = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    arr, _ = config2_batch(n_reads=10_000_000, genome=3_000_000_000, n_windows=1_000_000, n_germline=1_000_000, seed=2)
    body = {k: v for k, v in arr.items() if k != "ref_nt16"}
    ctxs = []
    for s in range(smax):
        m = native.HipMasker(0)
        st = torch.cuda.Stream()
        m.set_stream(st.cuda_stream)
        ref = m.upload_reference(arr["ref_nt16"])
        db = m.upload(body, ref=ref)
        ctxs.append((m, st, ref, db))
    out = {}
    for S in range(1, smax + 1):
        use = ctxs[:S]
        for i in range(10):
            _, _, _, db = use[i % S]
            db.replan()
            db.run()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(steps):
            _, _, _, db = use[i % S]
            db.replan()
            db.run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / steps * 1e3
        out[str(S)] = {"ms_per_batch": round(ms, 4), "reads_per_s": round(1e7 / (ms * 1e-3), 1)}
        print(json.dumps({"streams": S, **out[str(S)]}), file=sys.stderr, flush=True)
    # every batch's result still equals the first's
    ref_tot = None
    for m, st, ref, db in ctxs:
        tot = db.totals()
        ref_tot = tot if ref_tot is None else ref_tot
        assert (tot == ref_tot).all()
    for m, st, ref, db in ctxs:
        db.free()
        ref.free()
        m.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
