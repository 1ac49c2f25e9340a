#!/usr/bin/env python3
"""Phase timing of the group kernels on the config-2 batch (profiling aid, not a test).

Runs ganon_batch_run (device prep + masking) with HIP-event timing for each configuration
variant:unroll:skip[:group_target[:nt_copy[:ref2]]], interleaved over several rounds, and prints one
JSON object of median per-kernel times. skip != 0 leaves phases out (GANON_PARAM_GROUP_SKIP)
and gives invalid results: timing only. group_target is applied at upload (one upload per
distinct target).
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", help="bench.py workload (c2, c3, c5)")
    ap.add_argument("--reads", type=int, default=None)
    ap.add_argument("--genome", type=int, default=None)
    ap.add_argument("--windows", type=int, default=None)
    ap.add_argument("--germline", type=int, default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--configs", default="0:1:0,0:2:0,0:2:1,0:2:2,0:2:4",
                    help="comma list of variant:unroll:skip[:group_target[:nt_copy[:ref2]]]")
    args = ap.parse_args()
    from genomeanonymizer_amd import native
    import bench
    for k, v in bench.CONFIGS[args.config]["defaults"].items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    args.batches = args.pipeline = 1   # (one batch of the configured size)
    arr, info = bench.make_batch(args, 0, 0)
    m = native.HipMasker(0)
    cfgs = []
    for c in args.configs.split(","):
        f = [int(x) for x in c.split(":")]
        f += [704, 1, 1][len(f) - 3:] if len(f) < 6 else []
        cfgs.append(tuple(f[:6]))
    dbs = {}
    for c in cfgs:
        if c[3] not in dbs:
            m.set_param(native.PARAM_GROUP_TARGET, c[3])
            dbs[c[3]] = m.upload(arr)
    m.set_profiling(True)
    res = {c: {} for c in cfgs}
    for _ in range(args.rounds):
        for c in cfgs:
            v, u, sk, tgt, nt, r2 = c
            m.set_variant(v)
            m.set_param(native.PARAM_GROUP_UNROLL, u)
            m.set_param(native.PARAM_GROUP_SKIP, sk)
            m.set_param(native.PARAM_NT_COPY, nt)
            m.set_param(native.PARAM_REF2, r2)
            db = dbs[tgt]
            for _ in range(args.steps):
                db.run()
                db.sync()
                for name, launches, ms in db.kernel_times():
                    res[c].setdefault(name, []).append(ms / launches)
    m.set_param(native.PARAM_GROUP_SKIP, 0)
    out = {f"v{v}_k{u}_skip{sk}_t{tgt}_nt{nt}_ref2{r2}": {n: round(float(np.median(x)), 5) for n, x in d.items()}
           for (v, u, sk, tgt, nt, r2), d in res.items()}
    out["batch"] = next(iter(dbs.values())).info()
    for db in dbs.values():
        db.free()
    m.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
