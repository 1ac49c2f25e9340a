#!/usr/bin/env python3
"""Sweep the group kernel's tuning knobs (GANON_PARAM_GROUP_UNROLL, GANON_PARAM_GROUP_TARGET) on one
bench configuration: the batch is generated and uploaded once, each setting is timed over K steps of
``ganon_batch_run`` (device prep + masking), with per-kernel HIP-event times; totals must agree.

    python tools/sweep_group.py c3 [K]     # prints one JSON line per setting, then the best
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import argparse
    import numpy as np
    import torch
    import bench
    from genomeanonymizer_amd import native
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    args = argparse.Namespace(config=cfg, **bench.CONFIGS[cfg]["defaults"])
    # SWEEP_SHAPE="reads=10000000,genome=25000000,...": the shape of a bench side line instead of the
    # config's defaults; SWEEP_TARGETS / SWEEP_UNROLL: comma lists for the grid
    for kv in filter(None, os.environ.get("SWEEP_SHAPE", "").split(",")):
        k, v = kv.split("=")
        setattr(args, k, int(v))
    args.batches = args.pipeline = 1   # (one batch of the configured size)
    arr, _ = bench.make_batch(args, 0, 0)
    m = native.HipMasker(0)
    ref = m.upload_reference(arr["ref_nt16"])
    mode = sys.argv[3] if len(sys.argv) > 3 else "grid"
    tl = [int(x) for x in os.environ.get("SWEEP_TARGETS", "352,704,1408").split(",")]
    ul = [int(x) for x in os.environ.get("SWEEP_UNROLL", "1,2,4").split(",")]
    settings = [(u, t) for t in tl for u in ul] if mode == "grid" else [(0, 0)]
    obs_list = (512, 1024) if mode == "obs" else (0,)
    pu_list = (1, 2, 4) if mode == "prep" else (0,)
    if mode == "prep":
        obs_list = pu_list
    ref_tot, best, db, cur_t = None, None, None, None
    for (u, t), obs in [(x, o) for x in settings for o in obs_list]:
        if mode == "prep":
            m.set_param(native.PARAM_PREP_UNROLL, obs)
        else:
            m.set_param(native.PARAM_GROUP_OBS, obs)
        m.set_param(native.PARAM_GROUP_UNROLL, u)
        if t != cur_t:                   # the target applies at upload
            if db is not None:
                db.free()
            m.set_param(native.PARAM_GROUP_TARGET, t)
            db = m.upload({k: v for k, v in arr.items() if k != "ref_nt16"}, ref=ref)
            cur_t = t
        for _ in range(3):
            db.run()
        db.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            db.run()
        db.sync()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        m.set_profiling(True)
        kt = {}
        for _ in range(5):
            db.run()
            db.sync()
            for name, n, k_ms in db.kernel_times():
                kt[name] = kt.get(name, 0.0) + k_ms / 5
        m.set_profiling(False)
        tot = db.totals()[:2].tolist()
        ref_tot = ref_tot or tot
        line = {"config": cfg, "unroll": u, "target": t, "obs": obs, "ms_per_step": round(ms, 4),
                "kernels_ms": {k: round(v, 4) for k, v in kt.items()}, "totals": tot, "same": tot == ref_tot}
        print(json.dumps(line), flush=True)
        if best is None or ms < best[0]:
            best = (ms, u, t)
    print(json.dumps({"best": {"ms_per_step": round(best[0], 4), "unroll": best[1], "target": best[2]}}))
    db.free()
    ref.free()


if __name__ == "__main__":
    main()
