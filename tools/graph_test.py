#!/usr/bin/env python3
"""Timed-loop experiment (profiling aid): ms per ganon_batch_run on the config-2 batch when
launched eagerly vs replayed from a captured HIP graph (torch.cuda.CUDAGraph around the
run on torch's capture stream), and eagerly with a sync every step."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from genomeanonymizer_amd import native
    import argparse
    a = argparse.Namespace(config="c2", reads=None, genome=None, windows=None, germline=None)
    for k, v in bench.CONFIGS["c2"]["defaults"].items():
        setattr(a, k, v)
    a.batches = a.pipeline = 1   # (one batch of the configured size)
    arr, info = bench.make_batch(a, 0, 0)
    m = native.HipMasker(0)
    torch.cuda.set_device(0)
    m.set_stream(torch.cuda.current_stream().cuda_stream)
    db = m.upload(arr)
    steps = int(os.environ.get("STEPS", "100"))
    res = {}

    def timed(fn, name, sync_each=False):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            fn()
            if sync_each:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        res[name] = round((time.perf_counter() - t) / steps * 1e3, 4)

    timed(db.run, "eager")
    timed(db.run, "eager_sync_each", sync_each=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m.set_stream(s.cuda_stream)
        db.run()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m.set_stream(torch.cuda.current_stream().cuda_stream)
        db.run()
    m.set_stream(torch.cuda.current_stream().cuda_stream)
    timed(g.replay, "graph")
    timed(db.run, "eager_again")
    tot = db.totals()
    res["totals"] = [int(x) for x in tot]
    db.free()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
