"""BGZF inflate throughput: the GPU (ganon_inflate through native.GpuInflater, host buffers in and
out, PCIe included) against zlib on 1..T host threads, over the blocks of a synthetic BAM
(synth/fastpair.py) repeated to --blocks blocks. One JSON line.

    python tools/inflate_bench.py [--blocks 4096] [--iters 5] [--threads 1,8,16]
"""
import argparse
import json
import os
import sys
import tempfile
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def bgzf_blocks(path):
    data = open(path, "rb").read()
    pay, off = [], 0
    while off < len(data):
        xlen = data[off + 10] | (data[off + 11] << 8)
        x, bsize = off + 12, None
        while x < off + 12 + xlen:
            slen = data[x + 2] | (data[x + 3] << 8)
            if data[x] == 66 and data[x + 1] == 67:
                bsize = data[x + 4] | (data[x + 5] << 8)
            x += 4 + slen
        blen = bsize + 1
        n = int.from_bytes(data[off + blen - 4:off + blen], "little")
        if n:
            pay.append((data[off + 12 + xlen:off + blen - 8], n))
        off += blen
    return pay


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--threads", default="1,8,16")
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.fastpair import make_pair
    d = tempfile.mkdtemp(prefix="ganon_inf_")
    paths = make_pair(os.path.join(d, "in"), n_contigs=2, pairs_per_contig=20000)
    bam = paths["T"] if isinstance(paths, dict) else os.path.join(d, "in", "tumor.bam")
    blocks = bgzf_blocks(bam)
    blocks = (blocks * (a.blocks // len(blocks) + 1))[:a.blocks]
    comp = np.frombuffer(b"".join(p for p, _ in blocks), np.uint8)
    in_len = np.array([len(p) for p, _ in blocks], np.int32)
    in_off = np.zeros(len(blocks), np.int64)
    in_off[1:] = np.cumsum(in_len[:-1])
    out_len = np.array([n for _, n in blocks], np.int32)
    out_bytes, comp_bytes = int(out_len.sum()), int(comp.size)
    g = native.GpuInflater(0)
    ref = b"".join(zlib.decompress(p, -15) for p, _ in blocks[:64])
    assert g.inflate(comp, in_off, in_len, out_len)[:len(ref)].tobytes() == ref
    t0 = time.perf_counter()
    for _ in range(a.iters):
        g.inflate(comp, in_off, in_len, out_len)
    gpu_s = (time.perf_counter() - t0) / a.iters
    g.set_profiling(True)
    kms = []
    for _ in range(a.iters):
        g.inflate(comp, in_off, in_len, out_len)
        kms.append(g.kernel_ms())
    g.set_profiling(False)
    kms = float(np.median(kms))
    res = {"blocks": len(blocks), "compressed_MB": round(comp_bytes / 1e6, 1), "inflated_MB": round(out_bytes / 1e6, 1),
           "gpu": {"s": round(gpu_s, 5), "inflated_GB_per_s": round(out_bytes / gpu_s / 1e9, 3),
                   "kernel_ms": round(kms, 3), "kernel_inflated_GB_per_s": round(out_bytes / kms / 1e6, 3),
                   "note": "s: ganon_inflate call: H2D of the payloads, kernel, D2H of the output, host buffers; "
                           "kernel: k_inflate alone (HIP events)"}}
    if not a.no_cpu:
        pays = [p for p, _ in blocks]
        cpu = {}
        for nt in [int(x) for x in a.threads.split(",")]:
            with ThreadPoolExecutor(nt) as ex:
                list(ex.map(lambda p: zlib.decompress(p, -15), pays[:nt * 4]))
                t0 = time.perf_counter()
                list(ex.map(lambda p: zlib.decompress(p, -15), pays, chunksize=16))
                s = time.perf_counter() - t0
            cpu[str(nt)] = {"s": round(s, 4), "inflated_GB_per_s": round(out_bytes / s / 1e9, 3)}
        res["zlib_threads"] = cpu
    g.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
