#!/usr/bin/env python3
"""Host BAM decode scaling: BGZF inflate (zlib, libganon_host.so) + BAM -> SoA of
every contig of a tumor/normal pair, as the streamed product reads them (io.bam.BamReader.contig),
at 1, 2, 4, 8 and 16 inflate threads, in one process and in P processes (each its share of the
contigs and 16 / P threads, as the multi-process product runs). Prints one JSON line: reads/s and
inflated MB/s per setting, the host's CPU model and core counts.

    python tools/decode_scaling.py DIR     # DIR: tumor.bam normal.bam ref.fa (synth/fastpair.py)
"""
import json
import multiprocessing as mp
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _decode(d: str, threads: int, contigs) -> tuple:
    from genomeanonymizer_amd.io.bam import BamReader
    readers = [BamReader(os.path.join(d, f), threads, 0) for f in ("tumor.bam", "normal.bam")]
    n = nbytes = 0
    t = time.perf_counter()
    for c in contigs:
        for r in readers:
            tab = r.contig(r.tid_of(c))
            n += tab.n
            nbytes += int(tab.l_seq.astype("int64").sum()) * 2 + int(tab.name_len.astype("int64").sum())
    dt = time.perf_counter() - t
    for r in readers:
        r.close()
    return n, nbytes, dt


def _worker(args):
    return _decode(*args)


def main():
    d = sys.argv[1]
    from genomeanonymizer_amd.io.fasta import FastaRef
    contigs = list(FastaRef(os.path.join(d, "ref.fa")).references)
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    comp = sum(os.path.getsize(os.path.join(d, f)) for f in ("tumor.bam", "normal.bam"))
    out = {"host": {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "cpu_model": model},
           "compressed_bytes": comp, "contigs": len(contigs), "one_process": {}, "processes": {}}
    _decode(d, 4, contigs[:1])   # page cache warm
    for t in (1, 2, 4, 8, 16):
        n, nb, dt = _decode(d, t, contigs)
        out["one_process"][str(t)] = {"reads_per_s": round(n / dt, 1), "seq_qual_name_MB_per_s": round(nb / dt / 1e6, 1),
                                      "compressed_MB_per_s": round(comp / dt / 1e6, 1), "s": round(dt, 3)}
        print(json.dumps({"threads": t, **out["one_process"][str(t)]}), file=sys.stderr, flush=True)
    ctx = mp.get_context("spawn")
    for p in (2, 4, 8):
        shards = [contigs[i::p] for i in range(p)]
        t0 = time.perf_counter()
        with ctx.Pool(p) as pool:
            res = pool.map(_worker, [(d, max(1, 16 // p), s) for s in shards])
        wall = max(r[2] for r in res)
        n = sum(r[0] for r in res)
        out["processes"][str(p)] = {"threads_each": max(1, 16 // p), "reads_per_s": round(n / wall, 1),
                                    "compressed_MB_per_s": round(comp / wall / 1e6, 1), "slowest_s": round(wall, 3),
                                    "pool_wall_s": round(time.perf_counter() - t0, 3)}
        print(json.dumps({"processes": p, **out["processes"][str(p)]}), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
