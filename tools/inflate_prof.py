"""Where k_inflate's cycles go (tuning): run with a -DINF_PROF build of libganon_hip.so
(tools/build_variant.py prof -DINF_PROF; GANON_HIP_LIB=<that .so>) over the bench blocks of
tools/inflate_bench.py; prints the summed s_memtime cycles of round fill / chain / emit against the
blocks' total, per inflated byte."""
import ctypes as C
import json
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tools.inflate_bench import bgzf_blocks  # noqa: E402


def main():
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.fastpair import make_pair
    d = tempfile.mkdtemp(prefix="ganon_infp_")
    make_pair(os.path.join(d, "in"), n_contigs=2, pairs_per_contig=20000)
    blocks = bgzf_blocks(os.path.join(d, "in", "tumor.bam"))
    blocks = (blocks * (4096 // len(blocks) + 1))[:4096]
    comp = np.frombuffer(b"".join(p for p, _ in blocks), np.uint8)
    in_len = np.array([len(p) for p, _ in blocks], np.int32)
    in_off = np.zeros(len(blocks), np.int64)
    in_off[1:] = np.cumsum(in_len[:-1])
    out_len = np.array([n for _, n in blocks], np.int32)
    g = native.GpuInflater(0)
    lib = native.hip_lib()
    fn = lib.ganon_inflate_prof_read
    buf = (C.c_ulonglong * 6)()
    g.inflate(comp, in_off, in_len, out_len)
    fn(buf)
    g.inflate(comp, in_off, in_len, out_len)
    fn(buf)
    tot = int(out_len.sum())
    names = ["fill", "chain", "emit", "block_total", "rounds", "unused"]
    res = {n: int(v) for n, v in zip(names, buf)}
    res["per_byte"] = {n: round(int(v) / tot, 3) for n, v in zip(names[:4], buf)}
    res["bytes_per_round"] = round(tot / max(1, res["rounds"]), 1)
    res["note"] = "s_memtime units summed over waves; block_total - fill - chain - emit = scalar path, headers, refills"
    print(json.dumps(res))
    g.close()


if __name__ == "__main__":
    main()
