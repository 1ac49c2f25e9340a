"""Tile a generated sample: k renamed copies of every contig (reads, reference, windows).

Test infrastructure (the bounded-memory and sharding tests need samples with many contigs,
faster than synth.generate can write them): copy j of contig c is named ``{c}_{j}``; its records
are the originals with tid / mate tid remapped and ``_{j}`` appended to the read name (so names
stay disjoint between copies), written in coordinate order with a .bai.
"""
from __future__ import annotations

import gzip
import os
import struct
from typing import Dict, List, Tuple

from .bamwriter import BgzfWriter, _write_bai


def _read_bam(path: str):
    data = gzip.open(path, "rb").read()
    assert data[:4] == b"BAM\x01"
    l_text = struct.unpack_from("<i", data, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", data, p)[0]
    p += 4
    refs = []
    for _ in range(n_ref):
        ln = struct.unpack_from("<i", data, p)[0]
        name = data[p + 4:p + 4 + ln - 1].decode()
        L = struct.unpack_from("<i", data, p + 4 + ln)[0]
        refs.append((name, L))
        p += 8 + ln
    recs = []
    while p < len(data):
        bs = struct.unpack_from("<i", data, p)[0]
        recs.append(data[p + 4:p + 4 + bs])
        p += 4 + bs
    return refs, recs


def _retag(body: bytes, tid_map, suffix: bytes) -> Tuple[bytes, int, int, int, int]:
    tid, pos = struct.unpack_from("<ii", body, 0)
    l_rn = body[8]
    mtid = struct.unpack_from("<i", body, 20)[0]
    flag = struct.unpack_from("<H", body, 14)[0]
    ncig = struct.unpack_from("<H", body, 12)[0]
    name = body[32:32 + l_rn - 1] + suffix + b"\x00"
    nt = tid_map(tid)
    nm = tid_map(mtid)
    head = bytearray(body[:32])
    struct.pack_into("<i", head, 0, nt)
    head[8] = len(name)
    struct.pack_into("<i", head, 20, nm)
    rest = body[32 + l_rn:]
    rlen = 0
    for k in range(ncig):
        w = struct.unpack_from("<I", rest, 4 * k)[0]
        if (w & 0xF) in (0, 2, 3, 7, 8):
            rlen += w >> 4
    end = pos + (rlen if (rlen > 0 and not flag & 4) else 1)
    return bytes(head) + name + rest, nt, pos, end, flag


def tile_sample(paths: Dict[str, str], copies: int, outdir: str) -> Dict[str, str]:
    os.makedirs(outdir, exist_ok=True)
    out = {}
    refs = None
    for key, fn in (("T", "tumor.bam"), ("N", "normal.bam")):
        refs, recs = _read_bam(paths[key])
        n = len(refs)
        new_refs = [(f"{name}_{j}", L) for name, L in refs for j in range(copies)]
        by_tid: List[List[bytes]] = [[] for _ in range(n)]
        unplaced = []
        for r in recs:
            t = struct.unpack_from("<i", r, 0)[0]
            (by_tid[t] if t >= 0 else unplaced).append(r)
        text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join(f"@SQ\tSN:{a}\tLN:{b}\n" for a, b in new_refs)
        hdr = b"BAM\x01" + struct.pack("<i", len(text)) + text.encode() + struct.pack("<i", len(new_refs))
        for a, b in new_refs:
            nb = a.encode() + b"\x00"
            hdr += struct.pack("<i", len(nb)) + nb + struct.pack("<i", b)
        path = os.path.join(outdir, fn)
        w = BgzfWriter(path)
        w.write(hdr)
        spans = []
        for t in range(n):
            for j in range(copies):
                tmap = (lambda x, j=j: x * copies + j if x >= 0 else -1)
                sfx = f"_{j}".encode()
                for r in by_tid[t]:
                    body, nt, pos, end, flag = _retag(r, tmap, sfx)
                    v0 = w.tell_virtual()
                    w.write(struct.pack("<i", len(body)) + body)
                    spans.append((nt, pos, end, v0, w.tell_virtual(), bool(flag & 4)))
        for j in range(copies):
            tmap = (lambda x, j=j: x * copies + j if x >= 0 else -1)
            for r in unplaced:
                body, *_ = _retag(r, tmap, f"_{j}".encode())
                w.write(struct.pack("<i", len(body)) + body)
        w.close()
        _write_bai(path + ".bai", len(new_refs), spans)
        out[key] = path
    # reference
    seqs = []
    name, buf = None, []
    for line in open(paths["ref"]).read().splitlines():
        if line.startswith(">"):
            if name is not None:
                seqs.append((name, "".join(buf)))
            name, buf = line[1:].split()[0], []
        else:
            buf.append(line)
    if name is not None:
        seqs.append((name, "".join(buf)))
    from .bamwriter import write_fasta, write_vcf
    write_fasta(os.path.join(outdir, "ref.fa"), [(f"{a}_{j}", s) for a, s in seqs for j in range(copies)])
    vrecs = []
    for line in open(paths["vcf"]):
        if line.startswith("#"):
            continue
        f = line.rstrip("\n").split("\t")
        vrecs.append(f)
    order = {a: i for i, (a, _) in enumerate(seqs)}
    new_v = [(f"{f[0]}_{j}", int(f[1]), f[2] + f"_{j}", f[3], f[4]) for f in vrecs for j in range(copies)]
    new_v.sort(key=lambda r: (order[r[0].rsplit("_", 1)[0]] * copies + int(r[0].rsplit("_", 1)[1]), r[1]))
    write_vcf(os.path.join(outdir, "variants.vcf"), [(f"{a}_{j}", len(s)) for a, s in seqs for j in range(copies)],
              new_v)
    out.update(ref=os.path.join(outdir, "ref.fa"), vcf=os.path.join(outdir, "variants.vcf"))
    return out
