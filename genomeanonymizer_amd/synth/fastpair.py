"""Fast synthetic tumor/normal pair: BAM + BAI, FASTA + .fai, window VCF, samples.tsv.

Benchmark infrastructure (bench.py's end-to-end line, tools/e2e_bench.py): the product never
writes BAM. Vectorised numpy (no per-read Python), BGZF blocks compressed on a thread pool, so a
~2 M-read pair takes seconds instead of the minutes of the per-read generator (synth/generate.py,
which stays the source of the golden scenarios). Written from the SAM/BAM v1 specification.

Content (BASELINE configs[1] style): ``n_contigs`` contigs of random ACGT; per contig
a het germline SNP per ``1000 / snp_per_kb`` bases and a 1-3 bp het germline deletion per
``1000 / del_per_kb`` bases (both carried by haplotype 2, in the tumor AND the normal reads: the
germline variants the path masks); a somatic SNV window variant every ``window_every`` bases from
5,000 (the VCF; tumor reads carry it at AF 0.4); FR pairs with insert N(300, 30), flags 99/147 or
83/163, 0.1 % substitution errors, phred uniform in [2, 40], a 5-20 base soft clip on 2 % of the
reads; tumor and normal read names disjoint. ``sec_frac``: that fraction of the pairs of
every contig also has a secondary alignment of its read 1 (flag 0x100, 150M, the read's bases) at a
random position of another contig, its mate fields naming the primary mate — the aligner output
that makes the streamed path plan a job again when another rank decodes the secondary.
"""
from __future__ import annotations

import os
import struct
import zlib
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Tuple

import numpy as np

_CODE = np.array([1, 2, 4, 8], np.uint8)            # A C G T as nt16
_ASCII = np.frombuffer(b"ACGT", np.uint8)
_BGZF_BLOCK = 0xFF00
_BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
_HDR = np.dtype([("bs", "<i4"), ("ref", "<i4"), ("pos", "<i4"), ("lrn", "u1"), ("mapq", "u1"), ("bin", "<u2"),
                 ("ncig", "<u2"), ("flag", "<u2"), ("lseq", "<i4"), ("nref", "<i4"), ("npos", "<i4"),
                 ("tlen", "<i4")])
assert _HDR.itemsize == 36


def reg2bin(beg: np.ndarray, end: np.ndarray) -> np.ndarray:
    """SAM spec §5.3, vectorised: bin of [beg, end)."""
    e = end - 1
    out = np.zeros(len(beg), np.int64)
    done = np.zeros(len(beg), bool)
    for shift, base in ((14, 4681), (17, 585), (20, 73), (23, 9), (26, 1)):
        m = ~done & ((beg >> shift) == (e >> shift))
        out[m] = base + (beg[m] >> shift)
        done |= m
    return out


class _Contig:
    def __init__(self, rng, length: int, snp_per_kb: float, del_per_kb: float, window_every: int):
        self.length = length
        self.ref = rng.integers(0, 4, length, dtype=np.uint8)           # 0..3 = ACGT
        n_snp = int(length * snp_per_kb / 1000)
        snp = np.unique(rng.integers(300, length - 300, n_snp))
        self.alt = np.full(length, 255, np.uint8)                          # haplotype-2 SNP alts
        self.alt[snp] = (self.ref[snp] + rng.integers(1, 4, len(snp))) % 4
        grid = np.arange(1000, length - 1000, 400)
        n_del = min(len(grid), int(length * del_per_kb / 1000))
        self.dels = np.sort(rng.choice(grid, n_del, replace=False)) if n_del else np.zeros(0, np.int64)
        self.del_len = rng.integers(1, 4, len(self.dels))
        self.alt[self.dels] = 255                                          # no SNP at a deletion start
        self.windows = np.arange(5000, length - 2500, window_every)
        self.som = np.full(length, 255, np.uint8)                          # tumor-only window SNVs
        self.som[self.windows] = (self.ref[self.windows] + 1) % 4
        self.alt[self.windows] = 255


def _reads(rng, c: _Contig, n_pairs: int, read_len: int, tumor: bool, err: float, clip_frac: float):
    """Aligned reads of one sample on one contig: positions, CIGARs (up to 3 ops), bases, flags."""
    L = c.length
    frag = rng.integers(0, L - 800, n_pairs)
    ins = np.clip(rng.normal(300, 30, n_pairs).astype(np.int64), 2 * read_len // 3 + 100, 480)
    hap = rng.integers(0, 2, n_pairs)
    som = rng.random(n_pairs) < 0.4
    left_first = rng.random(n_pairs) < 0.5
    n = 2 * n_pairs
    pos = np.empty(n, np.int64)
    pos[0::2] = frag
    pos[1::2] = frag + ins - read_len
    hap2 = np.repeat(hap, 2)
    som2 = np.repeat(som, 2) & tumor
    # a haplotype-2 read that starts inside a deletion starts after it; one deletion strictly inside
    # a read gives aM dD bM
    k = np.searchsorted(c.dels, pos, side="right") - 1
    inside_del = (hap2 == 1) & (k >= 0) & (pos < c.dels[np.maximum(k, 0)] + c.del_len[np.maximum(k, 0)]) & \
        (pos >= c.dels[np.maximum(k, 0)]) if len(c.dels) else np.zeros(n, bool)
    if np.any(inside_del):
        pos[inside_del] = c.dels[k[inside_del]] + c.del_len[k[inside_del]]
    nxt = np.searchsorted(c.dels, pos, side="right")
    has_del = (hap2 == 1) & (nxt < len(c.dels))
    dpos = np.where(has_del, c.dels[np.minimum(nxt, len(c.dels) - 1)] if len(c.dels) else 0, 0)
    has_del &= dpos < pos + read_len - 1
    a = np.where(has_del, dpos - pos, read_len)
    dl = np.where(has_del, c.del_len[np.minimum(nxt, max(len(c.dels) - 1, 0))] if len(c.dels) else 0, 0)
    clip = np.where((~has_del) & (rng.random(n) < clip_frac), rng.integers(5, 21, n), 0)
    # bases: the reference windows (a row copy per read), then the few reads with a clip or a
    # deletion rebuilt, then the sparse variant sites and errors
    win = np.lib.stride_tricks.sliding_window_view(c.ref, read_len + 3)
    base = win[np.minimum(pos, L - read_len - 3)][:, :read_len].copy()
    odd = np.nonzero(has_del | (clip > 0))[0]
    if len(odd):
        q = np.arange(read_len)[None, :]
        po, ao, do, co = pos[odd, None], a[odd, None], dl[odd, None], clip[odd, None]
        rp = po + q - co + np.where(q >= ao, do, 0)
        b = c.ref[np.clip(rp, 0, L - 1)]
        cl = q < co
        b[cl] = rng.integers(0, 4, int(cl.sum()))
        base[odd] = b
    end = pos + read_len - clip + dl

    def apply(sites: np.ndarray, allele: np.ndarray, who: np.ndarray) -> None:
        """Put allele[site] at every base of a read of `who` aligned to a site."""
        if not len(sites) or not np.any(who):
            return
        rr = np.nonzero(who)[0]
        lo = np.searchsorted(sites, pos[rr])
        hi = np.searchsorted(sites, end[rr])
        cnt = hi - lo
        if not cnt.sum():
            return
        ri = np.repeat(rr, cnt)
        si = sites[np.repeat(lo, cnt) + (np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt))]
        qq = si - pos[ri] + clip[ri]
        after = has_del[ri] & (si >= pos[ri] + a[ri])
        inside = has_del[ri] & (si >= pos[ri] + a[ri]) & (si < pos[ri] + a[ri] + dl[ri])
        qq = np.where(after, qq - dl[ri], qq)
        ok = ~inside & (qq >= clip[ri]) & (qq < read_len)
        base[ri[ok], qq[ok]] = allele[si[ok]]
    apply(np.nonzero(c.alt != 255)[0], c.alt, hap2 == 1)
    apply(c.windows, c.som, som2)
    n_err = rng.binomial(n * read_len, err)
    e = rng.integers(0, n * read_len, n_err)
    flat = base.reshape(-1)
    flat[e] = (flat[e] + rng.integers(1, 4, n_err).astype(np.uint8)) % 4
    # CIGAR words (len << 4 | op): [cS] M or aM dD bM
    cig = np.zeros((n, 3), np.uint32)
    ncig = np.ones(n, np.int64)
    plain = ~has_del & (clip == 0)
    cig[plain, 0] = read_len << 4
    cm = clip > 0
    cig[cm, 0] = (clip[cm] << 4) | 4
    cig[cm, 1] = (read_len - clip[cm]) << 4
    ncig[cm] = 2
    cig[has_del, 0] = a[has_del] << 4
    cig[has_del, 1] = (dl[has_del] << 4) | 2
    cig[has_del, 2] = (read_len - a[has_del]) << 4
    ncig[has_del] = 3
    # flags: pair i is (left, right); read 1 is the left one or the right one
    flag = np.empty(n, np.int64)
    r1_left = np.repeat(left_first, 2)
    left = np.tile([True, False], n_pairs)
    is_r1 = left == r1_left
    flag[:] = 1 | 2 | np.where(is_r1, 0x40, 0x80) | np.where(left, 0x20, 0x10)
    mate = np.arange(n) ^ 1
    tlen = np.where(left, end[mate] - pos, -(end - pos[mate]))
    return pos, end, cig, ncig, base, flag, mate, tlen


def _encode(tid: int, pos, end, cig, ncig, base, flag, mpos, tlen, names: np.ndarray, qual, mtid=None) -> bytes:
    """BAM records (fixed read and name length) back to back (``mtid``: per-record mate
    reference, default the record's own)."""
    n, read_len = base.shape
    nl = names.shape[1] + 1
    size = 36 + nl + 4 * ncig + (read_len + 1) // 2 + read_len
    hdr = np.zeros(n, _HDR)
    hdr["bs"] = size - 4
    hdr["ref"] = tid
    hdr["pos"] = pos
    hdr["lrn"] = nl
    hdr["mapq"] = 60
    hdr["bin"] = reg2bin(pos, end)
    hdr["ncig"] = ncig
    hdr["flag"] = flag
    hdr["lseq"] = read_len
    hdr["nref"] = tid if mtid is None else mtid
    hdr["npos"] = mpos
    hdr["tlen"] = tlen
    codes = _CODE[base]
    if read_len & 1:
        codes = np.concatenate([codes, np.zeros((n, 1), np.uint8)], axis=1)
    packed = (codes[:, 0::2] << 4) | codes[:, 1::2]
    width = 36 + nl + 12 + packed.shape[1] + read_len
    rows = np.zeros((n, width), np.uint8)
    rows[:, :36] = hdr.view(np.uint8).reshape(n, 36)
    rows[:, 36:36 + nl - 1] = names
    c0 = 36 + nl
    cg = cig.view(np.uint8).reshape(n, 12)
    tail = np.concatenate([packed, qual], axis=1)
    # cigar bytes, then seq + qual right after the record's own cigar
    rows[:, c0:c0 + 12] = cg
    idx = c0 + 4 * ncig[:, None] + np.arange(tail.shape[1])[None, :]
    np.put_along_axis(rows, idx, tail, axis=1)
    mask = np.arange(width)[None, :] < size[:, None]
    return rows[mask].tobytes()


def _bgzf(data: bytes, level: int, pool: ThreadPoolExecutor) -> Tuple[List[bytes], np.ndarray]:
    chunks = [data[i:i + _BGZF_BLOCK] for i in range(0, len(data), _BGZF_BLOCK)]

    def block(payload: bytes) -> bytes:
        comp = zlib.compressobj(level, zlib.DEFLATED, -15)
        z = comp.compress(payload) + comp.flush()
        head = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, len(z) + 25)
        return head + z + struct.pack("<II", zlib.crc32(payload) & 0xFFFFFFFF, len(payload))
    blocks = list(pool.map(block, chunks))
    coff = np.concatenate([[0], np.cumsum([len(b) for b in blocks])]).astype(np.int64)
    return blocks, coff


def _voff(u: np.ndarray, coff: np.ndarray) -> np.ndarray:
    k = u // _BGZF_BLOCK
    return (coff[k] << 16) | (u % _BGZF_BLOCK)


def _bai(path: str, n_ref: int, tids, pos, end, v0, v1) -> None:
    out = [b"BAI\x01", struct.pack("<i", n_ref)]
    for t in range(n_ref):
        sel = np.nonzero(tids == t)[0]
        if not len(sel):
            out.append(struct.pack("<ii", 0, 0))
            continue
        p, e, a, b = pos[sel], end[sel], v0[sel], v1[sel]
        bins = reg2bin(p, e)
        order = np.lexsort((np.arange(len(sel)), bins))
        bo, ao, zo = bins[order], a[order], b[order]
        new = np.ones(len(order), bool)
        new[1:] = (bo[1:] != bo[:-1]) | (ao[1:] != zo[:-1])
        starts = np.nonzero(new)[0]
        ends = np.concatenate([starts[1:], [len(order)]]) - 1
        ub, first_chunk = np.unique(bo[starts], return_index=True)
        n_chunks = np.diff(np.concatenate([first_chunk, [len(starts)]]))
        parts = [struct.pack("<i", len(ub) + 1)]
        for bi, f, nc in zip(ub.tolist(), first_chunk.tolist(), n_chunks.tolist()):
            parts.append(struct.pack("<Ii", bi, nc))
            ch = np.stack([ao[starts[f:f + nc]], zo[ends[f:f + nc]]], axis=1).astype("<u8")
            parts.append(ch.tobytes())
        parts.append(struct.pack("<Ii", 37450, 2) + struct.pack("<QQ", int(a[0]), int(b[-1])) +
                     struct.pack("<QQ", len(sel), 0))
        w0, w1 = p >> 14, (e - 1) >> 14
        n_intv = int(w1.max()) + 1
        lin = np.full(n_intv, np.iinfo(np.int64).max, np.int64)
        np.minimum.at(lin, w0, a)
        np.minimum.at(lin, w1, a)
        lin[lin == np.iinfo(np.int64).max] = 0
        lin = np.maximum.accumulate(lin)      # empty windows take the previous offset
        parts.append(struct.pack("<i", n_intv) + lin.astype("<u8").tobytes())
        out.extend(parts)
    out.append(struct.pack("<Q", 0))
    with open(path, "wb") as fh:
        fh.write(b"".join(out))


def _write_bam(path: str, contigs: List[Tuple[str, int]], per_contig, level: int, pool) -> int:
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join(f"@SQ\tSN:{n}\tLN:{l}\n" for n, l in contigs)
    hdr = b"BAM\x01" + struct.pack("<i", len(text)) + text.encode() + struct.pack("<i", len(contigs))
    for n, l in contigs:
        nb = n.encode() + b"\x00"
        hdr += struct.pack("<i", len(nb)) + nb + struct.pack("<i", l)
    parts, starts, sizes, tids, poss, ends = [hdr], [], [], [], [], []
    u = len(hdr)
    for tid, (blob, sz, pos, end) in enumerate(per_contig):
        off = u + np.concatenate([[0], np.cumsum(sz)[:-1]])
        starts.append(off)
        sizes.append(sz)
        tids.append(np.full(len(sz), tid, np.int64))
        poss.append(pos)
        ends.append(end)
        parts.append(blob)
        u += len(blob)
    data = b"".join(parts)
    blocks, coff = _bgzf(data, level, pool)
    with open(path, "wb") as fh:
        for b in blocks:
            fh.write(b)
        fh.write(_BGZF_EOF)
    st = np.concatenate(starts)
    sz = np.concatenate(sizes)
    _bai(path + ".bai", len(contigs), np.concatenate(tids), np.concatenate(poss), np.concatenate(ends),
         _voff(st, coff), _voff(st + sz, coff))
    return len(st)


def write_reference(outdir: str, names: List[str], contigs: List[_Contig]) -> Dict[str, str]:
    """ref.fa (+ .fai), the window VCF and samples.tsv of a synthetic pair; the paths, with the BAM
    paths the caller writes."""
    paths = {"ref": os.path.join(outdir, "ref.fa"), "vcf": os.path.join(outdir, "variants.vcf"),
             "T": os.path.join(outdir, "tumor.bam"), "N": os.path.join(outdir, "normal.bam")}
    # FASTA (60 columns) + .fai
    fai, off = [], 0
    with open(paths["ref"], "wb") as fh:
        for nm, c in zip(names, contigs):
            head = f">{nm}\n".encode()
            fh.write(head)
            off += len(head)
            fai.append(f"{nm}\t{c.length}\t{off}\t60\t61\n")
            seq = _ASCII[c.ref]
            full = (len(seq) // 60) * 60
            body = np.concatenate([seq[:full].reshape(-1, 60), np.full((full // 60, 1), 10, np.uint8)], axis=1).tobytes()
            if full < len(seq):
                body += seq[full:].tobytes() + b"\n"
            fh.write(body)
            off += len(body)
    with open(paths["ref"] + ".fai", "w") as fh:
        fh.write("".join(fai))
    with open(paths["vcf"], "w") as fh:
        fh.write("##fileformat=VCFv4.2\n")
        for nm, c in zip(names, contigs):
            fh.write(f"##contig=<ID={nm},length={c.length}>\n")
        fh.write("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n")
        for nm, c in zip(names, contigs):
            r = _ASCII[c.ref[c.windows]].tobytes().decode()
            a = _ASCII[c.som[c.windows]].tobytes().decode()
            fh.write("".join(f"{nm}\t{p + 1}\tsom{i}\t{r[i]}\t{a[i]}\t.\tPASS\t.\n"
                             for i, p in enumerate(c.windows.tolist())))
    with open(os.path.join(outdir, "samples.tsv"), "w") as fh:
        fh.write("#tumor\tnormal\tvcf\ntumor.bam\tnormal.bam\tvariants.vcf\n")
    return paths


def make_pair(outdir: str, n_contigs: int = 24, contig_len: int = 2_000_000, pairs_per_contig: int = 23_000,
              read_len: int = 150, seed: int = 7, snp_per_kb: float = 1.0, del_per_kb: float = 0.1,
              window_every: int = 20_000, err: float = 0.001, clip_frac: float = 0.02, level: int = 1,
              threads: int = 16, sec_frac: float = 0.0) -> Dict[str, str]:
    os.makedirs(outdir, exist_ok=True)
    rng = np.random.default_rng(seed)
    names = [f"chr{i + 1}" for i in range(n_contigs)]
    contigs = [_Contig(rng, contig_len, snp_per_kb, del_per_kb, window_every) for _ in names]
    paths = write_reference(outdir, names, contigs)
    with ThreadPoolExecutor(threads) as pool:
        for tag, tumor in (("T", True), ("N", False)):
            recs = []   # per contig: the record columns, secondaries from other contigs appended below
            for tid, c in enumerate(contigs):
                pos, end, cig, ncig, base, flag, mate, tlen = _reads(rng, c, pairs_per_contig, read_len, tumor, err,
                                                                     clip_frac)
                pair_id = np.arange(len(pos)) // 2
                nm = np.frombuffer(b"".join(f"{tag}{tid:03d}:{p:08d}".encode() for p in range(pairs_per_contig)),
                                   np.uint8).reshape(pairs_per_contig, -1)[pair_id]
                qual = rng.integers(2, 41, base.shape, dtype=np.uint8)
                recs.append({"pos": pos, "end": end, "cig": cig, "ncig": ncig, "base": base, "flag": flag,
                             "mpos": pos[mate], "tlen": tlen, "nm": nm, "qual": qual,
                             "mtid": np.full(len(pos), tid, np.int64)})
            if sec_frac > 0 and len(contigs) > 1:
                add = [[] for _ in contigs]
                for tid, r in enumerate(recs):
                    k = int(pairs_per_contig * sec_frac)
                    i = 2 * rng.choice(pairs_per_contig, k, replace=False)
                    i = np.where(r["flag"][i] & 0x40, i, i + 1)          # the pair's read 1
                    dst = (tid + 1 + rng.integers(0, len(contigs) - 1, k)) % len(contigs)
                    for t in np.unique(dst).tolist():
                        sel = i[dst == t]
                        L = contigs[t].length
                        sp = rng.integers(0, L - read_len - 1, len(sel))
                        cg = np.zeros((len(sel), 3), np.uint32)
                        cg[:, 0] = read_len << 4
                        add[t].append({"pos": sp, "end": sp + read_len, "cig": cg, "ncig": np.ones(len(sel), np.int64),
                                       "base": r["base"][sel], "flag": r["flag"][sel] | 0x100,
                                       "mpos": r["mpos"][sel], "tlen": np.zeros(len(sel), np.int64),
                                       "nm": r["nm"][sel], "qual": r["qual"][sel],
                                       "mtid": np.full(len(sel), tid, np.int64)})
                for t, extra in enumerate(add):
                    if extra:
                        recs[t] = {k: np.concatenate([recs[t][k]] + [e[k] for e in extra]) for k in recs[t]}
            per = []
            for tid, r in enumerate(recs):
                o = np.argsort(r["pos"], kind="stable")
                blob = _encode(tid, r["pos"][o], r["end"][o], r["cig"][o], r["ncig"][o], r["base"][o], r["flag"][o],
                               r["mpos"][o], r["tlen"][o], r["nm"][o], r["qual"][o], r["mtid"][o])
                nl = r["nm"].shape[1] + 1
                sz = 36 + nl + 4 * r["ncig"][o] + (read_len + 1) // 2 + read_len
                per.append((blob, sz, r["pos"][o], r["end"][o]))
            _write_bam(paths[tag], [(n, c.length) for n, c in zip(names, contigs)], per, level, pool)
    return paths
