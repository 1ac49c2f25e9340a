"""Synthetic long-read tumor/normal pair (BASELINE configs[4] shape, file to file): BAM + BAI, FASTA
+ .fai, window VCF, samples.tsv.

Benchmark infrastructure (bench.py's long-read end-to-end line): the product never writes BAM.
The reference runs ONT pairs through the same driver as short reads
(short_read_tumor_normal_anonymizer.py:625-760); its per-read work is the CIGAR walk of
anonymizer_methods.py:431-535 over reads of 10-100 kb. Contigs, germline SNPs and deletions and
window variants are synth/fastpair.py's (_Contig); the reads are long and irregular:

* pairs whose reads have independent lengths, log-normal around ``mean_len``, clipped to
  [``min_len``, ``max_len``]; read 2 starts a N(1000, 300) gap after read 1's reference end; flags
  99/147 or 83/163 as in fastpair;
* a leading soft clip (20-300 bases) on ``clip_frac`` of the reads;
* sequencing insertions and deletions (1-3 bases) at ``indel_rate`` per base, plus every germline
  deletion of haplotype 2 a read spans: CIGARs of tens to hundreds of S / M / I / D ops;
* substitution errors at ``err`` per base (each one a pileup observation for the masking path),
  phred uniform in [2, 40]; tumor reads carry the window variants at AF 0.4.

Per-read numpy (reads are few and long), BGZF on a thread pool. Written from the SAM/BAM v1
specification.
"""
from __future__ import annotations

import os
import struct
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Tuple

import numpy as np

from .fastpair import _CODE, _HDR, _Contig, _write_bam, reg2bin, write_reference


def _read(rng, c: _Contig, p: int, q_len: int, hap: int, som: bool, err: float, indel_rate: float,
          clip_frac: float) -> Tuple[int, int, np.ndarray, np.ndarray]:
    """One read of query length q_len aligned from reference position p: (pos, end, CIGAR words,
    bases 0..3)."""
    clip = int(rng.integers(20, 301)) if rng.random() < clip_frac else 0
    a = q_len - clip                                   # aligned query bases (M + I)
    is_ins = np.zeros(a, bool)
    for _ in range(int(rng.poisson(a * indel_rate / 2))):
        k = int(rng.integers(10, a - 13))
        is_ins[k:k + int(rng.integers(1, 4))] = True
    n_m = int(a - is_ins.sum())
    # reference positions of the M bases: one apart, plus the sequencing deletions, plus haplotype 2's
    # germline deletions where the read spans them
    jump = np.zeros(n_m, np.int64)
    n_del = int(rng.poisson(a * indel_rate / 2))
    if n_del:
        at = rng.integers(10, n_m - 10, n_del)
        np.add.at(jump, at, rng.integers(1, 4, n_del))
    refpos = p + np.arange(n_m, dtype=np.int64) + np.cumsum(jump)
    if hap == 1 and len(c.dels):
        lo, hi = np.searchsorted(c.dels, [refpos[0] + 1, refpos[-1]])
        for r, dl in zip(c.dels[lo:hi].tolist(), c.del_len[lo:hi].tolist()):
            refpos[refpos >= r] += dl
    refpos = np.minimum(refpos, c.length - 1)
    keep = np.ones(n_m, bool)
    keep[1:] = refpos[1:] > refpos[:-1]            # (a read clamped at the contig's end)
    if not keep.all():
        ins_idx = np.nonzero(~is_ins)[0][~keep]
        is_ins[ins_idx] = True                         # those query bases become inserted bases
        refpos = refpos[keep]
        n_m = len(refpos)
    # bases: the reference, haplotype 2's SNP alleles, the tumor's window variants, errors
    mb = c.ref[refpos].copy()
    if hap == 1:
        alt = c.alt[refpos]
        mb = np.where(alt != 255, alt, mb)
    if som:
        s = c.som[refpos]
        mb = np.where(s != 255, s, mb)
    e = rng.random(n_m) < err
    mb[e] = (mb[e] + rng.integers(1, 4, int(e.sum())).astype(np.uint8)) % 4
    aligned = rng.integers(0, 4, a, dtype=np.uint8)
    aligned[~is_ins] = mb
    bases = np.concatenate([rng.integers(0, 4, clip, dtype=np.uint8), aligned])
    # CIGAR: S, then runs of M / I with a D before an M base that follows a reference gap
    qm = np.nonzero(~is_ins)[0]
    gap = np.zeros(a, np.int64)
    gap[qm[1:]] = refpos[1:] - refpos[:-1] - 1
    t = is_ins.astype(np.int8)
    start = np.ones(a, bool)
    start[1:] = (t[1:] != t[:-1]) | (gap[1:] > 0)
    st = np.nonzero(start)[0]
    ln = np.diff(np.concatenate([st, [a]]))
    ops: List[int] = [(clip << 4) | 4] if clip else []
    for s0, l0 in zip(st.tolist(), ln.tolist()):
        if gap[s0] > 0:
            ops.append((int(gap[s0]) << 4) | 2)
        ops.append((l0 << 4) | (1 if t[s0] else 0))
    return int(refpos[0]), int(refpos[-1]) + 1, np.array(ops, np.uint32), bases


def _record(tid: int, pos: int, end: int, cig: np.ndarray, bases: np.ndarray, qual: np.ndarray, flag: int,
            mpos: int, tlen: int, name: bytes) -> bytes:
    n = len(bases)
    codes = _CODE[bases]
    if n & 1:
        codes = np.concatenate([codes, np.zeros(1, np.uint8)])
    packed = ((codes[0::2] << 4) | codes[1::2]).astype(np.uint8)
    nl = len(name) + 1
    h = np.zeros(1, _HDR)
    h["bs"] = 32 + nl + 4 * len(cig) + len(packed) + n
    h["ref"], h["pos"], h["lrn"], h["mapq"] = tid, pos, nl, 60
    h["bin"] = reg2bin(np.array([pos]), np.array([end]))[0]
    h["ncig"], h["flag"], h["lseq"] = len(cig), flag, n
    h["nref"], h["npos"], h["tlen"] = tid, mpos, tlen
    return b"".join([h.tobytes(), name, b"\0", cig.astype("<u4").tobytes(), packed.tobytes(), qual.tobytes()])


def make_long_pair(outdir: str, n_contigs: int = 2, contig_len: int = 10_000_000, pairs_per_contig: int = 1500,
                   mean_len: int = 25_000, min_len: int = 10_000, max_len: int = 100_000, seed: int = 11,
                   snp_per_kb: float = 1.0, del_per_kb: float = 0.1, window_every: int = 20_000,
                   err: float = 0.005, indel_rate: float = 5e-4, clip_frac: float = 0.3, level: int = 1,
                   threads: int = 16) -> Dict[str, str]:
    os.makedirs(outdir, exist_ok=True)
    rng = np.random.default_rng(seed)
    names = [f"chr{i + 1}" for i in range(n_contigs)]
    contigs = [_Contig(rng, contig_len, snp_per_kb, del_per_kb, window_every) for _ in names]
    paths = write_reference(outdir, names, contigs)
    mu = np.log(mean_len) - 0.125      # (sigma 0.5: the log-normal's mean is mean_len)
    with ThreadPoolExecutor(threads) as pool:
        for tag, tumor in (("T", True), ("N", False)):
            per = []
            for tid, c in enumerate(contigs):
                recs = []   # (pos, record bytes, end)
                for j in range(pairs_per_contig):
                    l1, l2 = np.clip(np.exp(rng.normal(mu, 0.5, 2)), min_len, max_len).astype(np.int64).tolist()
                    gap = max(0, int(rng.normal(1000, 300)))
                    span = l1 + l2 + gap + 2000
                    s = int(rng.integers(100, max(101, c.length - span - 1000)))
                    hap = int(rng.integers(0, 2))
                    som = tumor and rng.random() < 0.4
                    p1, e1, c1, b1 = _read(rng, c, s, l1, hap, som, err, indel_rate, clip_frac)
                    p2, e2, c2, b2 = _read(rng, c, min(e1 + gap, c.length - l2 - 1000), l2, hap, som, err, indel_rate,
                                           clip_frac)
                    left_first = rng.random() < 0.5
                    nm = f"{tag}L{tid:02d}:{j:07d}".encode()
                    for left, (p_, e_, c_, b_, mp, me) in ((True, (p1, e1, c1, b1, p2, e2)),
                                                           (False, (p2, e2, c2, b2, p1, e1))):
                        r1 = left == left_first
                        flag = 1 | 2 | (0x40 if r1 else 0x80) | (0x20 if left else 0x10)
                        tlen = (me - p_) if left else -(e_ - mp)
                        q = rng.integers(2, 41, len(b_), dtype=np.uint8)
                        recs.append((p_, _record(tid, p_, e_, c_, b_, q, flag, mp, tlen, nm), e_))
                recs.sort(key=lambda r: r[0])
                blob = b"".join(r[1] for r in recs)
                sz = np.array([len(r[1]) for r in recs], np.int64)
                per.append((blob, sz, np.array([r[0] for r in recs], np.int64), np.array([r[2] for r in recs], np.int64)))
            _write_bam(paths[tag], [(n, c.length) for n, c in zip(names, contigs)], per, level, pool)
    return paths
