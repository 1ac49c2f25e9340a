"""Synthetic device batches (include/ganon.h layout) built directly in numpy, for kernel
parity tests and the benchmark — no BAM round trip.

* ``random_batch``: small batches full of edge cases (soft clips, I/D/N/H/=/X CIGAR ops,
  N / IUPAC / '=' read bases, kept variants on TN sites, empty scopes, zero-length reads,
  reads shared by several scopes, pass-through reads, scopes wider than the LDS cap).
* ``config2_batch``: BASELINE.json configs[1] — 10 M 150 bp reads (tumor + normal, FR
  pairs, insert N(300, 30)) on a 3.0 Gb 24-contig random genome with 1 M germline het SNPs,
  0.1 % errors, quals irrelevant to the kernel, and a window VCF of 1 M somatic SNVs spaced
  >= 2.5 kb (windows cover ~67 % of the genome). Scopes follow the
  planner's rules: one scope per window (reads overlapping [pos-1000, pos+1001)), and in
  the gaps one scope per chain of overlapping reads that holds both tumor and normal reads
  (iter_fetch_pair's union scopes, approximated by read chaining over both samples);
  reads in no scope are pass-through (write_scope -1); a read in two scopes is written
  from the first one (the first-writer rule).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

ACGT = np.array([1, 2, 4, 8], np.uint8)     # nt16 codes
IUPAC = np.array([3, 5, 6, 7, 9, 10, 11, 12, 13, 14], np.uint8)


def pack_nibbles(codes: np.ndarray) -> np.ndarray:
    c = codes.astype(np.uint8)
    if len(c) & 1:
        c = np.concatenate([c, np.zeros(1, np.uint8)])
    return ((c[0::2] << 4) | c[1::2]).astype(np.uint8)


def unpack_nibbles(packed: np.ndarray, n: int) -> np.ndarray:
    out = np.empty(2 * len(packed), np.uint8)
    out[0::2] = packed >> 4
    out[1::2] = packed & 0xF
    return out[:n]


def _cigar_word(op: str, n: int) -> int:
    return (n << 4) | "MIDNSHP=X".index(op)


def random_batch(seed: int, n_scopes: int = 64, max_reads: int = 40, read_len=(0, 220),
                 wide_scopes: int = 2, rare_frac: float = 0.02, wide_span=(20000, 40000)) -> Dict[str, np.ndarray]:
    """Edge-case batch. Every scope owns a private contig region so spans never collide. The
    first ``wide_scopes`` scopes span ``wide_span`` positions (over 2^20: the huge-scope tile path)."""
    rng = np.random.default_rng(seed)
    scopes = []
    region_len = []
    for s in range(n_scopes):
        wide = s < wide_scopes
        span = int(rng.integers(*wide_span)) if wide else int(rng.integers(50, 3000))
        region_len.append(span + 1200)
        scopes.append(wide)
    # reference: one contig per scope region, each starting on a byte boundary
    ref_codes, ref_nib_off = [], []
    nib = 0
    for L in region_len:
        r = ACGT[rng.integers(0, 4, L)]
        ns = rng.random(L) < 0.01
        r[ns] = 15                                   # N in the reference: never a call
        iu = rng.random(L) < 0.003
        r[iu] = IUPAC[rng.integers(0, len(IUPAC), int(iu.sum()))]
        ref_codes.append(r)
        ref_nib_off.append(nib)
        nib += L + (L & 1)
    ref_packed = np.concatenate([pack_nibbles(r) for r in ref_codes])
    reads: List[Tuple[int, int, list, np.ndarray, int]] = []   # (scope, pos, cigar, seq, dataset)
    scope_reads: List[List[int]] = []
    for s, wide in enumerate(scopes):
        ref = ref_codes[s]
        L = len(ref)
        # germline sites: alt alleles shared by tumor and normal reads
        n_sites = max(1, L // 60)
        sites = np.unique(rng.integers(300, L - 300, n_sites))
        alt = {int(p): int(ACGT[rng.integers(0, 4)]) for p in sites}
        rare_sites = {int(p): int(IUPAC[rng.integers(0, len(IUPAC))]) if rng.random() < 0.7 else 0
                      for p in sites[rng.random(len(sites)) < rare_frac * 10]}
        nr = int(rng.integers(0, max_reads + 1)) if not wide else int(rng.integers(150, 400))
        ids = []
        for _ in range(nr):
            ds = int(rng.integers(0, 2))
            rl = int(rng.integers(read_len[0], read_len[1] + 1))
            pos = int(rng.integers(250, max(251, L - 300 - min(rl, 200))))
            if wide and rng.random() < 0.3:
                rl = int(rng.integers(1000, 6000))       # long reads crossing tile borders
                pos = int(rng.integers(250, max(251, L - rl - 300)))
            cig, seq = _make_read(rng, ref, pos, rl, alt, rare_sites, ds)
            if cig is None:
                continue
            reads.append((s, pos, cig, seq, ds))
            ids.append(len(reads) - 1)
        scope_reads.append(ids)
    # a few reads also join the next scope's incidence list when regions allow it: skip,
    # spans are private; instead add cross-scope incidence by duplicating scope membership
    # for reads that lie in both (none here) — shared membership is covered in config2.
    n = len(reads)
    ref_start = np.array([r[1] for r in reads], np.int64)
    seq_parts, cig_parts = [], []
    seq_off = np.zeros(n, np.int64)
    cig_off = np.zeros(n, np.int64)
    so = co = 0
    for i, (_, _, cig, seq, _) in enumerate(reads):
        p = pack_nibbles(seq)
        seq_parts.append(p)
        seq_off[i] = so
        so += len(p)
        cig_parts.append(np.array(cig, np.uint32))
        cig_off[i] = co
        co += len(cig)
    arr = {
        "read_len": np.array([len(r[3]) for r in reads], np.int32),
        "seq_off": seq_off,
        "seq_nt16": np.concatenate(seq_parts) if seq_parts else np.zeros(0, np.uint8),
        "cig_off": cig_off,
        "n_cig": np.array([len(r[2]) for r in reads], np.int32),
        "cigar": np.concatenate(cig_parts) if cig_parts else np.zeros(0, np.uint32),
        "dataset": np.array([r[4] for r in reads], np.uint8),
        "ref_nt16": ref_packed,
    }
    # scope spans from their reads; the contig coordinate of scope s is the region offset
    ends = np.array([_ref_end(r[1], r[2]) for r in reads], np.int64)
    span_start, span_len, ref_off, incid, offs = [], [], [], [], [0]
    keep_pos, keep_code = [], []
    for s, ids in enumerate(scope_reads):
        if ids:
            a = int(ref_start[ids].min())
            b = int(ends[ids].max())
        else:
            a = b = 0
        span_start.append(a)
        span_len.append(b - a)
        ref_off.append(ref_nib_off[s] + a)
        order = rng.permutation(len(ids))
        incid.extend([ids[k] for k in order])
        offs.append(len(incid))
        # keep: half of the scopes keep one (alt) allele at a germline-ish site
        if ids and rng.random() < 0.5:
            r = reads[ids[0]]
            kp = r[1] + int(rng.integers(0, 30))
            keep_pos.append(kp)
            keep_code.append(int(ACGT[rng.integers(0, 4)]) if rng.random() < 0.8 else 5)
        else:
            keep_pos.append(-1)
            keep_code.append(0)
    arr["ref_start"] = ref_start.astype(np.int32)
    arr["scope_incid_off"] = np.array(offs, np.int64)
    arr["incid_read"] = np.array(incid, np.int32)
    arr["scope_span_start"] = np.array(span_start, np.int32)
    arr["scope_span_len"] = np.array(span_len, np.int32)
    arr["scope_ref_off"] = np.array(ref_off, np.int64)
    arr["keep_pos"] = np.array(keep_pos, np.int32)
    arr["keep_code"] = np.array(keep_code, np.uint8)
    ws = np.full(n, -1, np.int32)
    for s, ids in enumerate(scope_reads):
        for i in ids:
            if rng.random() < 0.85:
                ws[i] = s
    arr["write_scope"] = ws
    return arr


def indel_batch(seed: int, n_scopes: int = 40, reads_per_scope=(2, 40), read_len=(20, 200),
                indel_per_kb: float = 10.0, noise: float = 0.01) -> Dict[str, np.ndarray]:
    """Germline-indel batch for the indel tally: one contig, overlapping scope
    windows (a read may join the next scope's incidence list), germline INS/DEL alleles carried by
    tumor and normal reads, random indel noise, and the CIGAR corner cases of process_indels
    (variation_classifier.py:52-141): leading/trailing I and D, back-to-back I ops at one position,
    S/H clips (H counts toward in_read_pos), N skips. Incidences list tumor reads, then
    normal reads, in file order, as build_batch does."""
    rng = np.random.default_rng(seed)
    step, win = 1500, 2600
    Lc = n_scopes * step + win + 2000
    ref = ACGT[rng.integers(0, 4, Lc)]
    planted = {}
    for p in np.unique(rng.integers(50, Lc - 50, int(Lc * indel_per_kb / 1000))).tolist():
        if rng.random() < 0.5:
            k = int(rng.integers(1, 6))
            planted[p] = ("I", k, ACGT[rng.integers(0, 4, k)])
        else:
            planted[p] = ("D", int(rng.integers(1, 6)), None)
    reads = []        # (home scope, pos, cigar words, seq codes, dataset)

    def make(pos, rl):
        ops, seq = [], []

        def put(op, n, codes=None):
            if op == "M" and ops and ops[-1][0] == "M":
                ops[-1] = ("M", ops[-1][1] + n)
            else:
                ops.append((op, n))
            if codes is not None:
                seq.extend(int(c) for c in codes)

        if rng.random() < 0.15:
            put("H", int(rng.integers(1, 20)))
        if rng.random() < 0.2:
            k = int(rng.integers(1, 30))
            put("S", k, ACGT[rng.integers(0, 4, k)])
        if rng.random() < 0.05:
            k = int(rng.integers(1, 4))
            put("I", k, ACGT[rng.integers(0, 4, k)])
        p = pos
        left = rl - len(seq)
        while left > 0 and p < Lc - 10:
            pl = planted.get(p)
            if pl is not None and rng.random() < 0.8:
                if pl[0] == "I":
                    n = min(pl[1], left)
                    put("I", n, pl[2][:n])
                    left -= n
                    if left > 3 and rng.random() < 0.05:      # a second I op at the same position
                        put("I", 1, ACGT[rng.integers(0, 4, 1)])
                        left -= 1
                else:
                    put("D", pl[1])
                    p += pl[1]
                if left > 0:
                    put("M", 1, [ref[p]])
                    p += 1
                    left -= 1
                continue
            u = rng.random()
            if u < noise / 2:
                n = min(int(rng.integers(1, 4)), left)
                put("I", n, ACGT[rng.integers(0, 4, n)])
                left -= n
            elif u < noise:
                n = int(rng.integers(1, 4))
                put("D", n)
                p += n
            elif u < noise + 0.002:
                n = int(rng.integers(5, 30))
                put("N", n)
                p += n
            else:
                c = ref[p] if rng.random() > 0.01 else ACGT[rng.integers(0, 4)]
                put("M", 1, [c])
                p += 1
                left -= 1
        if left > 0:
            put("S", left, ACGT[rng.integers(0, 4, left)])
        u = rng.random()
        if u < 0.04:
            k = int(rng.integers(1, 4))
            put("I", k, ACGT[rng.integers(0, 4, k)])
        elif u < 0.08:
            put("D", int(rng.integers(1, 4)))
        if rng.random() < 0.1:
            put("H", int(rng.integers(1, 20)))
        if not any(o in ("M",) for o, _ in ops):
            return None, None
        return [_cigar_word(o, n) for o, n in ops], np.array(seq, np.uint8)

    for s in range(n_scopes):
        for _ in range(int(rng.integers(reads_per_scope[0], reads_per_scope[1] + 1))):
            rl = int(rng.integers(read_len[0], read_len[1] + 1))
            pos = int(rng.integers(s * step + 50, s * step + win - 400))
            cig, seq = make(pos, rl)
            if cig is not None:
                reads.append((s, pos, cig, seq, int(rng.integers(0, 2))))
    n = len(reads)
    ends = np.array([_ref_end(r[1], r[2]) for r in reads], np.int64)
    members = [[] for _ in range(n_scopes)]
    for i, (s, pos, _, _, _) in enumerate(reads):
        members[s].append(i)
        if s + 1 < n_scopes and ends[i] > (s + 1) * step and rng.random() < 0.5:
            members[s + 1].append(i)
    ws = np.full(n, -1, np.int32)
    for i, (s, _, _, _, _) in enumerate(reads):
        if rng.random() < 0.85:
            ws[i] = s
    seq_parts, cig_parts = [], []
    seq_off = np.zeros(n, np.int64)
    cig_off = np.zeros(n, np.int64)
    so = co = 0
    for i, (_, _, cig, seq, _) in enumerate(reads):
        pk = pack_nibbles(seq)
        seq_parts.append(pk)
        seq_off[i] = so
        so += len(pk)
        cig_parts.append(np.array(cig, np.uint32))
        cig_off[i] = co
        co += len(cig)
    ref_start = np.array([r[1] for r in reads], np.int64)
    dataset = np.array([r[4] for r in reads], np.uint8)
    span_start, span_len, incid, offs = [], [], [], [0]
    for s in range(n_scopes):
        ids = sorted(members[s], key=lambda i: (int(dataset[i]), i))
        a = int(ref_start[ids].min()) if ids else 0
        b = int(ends[ids].max()) if ids else 0
        span_start.append(a)
        span_len.append(b - a)
        incid.extend(ids)
        offs.append(len(incid))
    return {
        "ref_start": ref_start.astype(np.int32),
        "read_len": np.array([len(r[3]) for r in reads], np.int32),
        "seq_off": seq_off,
        "seq_nt16": np.concatenate(seq_parts) if seq_parts else np.zeros(0, np.uint8),
        "cig_off": cig_off,
        "n_cig": np.array([len(r[2]) for r in reads], np.int32),
        "cigar": np.concatenate(cig_parts) if cig_parts else np.zeros(0, np.uint32),
        "dataset": dataset,
        "write_scope": ws,
        "scope_incid_off": np.array(offs, np.int64),
        "incid_read": np.array(incid, np.int32),
        "scope_span_start": np.array(span_start, np.int32),
        "scope_span_len": np.array(span_len, np.int32),
        "scope_ref_off": np.array(span_start, np.int64),
        "ref_nt16": pack_nibbles(ref),
        "keep_pos": np.full(n_scopes, -1, np.int32),
        "keep_code": np.zeros(n_scopes, np.uint8),
    }


def dense_batch(seed: int, reads_per_scope=(8000, 400, 1200), span: int = 2200, read_len: int = 150,
                error_rate: float = 0.02, keep_hot_site: bool = False) -> Dict[str, np.ndarray]:
    """Very deep, error-rich scopes: thousands of observations per scope and one germline
    site carried by every read over it (one call seen thousands of times). Exercises the
    overflow handling of observation-list kernels; simple 150M reads only."""
    rng = np.random.default_rng(seed)
    n_s = len(reads_per_scope)
    region = span + 2 * read_len
    ref_codes = ACGT[rng.integers(0, 4, region * n_s)]
    reads, scope_reads = [], []
    keep_pos, keep_code = [], []
    for s, nr in enumerate(reads_per_scope):
        base = s * region
        hot = read_len + span // 2                   # every read over it carries hot_alt
        hot_alt = int(ACGT[(int(np.log2(ref_codes[base + hot])) + 1) % 4])
        het = read_len + span // 3
        het_alt = int(ACGT[(int(np.log2(ref_codes[base + het])) + 2) % 4])
        ids = []
        for _ in range(nr):
            pos = int(rng.integers(read_len // 2, read_len // 2 + span - read_len))
            seq = ref_codes[base + pos: base + pos + read_len].copy()
            err = rng.random(read_len) < error_rate
            seq[err] = ACGT[rng.integers(0, 4, int(err.sum()))]
            if pos <= hot < pos + read_len:
                seq[hot - pos] = hot_alt
            if pos <= het < pos + read_len and rng.random() < 0.5:
                seq[het - pos] = het_alt
            reads.append((base + pos, seq, int(rng.integers(0, 2))))
            ids.append(len(reads) - 1)
        scope_reads.append(ids)
        if keep_hot_site and s == 0:
            keep_pos.append(base + hot)
            keep_code.append(hot_alt)
        else:
            keep_pos.append(-1)
            keep_code.append(0)
    n = len(reads)
    L = np.full(n, read_len, np.int32)
    h = (read_len + 1) // 2
    arr = {
        "ref_start": np.array([r[0] for r in reads], np.int32),
        "read_len": L,
        "seq_off": np.arange(n, dtype=np.int64) * h,
        "seq_nt16": np.concatenate([pack_nibbles(r[1]) for r in reads]),
        "cig_off": np.arange(n, dtype=np.int64),
        "n_cig": np.ones(n, np.int32),
        "cigar": np.full(n, _cigar_word("M", read_len), np.uint32),
        "dataset": np.array([r[2] for r in reads], np.uint8),
        "ref_nt16": pack_nibbles(ref_codes),
    }
    starts = arr["ref_start"].astype(np.int64)
    span_start, span_len, incid, offs = [], [], [], [0]
    for s, ids in enumerate(scope_reads):
        a = int(starts[ids].min())
        b = int(starts[ids].max()) + read_len
        span_start.append(a)
        span_len.append(b - a)
        incid.extend(rng.permutation(ids).tolist())
        offs.append(len(incid))
    arr["scope_incid_off"] = np.array(offs, np.int64)
    arr["incid_read"] = np.array(incid, np.int32)
    arr["scope_span_start"] = np.array(span_start, np.int32)
    arr["scope_span_len"] = np.array(span_len, np.int32)
    arr["scope_ref_off"] = np.array(span_start, np.int64)      # one contig: nibble = position
    arr["keep_pos"] = np.array(keep_pos, np.int32)
    arr["keep_code"] = np.array(keep_code, np.uint8)
    ws = np.full(n, -1, np.int32)
    for s, ids in enumerate(scope_reads):
        for i in ids:
            if rng.random() < 0.9:
                ws[i] = s
    arr["write_scope"] = ws
    return arr


def _ref_end(pos: int, cig: list) -> int:
    rl = sum(w >> 4 for w in cig if (w & 0xF) in (0, 2, 3, 7, 8))
    return pos + (rl if rl > 0 else 1)


def _make_read(rng, ref, pos, rl, alt, rare_sites, ds):
    """Build (cigar words, nt16 codes) for a read of rl query bases starting at ref pos."""
    if rl == 0:
        return [_cigar_word("M", 0)] if rng.random() < 0.5 else [], np.zeros(0, np.uint8)
    ops = []
    left = rl
    if rng.random() < 0.1:
        k = int(rng.integers(1, min(20, left) + 1))
        ops.append(("S", k)); left -= k
    if rng.random() < 0.05:
        ops.insert(0, ("H", int(rng.integers(1, 10))))
    while left > 0:
        k = int(rng.integers(1, left + 1)) if rng.random() < 0.3 else left
        op = "M"
        u = rng.random()
        if u < 0.05:
            op = "="
        elif u < 0.1:
            op = "X"
        ops.append((op, k)); left -= k
        if left > 0:
            v = rng.random()
            if v < 0.3:
                n = int(rng.integers(1, min(8, left) + 1))
                ops.append(("I", n)); left -= n
            elif v < 0.6:
                ops.append(("D", int(rng.integers(1, 6))))
            elif v < 0.7:
                ops.append(("N", int(rng.integers(5, 60))))
    if rng.random() < 0.05:
        ops.append(("H", int(rng.integers(1, 10))))
    seq = []
    rp = pos
    for op, n in ops:
        if op in "M=X":
            for i in range(n):
                p = rp + i
                if p >= len(ref):
                    return None, None
                b = int(ref[p])
                if p in alt and rng.random() < 0.6:
                    b = alt[p]
                if p in rare_sites and rng.random() < 0.5:
                    b = rare_sites[p]
                u = rng.random()
                if u < 0.002:
                    b = int(ACGT[rng.integers(0, 4)])
                elif u < 0.004:
                    b = 15
                seq.append(b)
            rp += n
        elif op in "IS":
            seq.extend(int(x) for x in ACGT[rng.integers(0, 4, n)])
        elif op in "DN":
            rp += n
    if rp >= len(ref) - 1:
        return None, None
    return [_cigar_word(o, n) for o, n in ops], np.array(seq, np.uint8)


# ---------------------------------------------------------------------------------------
# long reads
# ---------------------------------------------------------------------------------------

def longread_batch(seed: int = 5, n_reads: int = 200, genome: int = 2_000_000, len_range=(10_000, 100_000),
                   indel_rate: float = 0.05, sub_rate: float = 0.01, clip_max: int = 2000,
                   window_spacing: int = 10_000, germline_every: int = 1000) -> Tuple[Dict[str, np.ndarray], dict]:
    """C5-like batch: ONT-style reads (log-uniform lengths, ~indel_rate 1-3 bp I/D ops, soft clips
    at both ends, substitutions), tumor and normal halves, het germline SNPs every
    ~germline_every bp, reference N runs and IUPAC codes, and a window scope every
    window_spacing bp (reads overlapping [pos - 1000, pos + 1001); scope spans reach ~200 kb).
    A read is written by the first window it overlaps; reads in no window pass through."""
    rng = np.random.default_rng(seed)
    ref = ACGT[rng.integers(0, 4, genome)]
    for a in range(250_000, genome - 1000, 700_000):          # N runs
        ref[a:a + 500] = 15
    iu = rng.random(genome) < 2e-5
    ref[iu] = IUPAC[rng.integers(0, len(IUPAC), int(iu.sum()))]
    gsnp = np.arange(500, genome - 500, germline_every) + rng.integers(-200, 200, (genome - 1000) // germline_every)
    gsnp = np.unique(gsnp[(gsnp > 0) & (gsnp < genome)])
    galt = ACGT[rng.integers(0, 4, len(gsnp))]
    lo, hi = np.log(len_range[0]), np.log(len_range[1])
    starts, cigars, seqs, dss = [], [], [], []
    for r in range(n_reads):
        span = int(np.exp(rng.uniform(lo, hi)))
        pos = int(rng.integers(0, max(1, genome - span - 10)))
        hap = rng.random() < 0.5
        # M runs (geometric) separated by 1-3 bp insertions/deletions, built vectorised
        runs = rng.geometric(indel_rate, size=int(span * indel_rate * 2) + 8).astype(np.int64)
        runs = runs[np.cumsum(runs) <= span]
        if not len(runs):
            continue
        nr = len(runs)
        ins = rng.random(nr) < 0.5                                # indel after run k: insertion?
        ilen = rng.integers(1, 4, nr).astype(np.int64)
        ins[-1] = False
        ilen[-1] = 0                                              # nothing after the last run
        c0 = int(rng.integers(0, clip_max + 1)) if rng.random() < 0.7 else 0
        c1 = int(rng.integers(0, clip_max + 1)) if rng.random() < 0.7 else 0
        radv = runs + np.where(ins, 0, ilen)
        qadv = runs + np.where(ins, ilen, 0)
        rstart = pos + np.concatenate([[0], np.cumsum(radv)[:-1]])
        qstart = c0 + np.concatenate([[0], np.cumsum(qadv)[:-1]])
        keep = rstart + runs < genome - 1
        if not keep.all():
            k = int(np.argmin(keep))
            if k == 0:
                continue
            runs, ins, ilen, rstart, qstart = runs[:k], ins[:k], ilen[:k], rstart[:k], qstart[:k]
            ins[-1] = False
            ilen[-1] = 0
        lq = int(c0 + runs.sum() + ilen[ins].sum() + c1)
        seq = ACGT[rng.integers(0, 4, lq)]                         # clips and insertions random
        tot = int(runs.sum())
        off = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(runs) - runs, runs)
        ridx = np.repeat(rstart, runs) + off
        b = ref[ridx].copy()
        if hap:
            gi = np.minimum(np.searchsorted(gsnp, ridx), len(gsnp) - 1)
            hit = gsnp[gi] == ridx
            b[hit] = galt[gi[hit]]
        err = rng.random(tot) < sub_rate
        b[err] = ACGT[rng.integers(0, 4, int(err.sum()))]
        seq[np.repeat(qstart, runs) + off] = b
        words = [np.full(1, (c0 << 4) | 4, np.int64)] if c0 else []
        mid = np.empty(2 * len(runs), np.int64)
        mid[0::2] = runs << 4                                    # M
        mid[1::2] = (ilen << 4) | np.where(ins, 1, 2)            # I / D
        mid = mid[:-1]                                           # no indel after the last run
        words.append(mid)
        if c1:
            words.append(np.full(1, (c1 << 4) | 4, np.int64))
        starts.append(pos)
        cigars.append(np.concatenate(words).astype(np.uint32))
        seqs.append(seq.astype(np.uint8))
        dss.append(r % 2)
    order = np.argsort(np.array(starts), kind="stable")     # coordinate-sorted, like a BAM
    starts = [starts[i] for i in order]
    cigars = [cigars[i] for i in order]
    seqs = [seqs[i] for i in order]
    dss = [dss[i] for i in order]
    n = len(starts)
    packed = [pack_nibbles(x) for x in seqs]
    seq_off = np.zeros(n, np.int64)
    seq_off[1:] = np.cumsum([len(x) for x in packed])[:-1]
    cig_off = np.zeros(n, np.int64)
    cig_off[1:] = np.cumsum([len(c) for c in cigars])[:-1]
    ends = np.array([_ref_end(starts[i], cigars[i].tolist()) for i in range(n)], np.int64)
    st = np.array(starts, np.int64)
    # window scopes
    wpos = np.arange(1002, genome - 1002, window_spacing, dtype=np.int64)
    max_span = int((ends - st).max()) if n else 0
    incid, offs, span_start, span_len, keep_pos, keep_code = [], [0], [], [], [], []
    ws = np.full(n, -1, np.int32)
    for w, wp in enumerate(wpos):
        a, b = wp - 1000, wp + 1001
        cand = np.arange(np.searchsorted(st, a - max_span), np.searchsorted(st, b))
        ids = cand[(st[cand] < b) & (ends[cand] > a)]
        incid.extend(ids.tolist())
        offs.append(len(incid))
        if len(ids):
            s0, s1 = int(st[ids].min()), int(ends[ids].max())
        else:
            s0 = s1 = 0
        span_start.append(s0)
        span_len.append(s1 - s0)
        keep_pos.append(int(wp - 1))
        keep_code.append(int(ACGT[rng.integers(0, 4)]))
        new = ids[ws[ids] < 0]
        ws[new] = w
    arr = {
        "ref_start": st.astype(np.int32),
        "read_len": np.array([len(x) for x in seqs], np.int32),
        "seq_off": seq_off,
        "seq_nt16": np.concatenate(packed) if packed else np.zeros(0, np.uint8),
        "cig_off": cig_off,
        "n_cig": np.array([len(c) for c in cigars], np.int32),
        "cigar": np.concatenate(cigars) if cigars else np.zeros(0, np.uint32),
        "dataset": np.array(dss, np.uint8),
        "write_scope": ws,
        "scope_incid_off": np.array(offs, np.int64),
        "incid_read": np.array(incid, np.int32),
        "scope_span_start": np.array(span_start, np.int32),
        "scope_span_len": np.array(span_len, np.int32),
        "scope_ref_off": np.array(span_start, np.int64),      # one contig: nibble = position
        "ref_nt16": pack_nibbles(ref),
        "keep_pos": np.array(keep_pos, np.int32),
        "keep_code": np.array(keep_code, np.uint8),
    }
    info = {"reads": n, "bases": int(arr["read_len"].astype(np.int64).sum()), "scopes": len(wpos),
            "incidences": len(incid), "max_span": int(max(span_len) if span_len else 0),
            "cigar_ops": int(len(arr["cigar"]))}
    return arr, info


# ---------------------------------------------------------------------------------------
# BASELINE.json configs[1]
# ---------------------------------------------------------------------------------------

def _random_genome(rng, total: int) -> np.ndarray:
    """Packed nt16 genome of random ACGT (2 bases per byte)."""
    nbytes = (total + 1) // 2
    raw = np.frombuffer(rng.bytes(nbytes), np.uint8)
    lut = np.zeros(256, np.uint8)
    for v in range(256):
        lut[v] = (ACGT[v & 3] << 4) | ACGT[(v >> 2) & 3]
    return lut[raw]


_SITES_CACHE: Dict[tuple, tuple] = {}


def config2_batch(n_reads: int = 10_000_000, genome: int = 3_000_000_000, n_contigs: int = 24,
                  n_windows: int = 1_000_000, n_germline: int = 1_000_000, read_len: int = 150,
                  seed: int = 2, window_spacing: int = 2500, read_seed: int = None,
                  germline_del_per_kb: float = 0.0, seq_indel_per_base: float = 0.0) -> Tuple[Dict[str, np.ndarray], dict]:
    """Vectorised BASELINE configs[1] batch. Returns (arrays, info). ``read_seed``: the reads come
    from their own generator (the genome, germline sites and windows from ``seed``, generated once
    per process and shared): batches of other reads on the same sample.

    Realistic CIGARs (the ``c2id`` shape): ``germline_del_per_kb`` het deletions of 1-3 bp per kb of
    genome (on haplotype 1 of tumor and normal alike, as synth/fastpair.py plants them: a read of
    haplotype 1 over one is ``aM dD bM``), and ``seq_indel_per_base`` sequencing indels of 1-3 bp
    (a read with one is ``aM dI/D bM``). Zero (the default) keeps every read ``150M``."""
    L = read_len
    key = (seed, genome, n_contigs, n_windows, n_germline, window_spacing)
    idp = (germline_del_per_kb, seq_indel_per_base)
    if read_seed is not None and key in _SITES_CACHE:
        clen, cstart, ref, gsnp, galt, win_contig, win_pos = _SITES_CACHE[key]
        return _config2_reads(np.random.default_rng(read_seed), n_reads, L, n_contigs, clen, cstart, ref, gsnp, galt,
                              win_contig, win_pos, idp)
    rng = np.random.default_rng(seed)
    # contigs: 24 of decreasing length summing to `genome`, each starting on a byte boundary
    w = np.linspace(2.0, 1.0, n_contigs)
    clen = np.floor(w / w.sum() * genome).astype(np.int64)
    clen -= clen % 2
    cstart = np.concatenate([[0], np.cumsum(clen)[:-1]])      # nibble offsets (even)
    ref = _random_genome(rng, int(clen.sum()))

    def ref_codes(gpos: np.ndarray) -> np.ndarray:
        b = ref[gpos >> 1]
        return np.where(gpos & 1, b & 0xF, b >> 4).astype(np.uint8)

    # germline het SNPs (global positions) and their alt codes
    gsnp = np.unique(rng.integers(0, int(clen.sum()), n_germline))
    galt = ACGT[(np.searchsorted(ACGT, ref_codes(gsnp)) + rng.integers(1, 4, len(gsnp))) % 4]
    # windows: evenly spaced per contig (>= window_spacing apart), 1-based pos >= 1002
    per = np.maximum(1, (clen / clen.sum() * n_windows).astype(np.int64))
    win_contig, win_pos = [], []
    for c in range(n_contigs):
        k = min(int(per[c]), max(0, (int(clen[c]) - 4000) // window_spacing))
        pos = 1002 + np.arange(k, dtype=np.int64) * window_spacing + rng.integers(0, window_spacing - 2003 + 1, k)
        pos = pos[pos <= clen[c] - 1003]
        win_contig.append(np.full(len(pos), c, np.int64))
        win_pos.append(pos)
    win_contig = np.concatenate(win_contig)
    win_pos = np.concatenate(win_pos)
    if read_seed is not None:
        _SITES_CACHE[key] = (clen, cstart, ref, gsnp, galt, win_contig, win_pos)
        rng = np.random.default_rng(read_seed)
    return _config2_reads(rng, n_reads, L, n_contigs, clen, cstart, ref, gsnp, galt, win_contig, win_pos, idp)


def _read_indels(rng, n, L, gstart, hap, del_per_kb, seq_per_base, genome_seed):
    """Per read (offset a, length d, kind: 0 none, 1 deletion, 2 insertion) for the c2id shape:
    germline het deletions (a deterministic site set of the genome: hash of the 1-kb bin, so every
    batch of the sample sees the same sites) on haplotype-1 reads, then sequencing indels on reads
    without one."""
    a = np.zeros(n, np.int64)
    d = np.zeros(n, np.int64)
    kind = np.zeros(n, np.int8)
    if del_per_kb > 0:
        # sites: bin b of 1 kb holds a deletion iff hash(b) < del_per_kb; position and length from the hash
        def h(x):
            x = (x.astype(np.uint64) + np.uint64(genome_seed) * np.uint64(0x9E3779B97F4A7C15)) & np.uint64(2**64 - 1)
            x ^= x >> np.uint64(31)
            x *= np.uint64(0xBF58476D1CE4E5B9)
            x ^= x >> np.uint64(29)
            return x
        with np.errstate(over="ignore"):
            for b in (gstart // 1000, gstart // 1000 + 1):   # a 150 bp read touches at most two bins
                hv = h(b)
                has = (hv >> np.uint64(40)).astype(np.float64) / float(1 << 24) < del_per_kb
                site = b * 1000 + ((hv & np.uint64(0xFFFF)).astype(np.int64) % 1000)
                ln = 1 + ((hv >> np.uint64(16)) & np.uint64(3)).astype(np.int64) % 3
                off = site - gstart
                ok = has & hap & (kind == 0) & (off >= 10) & (off <= L - 10)
                a[ok], d[ok], kind[ok] = off[ok], ln[ok], 1
    if seq_per_base > 0:
        hit = (rng.random(n) < seq_per_base * L) & (kind == 0)
        k = int(hit.sum())
        a[hit] = rng.integers(10, L - 10, k)
        d[hit] = rng.integers(1, 4, k)
        kind[hit] = np.where(rng.random(k) < 0.5, 1, 2)
    return a, d, kind


def _config2_reads(rng, n_reads, L, n_contigs, clen, cstart, ref, gsnp, galt, win_contig, win_pos, idp=(0.0, 0.0)):
    def ref_codes(gpos: np.ndarray) -> np.ndarray:
        b = ref[gpos >> 1]
        return np.where(gpos & 1, b & 0xF, b >> 4).astype(np.uint8)

    # reads: FR pairs, half tumor half normal
    n_pairs = n_reads // 2
    pc = rng.choice(n_contigs, size=n_pairs, p=clen / clen.sum())
    flen = np.clip(np.round(rng.normal(300, 30, n_pairs)).astype(np.int64), L + 10, None)
    fstart = (rng.random(n_pairs) * (clen[pc] - flen - 2)).astype(np.int64)
    ds_pair = (np.arange(n_pairs) >= n_pairs // 2).astype(np.uint8)      # 0 tumor, 1 normal
    rc = np.concatenate([pc, pc])
    rpos = np.concatenate([fstart, fstart + flen - L]).astype(np.int64)
    rds = np.concatenate([ds_pair, ds_pair])
    hap = np.concatenate([rng.integers(0, 2, n_pairs)] * 2).astype(bool)
    # order reads like a coordinate-sorted pair of BAMs: by (contig, pos)
    order = np.lexsort((rpos, rc))
    rc, rpos, rds, hap = rc[order], rpos[order], rds[order], hap[order]
    gstart = cstart[rc] + rpos
    n = len(rpos)
    del_kb, seq_pb = idp
    with_id = del_kb > 0 or seq_pb > 0
    ia, idd, ikind = _read_indels(rng, n, L, gstart, hap, del_kb, seq_pb, int(cstart[-1]) + len(ref)) if with_id \
        else (None, None, None)
    W = L + 3 if with_id else L    # (a deletion's read takes up to 3 reference bases past L)
    # bases: reference + germline het alts on haplotype 1 + 0.1 % errors
    # (the genome one code per byte, each read's codes one row of a sliding-window view: a row copy
    # per read instead of a per-base gather)
    nib = np.zeros(2 * len(ref) + 4, np.uint8)
    nib[0:2 * len(ref):2] = ref >> 4
    nib[1:2 * len(ref):2] = ref & 0xF
    codes = np.lib.stride_tricks.sliding_window_view(nib, W)[gstart]
    del nib
    lo = np.searchsorted(gsnp, gstart)
    hi = np.searchsorted(gsnp, gstart + W)
    cnt = hi - lo
    rid = np.repeat(np.arange(n), cnt)
    k = np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    sidx = lo[rid] + k
    carry = hap[rid]
    codes[rid[carry], (gsnp[sidx] - gstart[rid])[carry]] = galt[sidx][carry]
    span = np.full(n, L, np.int64)
    if with_id:
        # the indel reads' rows: a deletion skips d reference columns at a, an insertion puts d
        # random bases there (column index -1) and shifts the rest
        sel = np.nonzero(ikind > 0)[0]
        j = np.arange(L)[None, :]
        aa, dd, kk = ia[sel][:, None], idd[sel][:, None], ikind[sel][:, None]
        col = np.where(kk == 1, j + dd * (j >= aa), np.where(j < aa, j, np.where(j < aa + dd, -1, j - dd)))
        rows = np.take_along_axis(codes[sel], np.maximum(col, 0), axis=1)
        rows = np.where(col < 0, ACGT[rng.integers(0, 4, rows.shape)], rows).astype(np.uint8)
        codes = codes[:, :L].copy()
        codes[sel] = rows
        span[sel] = np.where(ikind[sel] == 1, L + idd[sel], L - idd[sel])
    n_err = int(n * L * 0.001)
    er = rng.integers(0, n, n_err)
    eo = rng.integers(0, L, n_err)
    codes[er, eo] = ACGT[rng.integers(0, 4, n_err)]
    seq = ((codes[:, 0::2] << 4) | codes[:, 1::2]).reshape(-1)
    del codes
    # scopes: windows first (in contig/position order), then gap union scopes
    rend = rpos + span
    key = rc * (1 << 40) + rpos
    span = L
    wkey_lo = win_contig * (1 << 40) + (win_pos - 1000 - span)
    wkey_hi = win_contig * (1 << 40) + (win_pos + 1001)
    wlo = np.searchsorted(key, wkey_lo, side="left")
    whi = np.searchsorted(key, wkey_hi, side="left")
    wcnt = whi - wlo
    w_rid = np.repeat(np.arange(len(win_pos)), wcnt)
    w_k = np.arange(int(wcnt.sum())) - np.repeat(np.cumsum(wcnt) - wcnt, wcnt)
    w_read = wlo[w_rid] + w_k
    keep_hit = rend[w_read] > (win_pos[w_rid] - 1000)
    w_rid, w_read = w_rid[keep_hit], w_read[keep_hit]
    in_window = np.zeros(n, bool)
    in_window[w_read] = True
    # gap chains over reads that are in no window: consecutive overlapping reads (same contig)
    g = np.nonzero(~in_window)[0]
    gc, gp, ge = rc[g], rpos[g], rend[g]
    run_end = np.maximum.accumulate(gc * (1 << 40) + ge)
    new_chain = np.ones(len(g), bool)
    new_chain[1:] = (gc[1:] != gc[:-1]) | (gc[1:] * (1 << 40) + gp[1:] > run_end[:-1])
    chain = np.cumsum(new_chain) - 1
    n_chain = int(chain[-1]) + 1 if len(g) else 0
    has_t = np.zeros(n_chain, bool)
    has_n = np.zeros(n_chain, bool)
    has_t[chain[rds[g] == 0]] = True
    has_n[chain[rds[g] == 1]] = True
    union = has_t & has_n
    u_ids = np.nonzero(union)[0]
    u_map = np.full(n_chain, -1, np.int64)
    u_map[u_ids] = np.arange(len(u_ids))
    g_scope = u_map[chain]
    g_sel = g_scope >= 0
    n_win = len(win_pos)
    n_scopes = n_win + len(u_ids)
    inc_scope = np.concatenate([w_rid, n_win + g_scope[g_sel]])
    inc_read = np.concatenate([w_read, g[g_sel]])
    o = np.argsort(inc_scope, kind="stable")
    inc_scope, inc_read = inc_scope[o], inc_read[o]
    counts = np.bincount(inc_scope, minlength=n_scopes)
    incid_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    # spans and reference offsets
    s_start = np.full(n_scopes, np.iinfo(np.int64).max, np.int64)
    s_end = np.zeros(n_scopes, np.int64)
    np.minimum.at(s_start, inc_scope, rpos[inc_read])
    np.maximum.at(s_end, inc_scope, rend[inc_read])
    empty = counts == 0
    s_start[empty] = 0
    s_end[empty] = 0
    s_contig = np.concatenate([win_contig, np.zeros(len(u_ids), np.int64)])
    first_read = np.full(n_scopes, -1, np.int64)
    first_read[inc_scope[::-1]] = inc_read[::-1]
    has_read = first_read >= 0
    s_contig[has_read] = rc[first_read[has_read]]
    # first-writer rule: the earliest scope (lowest id) a read belongs to writes it
    first_scope = np.full(n, n_scopes, np.int64)
    np.minimum.at(first_scope, inc_read, inc_scope)
    ws = np.where(first_scope < n_scopes, first_scope, -1).astype(np.int32)
    keep_pos = np.concatenate([win_pos - 1, np.full(len(u_ids), -1, np.int64)])
    keep_code = np.concatenate([ACGT[rng.integers(0, 4, n_win)], np.zeros(len(u_ids), np.uint8)])
    # scope ids in genome order, windows and gap union scopes interleaved, as the product planner
    # lays a sample's scopes out (a read is in one scope here, so the writer is unchanged)
    order = np.lexsort((s_start, s_contig))
    new_id = np.empty(n_scopes, np.int64)
    new_id[order] = np.arange(n_scopes)
    o = np.argsort(new_id[inc_scope], kind="stable")
    inc_scope, inc_read = new_id[inc_scope][o], inc_read[o]
    counts = counts[order]
    incid_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    s_start, s_end, s_contig = s_start[order], s_end[order], s_contig[order]
    keep_pos, keep_code = keep_pos[order], keep_code[order]
    ws = np.where(ws >= 0, new_id[np.maximum(ws, 0)], -1).astype(np.int32)
    if with_id:
        # aM dD (L-a)M or aM dI (L-a-d)M; every other read L M
        n_cig = np.where(ikind > 0, 3, 1).astype(np.int32)
        cig_off = np.concatenate([[0], np.cumsum(n_cig)[:-1]]).astype(np.int64)
        cigar = np.empty(int(n_cig.sum()), np.uint32)
        plain = ikind == 0
        cigar[cig_off[plain]] = (L << 4) | 0
        s = np.nonzero(~plain)[0]
        o = cig_off[s]
        dl = ikind[s] == 1
        cigar[o] = (ia[s] << 4).astype(np.uint32)
        cigar[o + 1] = ((idd[s] << 4) | np.where(dl, 2, 1)).astype(np.uint32)
        cigar[o + 2] = (np.where(dl, L - ia[s], L - ia[s] - idd[s]) << 4).astype(np.uint32)
    else:
        n_cig = np.ones(n, np.int32)
        cig_off = np.arange(n, dtype=np.int64)
        cigar = np.full(n, (L << 4) | 0, np.uint32)
    arr = {
        "ref_start": rpos.astype(np.int32),
        "read_len": np.full(n, L, np.int32),
        "seq_off": (np.arange(n, dtype=np.int64) * (L // 2)),
        "seq_nt16": seq,
        "cig_off": cig_off,
        "n_cig": n_cig,
        "cigar": cigar,
        "dataset": rds.astype(np.uint8),
        "write_scope": ws,
        "scope_incid_off": incid_off,
        "incid_read": inc_read.astype(np.int32),
        "scope_span_start": s_start.astype(np.int32),
        "scope_span_len": (s_end - s_start).astype(np.int32),
        "scope_ref_off": (cstart[s_contig] + s_start).astype(np.int64),
        "ref_nt16": ref,
        "keep_pos": keep_pos.astype(np.int32),
        "keep_code": keep_code.astype(np.uint8),
    }
    info = {"reads": n, "read_len": L, "scopes": n_scopes, "window_scopes": n_win,
            "union_scopes": int(len(u_ids)), "incidences": int(len(inc_read)),
            "passthrough_reads": int((ws < 0).sum()), "genome": int(clen.sum()), "contigs": n_contigs,
            "germline_snps": int(len(gsnp))}
    if with_id:
        info["indel_reads"] = int((ikind > 0).sum())
    return arr, info


def algorithmic_bytes(arr: Dict[str, np.ndarray]) -> int:
    """SURVEY §8(d) bytes of one launch over the batch: per read ceil(L/2) in + ceil(L/2)
    out + 4*n_cigar + 16; per extra scope incidence ceil(L/2) + 4*n_cigar + 8; per scope
    ceil(span/2) reference bytes."""
    L = arr["read_len"].astype(np.int64)
    half = (L + 1) // 2
    nc = arr["n_cig"].astype(np.int64)
    per_read = 2 * half + 4 * nc + 16
    inc = np.bincount(arr["incid_read"], minlength=len(L)).astype(np.int64)
    extra = np.maximum(inc - 1, 0) * (half + 4 * nc + 8)
    ref = (arr["scope_span_len"].astype(np.int64) + 1) // 2
    return int(per_read.sum() + extra.sum() + ref.sum())


def dataset_major(arr: Dict[str, np.ndarray], chunk: int = 1 << 20) -> Dict[str, np.ndarray]:
    """The same batch with its sequence buffer laid out as the product path builds it
    (anonymizer_methods.build_batch): every dataset-0 read's packed bases, then every dataset-1
    read's, each dataset in its original buffer order. Only seq_nt16 and seq_off change, so
    results are comparable read by read with the interleaved original."""
    order = np.lexsort((arr["seq_off"].astype(np.int64), arr["dataset"].astype(np.int64)))
    return relayout(arr, order, chunk)


def relayout(arr: Dict[str, np.ndarray], order: np.ndarray, chunk: int = 1 << 20) -> Dict[str, np.ndarray]:
    """The same batch with the reads' packed bases stored in the buffer in ``order`` (read
    indices), back to back; only seq_nt16 and seq_off change."""
    so = arr["seq_off"].astype(np.int64)
    nb = (arr["read_len"].astype(np.int64) + 1) // 2
    order = np.asarray(order, np.int64)
    new_off = np.empty_like(so)
    new_off[order] = np.concatenate([[0], np.cumsum(nb[order])[:-1]])
    seq = arr["seq_nt16"]
    out = np.zeros(len(seq), np.uint8)
    for k in range(0, len(order), chunk):
        o = order[k:k + chunk]
        n = nb[o]
        if n.sum() == 0:
            continue
        first = np.concatenate([[0], np.cumsum(n)[:-1]])
        rel = np.arange(int(n.sum()), dtype=np.int64) - np.repeat(first, n)
        out[np.repeat(new_off[o], n) + rel] = seq[np.repeat(so[o], n) + rel]
    res = dict(arr)
    res["seq_off"] = new_off
    res["seq_nt16"] = out
    return res
