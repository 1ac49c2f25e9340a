#!/usr/bin/env python3
"""Golden vectors for the reference-protocol adapter (genomeanonymizer_amd/reference_adapter.py):
run the UNMODIFIED reference ``CompleteGermlineAnonymizer.anonymize`` (anonymizer_methods.py:431-535)
on every scope of paired synthetic samples, fed by the reference's own ``pileup_io.iter_pileups``
(pileup_io.pyx:8-41), and store what it yields: per scope, the pairs in yield order as FASTQ
records (``get_anonymized_fastq_record``, AM:215-243) and the statistics counts by variant type.

TEST INFRASTRUCTURE ONLY (oracle/), build container only (imports /root/reference at run time
through the same stubs as run_reference.py). Output: tests/golden/adapter/<name>/ holding the
inputs (t.bam, n.bam, ref.fa(+.fai), scopes.json) and expected.json; nothing derived from the
reference's source is written.

usage: python oracle/make_adapter_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

NT16 = "=ACMGRSVTWYHKDBN"


def _nibbles(packed, off_nib, n):
    i = off_nib + np.arange(n, dtype=np.int64)
    b = packed[i >> 1]
    return np.where(i & 1, b & 0xF, b >> 4).astype(np.uint8)


def write_inputs(arr: dict, dest: str, seed: int) -> list:
    """One contig per scope; the scope's reads paired two by two within each dataset (FR flags),
    reverse strand only for reads whose bases are all ACGTN (others would hit the reference's
    KeyError). Returns the scopes as (contig, start, stop, keep)."""
    from genomeanonymizer_amd.synth.bamwriter import BamRecord, write_bam, write_fasta
    rng = np.random.default_rng(seed)
    n = len(arr["read_len"])
    ok = (arr["read_len"] > 0) & (arr["n_cig"] > 0)
    S = len(arr["scope_span_len"])
    contigs, seqs = [], []
    for s in range(S):
        a = int(arr["scope_span_start"][s])
        L = int(arr["scope_span_len"][s])
        codes = _nibbles(arr["ref_nt16"], int(arr["scope_ref_off"][s]) - a, a + L + 2)
        seqs.append("".join(NT16[c] for c in codes))
        contigs.append((f"s{s}", len(seqs[-1])))
    write_fasta(os.path.join(dest, "ref.fa"), [(c[0], q) for c, q in zip(contigs, seqs)])
    owner = np.full(n, -1, np.int64)
    offs = arr["scope_incid_off"]
    for s in range(S):
        for r in arr["incid_read"][offs[s]:offs[s + 1]].tolist():
            owner[r] = s
    recs = {0: [], 1: []}
    for s in range(S):
        for ds in (0, 1):
            rows = [r for r in range(n) if owner[r] == s and ok[r] and int(arr["dataset"][r]) == ds]
            rng.shuffle(rows)
            for k, r in enumerate(rows):
                mate = k % 2
                name = f"s{s}d{ds}p{k // 2}" if k // 2 < len(rows) // 2 else f"s{s}d{ds}u{k}"
                L = int(arr["read_len"][r])
                codes = _nibbles(arr["seq_nt16"], 2 * int(arr["seq_off"][r]), L)
                seq = "".join(NT16[c] for c in codes)
                rev = mate == 1 and set(seq) <= set("ACGTN")
                flag = 1 | (64 if mate == 0 else 128) | (16 if rev else 0)
                cig = arr["cigar"][arr["cig_off"][r]:arr["cig_off"][r] + arr["n_cig"][r]]
                ops = [("MIDNSHP=X"[int(w) & 0xF], int(w) >> 4) for w in cig]
                qual = rng.integers(2, 41, L).tolist()
                recs[ds].append(BamRecord(name, flag, s, int(arr["ref_start"][r]), 60, ops, s,
                                          int(arr["ref_start"][r]), 0, seq, qual))
    for ds, fn in ((0, "t.bam"), (1, "n.bam")):
        write_bam(os.path.join(dest, fn), contigs, sorted(recs[ds], key=lambda x: (x.tid, x.pos)))
    scopes = []
    for s in range(S):
        a = int(arr["scope_span_start"][s])
        b = max(a + int(arr["scope_span_len"][s]), a + 1)
        keep = None
        if arr["keep_pos"][s] >= 0:
            kp = int(arr["keep_pos"][s])
            keep = [kp, NT16[int(arr["keep_code"][s])], seqs[s][kp].upper()]
        scopes.append([f"s{s}", a, b, keep])
    return scopes


def run_reference(dest: str, scopes: list) -> list:
    from make_scope_golden import _setup_reference
    _setup_reference()
    import pysam
    import pileup_io
    from src.GenomeAnonymizer.anonymizer_methods import CompleteGermlineAnonymizer
    from src.GenomeAnonymizer.variants import CalledGenomicVariant
    from variant_extractor.variants import VariantType

    class Counter:
        def __init__(self):
            self.by_type = {}

        def count_variant(self, v):
            self.by_type[v.variant_type.name] = self.by_type.get(v.variant_type.name, 0) + 1

    T = pysam.AlignmentFile(os.path.join(dest, "t.bam"))
    N = pysam.AlignmentFile(os.path.join(dest, "n.bam"))
    fasta = pysam.FastaFile(os.path.join(dest, "ref.fa"))
    anon = CompleteGermlineAnonymizer()
    out = []
    for contig, a, b, keep in scopes:
        kv = None
        if keep is not None:
            kv = CalledGenomicVariant(contig, keep[0], keep[0], VariantType.SNV, 1, keep[1], keep[2])
        rec = Counter()
        pairs = []
        for pair in anon.anonymize(kv, pileup_io.iter_pileups(T, N, fasta, contig, a, b), fasta, stats_recorder=rec):
            pairs.append([None if x is None else x.get_anonymized_fastq_record() for x in pair])
        out.append({"pairs": pairs, "counts": rec.by_type})
    return out


def make(name: str, arr: dict, seed: int) -> dict:
    dest = os.path.join(REPO, "tests", "golden", "adapter", name)
    os.makedirs(dest, exist_ok=True)
    scopes = write_inputs(arr, dest, seed)
    expected = run_reference(dest, scopes)
    json.dump(scopes, open(os.path.join(dest, "scopes.json"), "w"))
    json.dump(expected, open(os.path.join(dest, "expected.json"), "w"))
    return {"scopes": len(scopes), "pairs": sum(len(e["pairs"]) for e in expected),
            "counts": {k: sum(e["counts"].get(k, 0) for e in expected) for k in ("SNV", "DEL", "INS")}}


def make_long(name: str, seed: int, n_reads: int = 8, genome: int = 36_000, len_range=(10_000, 16_000)) -> dict:
    """Long reads (SURVEY §8(d) C5 shape): a ``longread_batch`` of 10-30 kb reads with 1-3 bp indels
    every ~20 bases, soft clips up to 2 kb, substitutions and IUPAC reference codes, on ONE contig,
    paired two by two within each dataset (FR, mate fields set); every window scope (window
    +-1000; the pileup takes whole read extents, so the scopes span tens of kb and share reads) is
    run through the unmodified reference. Germline indels (the same indel in a tumor and a normal
    read) occur, so the yielded records carry the reference's indel edits too."""
    from genomeanonymizer_amd.synth.batch import longread_batch
    from genomeanonymizer_amd.synth.bamwriter import BamRecord, write_bam, write_fasta
    arr, info = longread_batch(seed, n_reads=n_reads, genome=genome, len_range=len_range)
    dest = os.path.join(REPO, "tests", "golden", "adapter", name)
    os.makedirs(dest, exist_ok=True)
    rng = np.random.default_rng(seed)
    ref_seq = "".join(NT16[c] for c in _nibbles(arr["ref_nt16"], 0, genome))
    write_fasta(os.path.join(dest, "ref.fa"), [("c0", ref_seq)])
    n = len(arr["read_len"])
    recs = {0: [], 1: []}
    for ds in (0, 1):
        rows = [r for r in range(n) if int(arr["dataset"][r]) == ds]
        rng.shuffle(rows)
        for k in range(0, len(rows), 2):
            grp = rows[k:k + 2]
            for m, r in enumerate(grp):
                mate = grp[1 - m] if len(grp) == 2 else r
                name_ = f"d{ds}p{k // 2}" if len(grp) == 2 else f"d{ds}u{k}"
                L = int(arr["read_len"][r])
                seq = "".join(NT16[c] for c in _nibbles(arr["seq_nt16"], 2 * int(arr["seq_off"][r]), L))
                rev = m == 1 and set(seq) <= set("ACGTN")
                flag = 1 | (64 if m == 0 else 128) | (16 if rev else 0) | (32 if (m == 0 and len(grp) == 2) else 0)
                cig = arr["cigar"][arr["cig_off"][r]:arr["cig_off"][r] + arr["n_cig"][r]]
                ops = [("MIDNSHP=X"[int(w) & 0xF], int(w) >> 4) for w in cig]
                qual = rng.integers(20, 24, L).tolist()
                recs[ds].append(BamRecord(name_, flag, 0, int(arr["ref_start"][r]), 60, ops, 0,
                                          int(arr["ref_start"][mate]), 0, seq, qual))
    for ds, fn in ((0, "t.bam"), (1, "n.bam")):
        write_bam(os.path.join(dest, fn), [("c0", genome)], sorted(recs[ds], key=lambda x: x.pos))
    scopes = []
    for s in range(len(arr["scope_span_len"])):
        kp = int(arr["keep_pos"][s])                  # the window's variant (0-based)
        scopes.append(["c0", kp - 1000, kp + 1001, [kp, NT16[int(arr["keep_code"][s])], ref_seq[kp].upper()]])
    expected = run_reference(dest, scopes)
    json.dump(scopes, open(os.path.join(dest, "scopes.json"), "w"))
    json.dump(expected, open(os.path.join(dest, "expected.json"), "w"))
    return {"reads": n, "scopes": len(scopes), "pairs": sum(len(e["pairs"]) for e in expected),
            "cigar_ops": int(len(arr["cigar"])), "max_span": info["max_span"],
            "counts": {k: sum(e["counts"].get(k, 0) for e in expected) for k in ("SNV", "DEL", "INS")}}


if __name__ == "__main__":
    from genomeanonymizer_amd.synth.batch import indel_batch, random_batch
    if "long" in sys.argv[1:]:
        print("long", make_long("long", 601))
    else:
        print("snv", make("snv", random_batch(404, n_scopes=24, rare_frac=0.1, wide_scopes=1), 404))
        print("indel", make("indel", indel_batch(505, n_scopes=16), 505))
