"""Synthetic FASTQ record sets over a masking batch (formatter tests and bench).

A record set is the dict ``native.fastq_records`` layout — the arguments of the host
formatter ``ganon_fastq_format`` (include/ganon_host.h) and of ``ganon_fastq_format_hip``
(include/ganon.h): sequence buffers + per-record (buffer, nibble offset, length, reverse),
quality buffers + (buffer, offset, length, reversed), a name blob + (offset, length), mate.

Reads come from the batch's nt16 sequence buffer; qualities are uniform phred [2, 40]
(SURVEY §8(d)); names are random ``[A-Za-z0-9:_]`` strings. Reverse reads carrying a base
outside ACGTN would make the reference raise (reverse_complement, anonymizer_methods.py
:205-213), so they are kept forward unless ``allow_bad``.
"""
from __future__ import annotations

import numpy as np

NAME_ALPHABET = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789:_", np.uint8)
ACGTN = np.zeros(16, bool)
ACGTN[[1, 2, 4, 8, 15]] = True


def bad_for_reverse(seq_nt16: np.ndarray, nib_off: np.ndarray, length: np.ndarray, chunk: int = 1 << 18) -> np.ndarray:
    """Per record: does it hold a base outside ACGTN (chunked over records)."""
    n = len(length)
    out = np.zeros(n, bool)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        L = length[a:b].astype(np.int64)
        tot = int(L.sum())
        if tot == 0:
            continue
        rec = np.repeat(np.arange(b - a), L)
        starts = np.concatenate([[0], np.cumsum(L)[:-1]])
        nib = nib_off[a:b][rec] + (np.arange(tot) - starts[rec])
        byte = seq_nt16[nib >> 1]
        code = np.where(nib & 1, byte & 0xF, byte >> 4)
        bad = ~ACGTN[code]
        out[a:b] = np.bincount(rec, weights=bad, minlength=b - a) > 0
    return out


def fastq_records(arr: dict, seed: int = 0, reverse_frac: float = 0.5, qual_rev_frac: float = 0.0,
                  name_len=(8, 40), allow_bad: bool = False, order: np.ndarray = None,
                  check_bad: bool = True) -> dict:
    """Records for the reads of a masking batch (``order``: which reads, in which order)."""
    rng = np.random.default_rng(seed)
    n_reads = len(arr["read_len"])
    idx = np.arange(n_reads) if order is None else np.asarray(order, np.int64)
    n = len(idx)
    seq_len = arr["read_len"][idx].astype(np.int32)
    nib = (2 * arr["seq_off"][idx]).astype(np.int64)
    reverse = (rng.random(n) < reverse_frac).astype(np.uint8)
    if not allow_bad and check_bad and reverse.any():
        reverse[bad_for_reverse(arr["seq_nt16"], nib, seq_len)] = 0
    qual_len = seq_len.copy()
    qual_off = np.concatenate([[0], np.cumsum(qual_len.astype(np.int64))[:-1]]).astype(np.int64)
    quals = rng.integers(2, 41, int(qual_len.sum(dtype=np.int64)), dtype=np.uint8)
    nl = rng.integers(name_len[0], name_len[1] + 1, n).astype(np.int32)
    name_off = np.concatenate([[0], np.cumsum(nl.astype(np.int64))[:-1]]).astype(np.int64)
    names = NAME_ALPHABET[rng.integers(0, len(NAME_ALPHABET), int(nl.sum(dtype=np.int64)))]
    return {
        "seq_bufs": [arr["seq_nt16"]], "seq_sel": np.zeros(n, np.uint8), "seq_nib_off": nib,
        "seq_len": seq_len, "reverse": reverse,
        "qual_bufs": [quals], "qual_sel": np.zeros(n, np.uint8), "qual_off": qual_off,
        "qual_len": qual_len, "qual_rev": (rng.random(n) < qual_rev_frac).astype(np.uint8),
        "names": names, "name_off": name_off, "name_len": nl,
        "mate": (1 + (idx & 1)).astype(np.uint8),
    }


def algorithmic_bytes(recs: dict) -> int:
    """Per record (SURVEY §8(d)-style figure for the formatter): ceil(L/2) nt16 in + Q quality
    bytes in + name bytes in + 36 bytes of record metadata (the 32-byte packed record and its
    u32 length) + the record out (8 + name + L + Q)."""
    L = recs["seq_len"].astype(np.int64)
    Q = recs["qual_len"].astype(np.int64)
    NL = recs["name_len"].astype(np.int64)
    return int(((L + 1) // 2 + Q + NL + 36 + 8 + NL + L + Q).sum())
