"""CPU restatement of the germline indel tally over a ganon_batch.

TEST INFRASTRUCTURE ONLY: imported by tests/ (and through ``pyoracle.OracleEngine``) as the
checker of ``ganon_indel_*`` (genomeanonymizer_amd/csrc/ganon_indel.hip) — never by the product.

Per scope it follows the reference literally:
* reads are met in registration order — by first pileup column (ref_start), tumor before normal,
  file order (the scope's incidence order lists tumor then normal reads in file order) — and each
  read's CIGAR is walked once (classify_variation_in_pileup_column's seen_read_alns,
  variation_classifier.py:208-215);
* ``process_indels`` (variation_classifier.py:52-141): for an I/D op,
  ``pos = reference_start + current_cigar_len`` (M/D/N/=/X before it),
  ``in_read_pos = current_cigar_len + read_consumed_bases`` (the counter adds S/H/I and subtracts
  D), ``end = pos + 1`` (INS) or ``pos + length - 1`` (DEL),
  ``allele = query_sequence[in_read_pos:in_read_end + 1]`` with ``in_read_end = in_read_pos +
  length - 1`` (INS) or ``in_read_pos + 1`` (DEL); calls are equal on (pos, end, type, length,
  allele) (variants.py:83-96); ``supporting_reads[read] = in_read_pos`` (last assignment wins,
  first insertion keeps its place); the SomaticVariationType state machine (variants.py:33-39);
* ``mask_germline_variants`` (anonymizer_methods.py:537-556) runs at normal pileup columns only:
  a call is masked iff it is TUMORAL_NORMAL and a normal read of the scope covers ``pos``
  (``ref_start <= pos < bam_endpos``). The kept window variant is the host's check, as in the
  product.

Output: the same records as ``ganon_indel_download`` (include/ganon.h), as a list of tuples
``(scope, pos, length, type, rank, kind, read, in_read_pos)``; rank = index of the call in the
reference's ``called_indels[pos]`` list.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np

NT16 = "=ACMGRSVTWYHKDBN"
DEL, INS = 2, 3
CALL, SUPPORT = 0, 1
_TN = 3   # state: bit 0 tumor seen, bit 1 normal seen


def _read_seq(a: dict, r: int) -> str:
    L = int(a["read_len"][r])
    o = int(a["seq_off"][r])
    b = a["seq_nt16"][o:o + (L + 1) // 2]
    nib = np.empty(2 * len(b), np.uint8)
    nib[0::2] = b >> 4
    nib[1::2] = b & 0xF
    return "".join(NT16[c] for c in nib[:L])


def _read_end(a: dict, r: int) -> int:
    c = a["cigar"][int(a["cig_off"][r]):int(a["cig_off"][r]) + int(a["n_cig"][r])]
    op, ln = c & 0xF, c >> 4
    rl = int(ln[np.isin(op, (0, 2, 3, 7, 8))].sum())
    return int(a["ref_start"][r]) + (rl if rl > 0 else 1)


class _Call:
    __slots__ = ("key", "state", "support", "first_read", "first_irp")

    def __init__(self, key, read, irp):
        self.key = key
        self.state = 0
        self.support: Dict[int, int] = {}
        self.first_read = read
        self.first_irp = irp


def indel_records(a: dict) -> List[tuple]:
    n_scopes = len(a["scope_span_start"])
    inc_off = a["scope_incid_off"]
    # tallied reads: the batch's indel CSR when the plan leaves later alignments out (seen_read_alns)
    t_off = a.get("indel_incid_off", inc_off)
    t_read = a.get("indel_incid_read", a["incid_read"])
    out: List[tuple] = []
    seq_cache: Dict[int, str] = {}
    end_cache: Dict[int, int] = {}
    # a scope registers calls only through tallied reads with an I/D op: the others are skipped up
    # front (a full configs[1] batch has ~1.2 M scopes, ~15 % of them with such a read)
    n_cig = a["n_cig"].astype(np.int64)
    tot = int(n_cig.sum())
    first = np.concatenate([[0], np.cumsum(n_cig)[:-1]]) if len(n_cig) else np.zeros(0, np.int64)
    # every read's own CIGAR words (cig_off: the buffer may hold them in any order)
    idx = np.repeat(a["cig_off"].astype(np.int64) - first, n_cig) + np.arange(tot)
    ops = a["cigar"][idx] & 0xF
    id_op = (ops == 1) | (ops == 2)
    has_id = np.zeros(len(n_cig), bool)
    if id_op.any():
        has_id[np.repeat(np.arange(len(n_cig)), n_cig)[id_op]] = True
    t_has = has_id[np.asarray(t_read, np.int64)].astype(np.int64)
    per_scope = np.add.reduceat(np.concatenate([t_has, [0]]), np.asarray(t_off[:-1], np.int64)) \
        if n_scopes else np.zeros(0, np.int64)
    per_scope[np.asarray(t_off[1:]) == np.asarray(t_off[:-1])] = 0   # (reduceat of an empty range)
    for s in np.nonzero(per_scope)[0].tolist():
        reads = a["incid_read"][int(inc_off[s]):int(inc_off[s + 1])].astype(np.int64)
        tallied = t_read[int(t_off[s]):int(t_off[s + 1])].astype(np.int64)
        order = np.argsort(a["ref_start"][tallied], kind="stable")
        calls: Dict[int, List[_Call]] = {}
        for r in tallied[order].tolist():
            c0 = int(a["cig_off"][r])
            cig = a["cigar"][c0:c0 + int(a["n_cig"][r])].tolist()
            if not any((w & 0xF) in (1, 2) for w in cig):
                continue
            seq = seq_cache.get(r)
            if seq is None:
                seq = seq_cache[r] = _read_seq(a, r)
            ds = int(a["dataset"][r])
            start = int(a["ref_start"][r])
            cur_len = 0
            consumed = 0
            for w in cig:
                op, n = w & 0xF, w >> 4
                if op in (1, 2):
                    pos = start + cur_len
                    irp = cur_len + consumed
                    vt = INS if op == 1 else DEL
                    end = pos + 1 if vt == INS else pos + n - 1
                    in_read_end = irp + n - 1 if vt == INS else irp + 1
                    key = (end, vt, n, seq[irp:in_read_end + 1].upper())
                    lst = calls.setdefault(pos, [])
                    call = next((c for c in lst if c.key == key), None)
                    if call is None:
                        call = _Call(key, r, irp)
                        lst.append(call)
                    call.support[r] = irp
                    call.state |= 1 << ds
                if op in (0, 2, 3, 7, 8):
                    cur_len += n
                if op in (4, 5, 1):
                    consumed += n
                if op == 2:
                    consumed -= n
        if not calls:
            continue
        normals = [r for r in reads.tolist() if int(a["dataset"][r]) == 1]
        for r in normals:
            if r not in end_cache:
                end_cache[r] = _read_end(a, r)
        for pos in sorted(calls):
            covered = any(int(a["ref_start"][r]) <= pos < end_cache[r] for r in normals)
            if not covered:
                continue
            for rank, c in enumerate(calls[pos]):
                if c.state != _TN:
                    continue
                _, vt, n, _ = c.key
                out.append((s, pos, n, vt, rank, CALL, c.first_read, c.first_irp))
                for r, irp in c.support.items():
                    if int(a["write_scope"][r]) == s:
                        out.append((s, pos, n, vt, rank, SUPPORT, r, irp))
    return out
