"""Host path for germline indels (GPU indel tally is a §8(f) "next" row).

Restates, per scope:
* ``process_indels`` (variation_classifier.py:52-141), called once per read when the scope
  first meets it: every I/D CIGAR op becomes a call keyed by (pos, end, type, length,
  allele) with the reference's read-offset bookkeeping, including its quirks — ``H`` is
  counted as read-consuming and ``N`` as reference- but not read-consuming;
  INS allele = the inserted read bases, DEL allele = the 2 read bases after the gap,
  ref allele = FASTA[pos:end + 1];
* the same tumor/normal state machine as SNVs;
* masking at the normal column ``pos`` (anonymizer_methods.py:477-488, :537-556): TN calls
  other than the kept variant are counted for the statistics and appended to every
  supporting read's left-over list — only when a normal read of the scope covers ``pos``
  (no normal column there means no masking);
* applying left-overs when the pair is yielded (AM:254-270): stable sort by
  ``VariantType`` value (DEL before INS), offsets not shifted between edits;
  ``mask_or_modify_indel`` (AM:178-203) edits the sequence and the *forward-oriented*
  qualities (which interacts with SURVEY Q1 on reverse reads).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

import numpy as np

from .io.bam import ReadTable
from .io.fasta import FastaRef
from .variants import SomaticVariationType, VariantType, WindowVariant, advance_state

NT16 = "=ACMGRSVTWYHKDBN"
_TN = SomaticVariationType.TUMORAL_NORMAL_VARIANT


def query_sequence(t: ReadTable, row: int) -> str:
    L = int(t.l_seq[row])
    o = int(t.seq_off[row])
    b = t.seq[o:o + (L + 1) // 2]
    nib = np.empty(2 * len(b), np.uint8)
    nib[0::2] = b >> 4
    nib[1::2] = b & 0xF
    return "".join(NT16[c] for c in nib[:L])


@dataclasses.dataclass
class IndelCall:
    pos: int
    end: int
    variant_type: VariantType
    length: int
    allele: str
    ref_allele: str
    state: SomaticVariationType = SomaticVariationType.UNCLASSIFIED
    support: Dict[Tuple[int, int], int] = dataclasses.field(default_factory=dict)


def has_indel_ops(t: ReadTable, row: int) -> bool:
    c = t.cigar_of(row) & 0xF
    return bool(np.any((c == 1) | (c == 2)))


def scope_indels(contig: str, reg_order: List[Tuple[int, int]], tables: Tuple[ReadTable, ReadTable],
                 fasta: FastaRef, normal_cover, keep: Optional[WindowVariant]):
    """Returns (counts[VariantType] of masked TN indel calls, left-overs per (ds,row)).

    ``reg_order``: the scope's reads in first-appearance order; ``normal_cover(pos)`` tells
    whether a normal read of the scope covers ``pos`` (a normal pileup column exists)."""
    calls: Dict[int, List[IndelCall]] = {}
    for ds, row in reg_order:
        t = tables[ds]
        if not has_indel_ops(t, row):
            continue
        seq = None
        start = int(t.pos[row])
        cur_len = 0
        consumed = 0
        for w in t.cigar_of(row).tolist():
            op, n = w & 0xF, w >> 4
            if op in (1, 2):
                if seq is None:
                    seq = query_sequence(t, row)
                pos = start + cur_len
                irp = cur_len + consumed
                vt = VariantType.INS if op == 1 else VariantType.DEL
                end = pos + 1 if vt is VariantType.INS else pos + n - 1
                in_read_end = irp + n - 1 if vt is VariantType.INS else irp + 1
                alt = seq[irp:in_read_end + 1].upper()
                ref = fasta.fetch(contig, pos, end + 1).upper()
                lst = calls.setdefault(pos, [])
                call = None
                for c in lst:
                    if (c.variant_type, c.end, c.length, c.allele) == (vt, end, n, alt):
                        call = c
                        break
                if call is None:
                    call = IndelCall(pos, end, vt, n, alt, ref)
                    lst.append(call)
                call.support[(ds, row)] = irp
                call.state = advance_state(call.state, ds)
            if op in (0, 2, 3, 7, 8):
                cur_len += n
            if op in (4, 5, 1):
                consumed += n
            if op == 2:
                consumed -= n
    counts = {VariantType.DEL: 0, VariantType.INS: 0}
    left: Dict[Tuple[int, int], List[Tuple[int, IndelCall]]] = {}
    keep_id = keep.identity() if keep is not None else None
    for pos in sorted(calls):
        if not normal_cover(pos):
            continue
        for c in calls[pos]:
            if c.state is not _TN:
                continue
            if keep_id is not None and (contig, c.variant_type, c.pos, c.end, c.length, c.allele) == keep_id:
                continue
            counts[c.variant_type] += 1
            for key, irp in c.support.items():
                left.setdefault(key, []).append((irp, c))
    return counts, left


def apply_leftovers(seq: bytearray, qual_fwd: List[int], edits: List[Tuple[int, IndelCall]]):
    """mask_or_anonymize_left_over_variants + mask_or_modify_indel on (ASCII seq, forward
    qualities). Raises ValueError like the reference when lengths diverge."""
    for irp, c in sorted(edits, key=lambda e: e[1].variant_type.value):
        if c.variant_type is VariantType.INS:
            seq = seq[:irp] + seq[irp + c.length:]
            qual_fwd = qual_fwd[:irp] + qual_fwd[irp + c.length:]
        elif c.variant_type is VariantType.DEL:
            avg = int(float(sum(qual_fwd)) / len(qual_fwd)) if qual_fwd else _nan_int()
            seq = seq[:irp] + bytearray(c.ref_allele.encode()) + seq[irp:]
            qual_fwd = qual_fwd[:irp] + [avg] * c.length + qual_fwd[irp:]
        if len(seq) != len(qual_fwd):
            raise ValueError("Length of the modified qualities does not match the length of the modified sequence")
    return seq, qual_fwd


def _nan_int():
    # int(np.mean([])) -> int(nan) raises ValueError in the reference as well
    raise ValueError("cannot convert float NaN to integer")
