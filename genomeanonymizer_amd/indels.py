"""Host side of germline indels: the variable-length edits.

The tally — ``process_indels`` (variation_classifier.py:52-141), the tumor/normal state machine
and the normal-column check of ``mask_germline_variants`` (anonymizer_methods.py:537-556) — runs on
the GPU (``ganon_indel_*``, csrc/ganon_indel.hip); ``anonymizer_methods.indel_results`` turns its
records into per-read left-over lists. This module applies them when a pair is yielded
(AM:254-270): stable sort by ``VariantType`` value (DEL before INS), offsets not shifted between
edits; ``mask_or_modify_indel`` (AM:178-203) edits the sequence and the
*forward-oriented* qualities (which interacts with SURVEY Q1 on reverse reads).
"""
from __future__ import annotations

import dataclasses
from typing import List, Tuple

import numpy as np

from .io.bam import ReadTable
from .variants import VariantType

NT16 = "=ACMGRSVTWYHKDBN"


_NT16_BYTES = np.frombuffer(NT16.encode(), np.uint8)


def query_sequence(t: ReadTable, row: int) -> str:
    L = int(t.l_seq[row])
    o = int(t.seq_off[row])
    b = t.seq[o:o + (L + 1) // 2]
    nib = np.empty(2 * len(b), np.uint8)
    nib[0::2] = b >> 4
    nib[1::2] = b & 0xF
    return _NT16_BYTES[nib[:L]].tobytes().decode()


@dataclasses.dataclass
class IndelCall:
    """A masked TN indel call as CalledGenomicVariant holds it (variants.py:40-56): 0-based pos,
    end (pos + 1 for INS, pos + length - 1 for DEL), type, length, read allele, reference allele."""
    pos: int
    end: int
    variant_type: VariantType
    length: int
    allele: str
    ref_allele: str


def apply_indel(seq: bytearray, qual_fwd: List[int], irp: int, c: IndelCall):
    """mask_or_modify_indel (AM:178-203) on (ASCII seq, forward qualities). Raises ValueError like
    the reference when the lengths diverge."""
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


def apply_leftovers(seq: bytearray, qual_fwd: List[int], edits: List[Tuple[int, IndelCall]]):
    """mask_or_anonymize_left_over_variants + mask_or_modify_indel on (ASCII seq, forward
    qualities)."""
    for irp, c in sorted(edits, key=lambda e: e[1].variant_type.value):
        seq, qual_fwd = apply_indel(seq, qual_fwd, irp, c)
    return seq, qual_fwd


def _nan_int():
    # int(np.mean([])) -> int(nan) raises ValueError in the reference as well
    raise ValueError("cannot convert float NaN to integer")
