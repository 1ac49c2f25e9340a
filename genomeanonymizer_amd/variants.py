"""Variant data model of the reference, restated for the host side.

* ``VariantType`` — variant-extractor's enum in the order the statistics header uses
  (short_read_tumor_normal_anonymizer.py:218-219: SNV, DEL, INS, DUP, INV, CNV, TRA, SGL).
* ``SomaticVariationType`` and its state machine (variants.py:33-39,
  variation_classifier.py:163-182).
* ``compare`` (variants.py:9-25) used by the region clustering.
* ``WindowVariant`` — the VCF variant a window keeps (CalledGenomicVariant.from_variant_record,
  variants.py:58-62) with the identity used at anonymizer_methods.py:546-547
  (``__eq__`` on seq_name, variant_type, pos, end, length, allele; variants.py:83-96) and the
  ``__str__`` that ends up in the statistics keys (variants.py:98-101).
"""
from __future__ import annotations

import dataclasses
from enum import Enum
from typing import Optional, Tuple


class VariantType(Enum):
    SNV = 1
    DEL = 2
    INS = 3
    DUP = 4
    INV = 5
    CNV = 6
    TRA = 7
    SGL = 8


class SomaticVariationType(Enum):
    UNCLASSIFIED = 0
    NORMAL_SINGLE_READ_VARIANT = 1
    TUMORAL_SINGLE_READ_VARIANT = 2
    NORMAL_ONLY_VARIANT = 3
    TUMORAL_ONLY_VARIANT = 4
    TUMORAL_NORMAL_VARIANT = 5


_S = SomaticVariationType


def advance_state(state: SomaticVariationType, dataset: int) -> SomaticVariationType:
    """One observation of a call in a tumor (0) or normal (1) read."""
    if state is _S.UNCLASSIFIED:
        return _S.TUMORAL_SINGLE_READ_VARIANT if dataset == 0 else _S.NORMAL_SINGLE_READ_VARIANT
    if dataset == 0:
        if state in (_S.NORMAL_SINGLE_READ_VARIANT, _S.NORMAL_ONLY_VARIANT):
            return _S.TUMORAL_NORMAL_VARIANT
        if state is _S.TUMORAL_SINGLE_READ_VARIANT:
            return _S.TUMORAL_ONLY_VARIANT
    else:
        if state in (_S.TUMORAL_SINGLE_READ_VARIANT, _S.TUMORAL_ONLY_VARIANT):
            return _S.TUMORAL_NORMAL_VARIANT
        if state is _S.NORMAL_SINGLE_READ_VARIANT:
            return _S.NORMAL_ONLY_VARIANT
    return state


def compare(seq_idx1: int, first1: int, last1: int, seq_idx2: int, first2: int, last2: int) -> int:
    """Interval order with overlap: -3/3 other contig, -2/2 disjoint, -1/1 overlapping, 0 equal."""
    overlap = first2 <= last1 and last2 >= first1
    if seq_idx1 != seq_idx2:
        return -3 if seq_idx1 < seq_idx2 else 3
    if last1 != last2:
        if last1 < last2:
            return -1 if overlap else -2
        return 1 if overlap else 2
    if first1 != first2:
        return -1 if first1 < first2 else 1
    return 0


@dataclasses.dataclass(frozen=True)
class VariantRecord:
    """What the reference reads from a variant-extractor record (1-based pos/end)."""
    contig: str
    pos: int
    end: int
    length: int
    ref: str
    alt: str
    variant_type: VariantType
    alt_sv_breakend: Optional[Tuple[str, int]] = None   # (contig, pos) of a breakend mate


@dataclasses.dataclass(frozen=True)
class WindowVariant:
    """CalledGenomicVariant built from a VCF record: 0-based pos and end."""
    seq_name: str
    pos: int
    end: int
    variant_type: VariantType
    length: int
    allele: str
    ref_allele: str

    @classmethod
    def from_record(cls, r: VariantRecord) -> "WindowVariant":
        return cls(r.contig, r.pos - 1, r.end - 1, r.variant_type, r.length, r.alt, r.ref)

    def identity(self):
        return (self.seq_name, self.variant_type, self.pos, self.end, self.length, self.allele)

    def __str__(self) -> str:
        return (f"seq_name: {self.seq_name} pos: {self.pos} end: {self.end} var_type: {self.variant_type} "
                f"length: {self.length} alt_allele: {self.allele} ref_allele: {self.ref_allele} "
                f"somatic_variation_type: {SomaticVariationType.UNCLASSIFIED}")


NT16 = "=ACMGRSVTWYHKDBN"


def kept_snv(variant: Optional[WindowVariant]) -> Tuple[int, int]:
    """(keep_pos, keep_code) for the device: the SNV call (p, allele) equal to the kept
    variant, i.e. pos == end == p, length == 1 and allele == alt; (-1, 0) when no called SNV
    can equal it."""
    if variant is None or variant.variant_type is not VariantType.SNV:
        return -1, 0
    if variant.end != variant.pos or variant.length != 1 or len(variant.allele) != 1:
        return -1, 0
    a = variant.allele
    if a not in NT16 or a == "N":
        return -1, 0
    return variant.pos, NT16.index(a)
