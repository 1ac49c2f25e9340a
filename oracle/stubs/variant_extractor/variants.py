"""Stand-in for variant-extractor 4.0.6's record types (TEST INFRASTRUCTURE ONLY, oracle/).

variant-extractor is a pinned dependency of the reference (pyproject.toml:12) that is not
installed here. Only the members the reference reads are modelled: ``VariantType`` with the
order of the statistics header (short_read_tumor_normal_anonymizer.py:218-219) and a
``VariantRecord`` with contig, 1-based pos/end, length, ref, alt, variant_type and
alt_sv_breakend. Conventions for ``end``/``length`` are this build's choice (parity unpinned):
SNV end = pos, length = 1; DEL end = pos + len(ref) - 1, length = len(ref) - len(alt);
INS end = pos, length = len(alt) - len(ref).
"""
from enum import Enum
from typing import NamedTuple, Optional


class VariantType(Enum):
    SNV = 1
    DEL = 2
    INS = 3
    DUP = 4
    INV = 5
    CNV = 6
    TRA = 7
    SGL = 8


class BreakendSVRecord(NamedTuple):
    prefix: Optional[str]
    bracket: str
    contig: str
    pos: int
    suffix: Optional[str]


class VariantRecord(NamedTuple):
    contig: str
    pos: int
    end: int
    length: int
    id: Optional[str]
    ref: str
    alt: str
    variant_type: VariantType
    alt_sv_breakend: Optional[BreakendSVRecord]
