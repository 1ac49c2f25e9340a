"""Minimal VCF reader producing the fields the reference takes from variant-extractor
4.0.6 (``VariantExtractor`` records: contig, pos, end, length, ref, alt, variant_type,
alt_sv_breakend; short_read_tumor_normal_anonymizer.py:71-131, :915-923).

variant-extractor is a pinned dependency of the reference that is absent here, so its
exact ``end``/``length`` conventions are not pinned. This reader uses:
equal-length REF/ALT -> SNV with end = pos + len(ref) - 1, length = len(ref);
longer REF -> DEL with end = pos + len(ref) - 1, length = len(ref) - len(alt);
longer ALT -> INS with end = pos, length = len(alt) - len(ref);
symbolic ALTs <DEL>/<INS>/<DUP>/<INV>/<CNV> use INFO END/SVLEN; breakend ALTs -> TRA
(other contig) or SGL. These only decide window bounds and the kept-variant identity.
"""
from __future__ import annotations

import re
from typing import List

from ..variants import VariantRecord, VariantType

_BND = re.compile(r"[\[\]]([^:\[\]]+):(\d+)[\[\]]")


def _info(info: str) -> dict:
    d = {}
    for item in info.split(";"):
        if "=" in item:
            k, v = item.split("=", 1)
            d[k] = v
    return d


def read_vcf(path: str) -> List[VariantRecord]:
    out: List[VariantRecord] = []
    opener = open
    if path.endswith(".gz"):
        import gzip
        opener = gzip.open
    with opener(path, "rt") as fh:
        for line in fh:
            if not line.strip() or line.startswith("#"):
                continue
            f = line.rstrip("\n").split("\t")
            contig, pos, ref, alt = f[0], int(f[1]), f[3], f[4]
            info = _info(f[7]) if len(f) > 7 else {}
            for a in alt.split(","):
                out.append(_record(contig, pos, ref, a, info))
    return out


def _record(contig: str, pos: int, ref: str, alt: str, info: dict) -> VariantRecord:
    if alt.startswith("<") and alt.endswith(">"):
        kind = alt[1:-1].split(":")[0]
        end = int(info.get("END", pos))
        svlen = abs(int(info.get("SVLEN", end - pos)))
        vt = {"DEL": VariantType.DEL, "INS": VariantType.INS, "DUP": VariantType.DUP,
              "INV": VariantType.INV, "CNV": VariantType.CNV}.get(kind, VariantType.SGL)
        return VariantRecord(contig, pos, end, svlen, ref, alt, vt)
    m = _BND.search(alt)
    if m:
        mate_contig, mate_pos = m.group(1), int(m.group(2))
        vt = VariantType.TRA if mate_contig != contig else VariantType.INV
        return VariantRecord(contig, pos, mate_pos if mate_contig == contig else pos,
                             abs(mate_pos - pos) if mate_contig == contig else 0, ref, alt, vt,
                             (mate_contig, mate_pos))
    if alt in (".", "*") or alt.endswith(".") or alt.startswith("."):
        return VariantRecord(contig, pos, pos, 0, ref, alt, VariantType.SGL)
    if len(ref) == len(alt):
        return VariantRecord(contig, pos, pos + len(ref) - 1, len(ref), ref, alt, VariantType.SNV)
    if len(ref) > len(alt):
        return VariantRecord(contig, pos, pos + len(ref) - 1, len(ref) - len(alt), ref, alt, VariantType.DEL)
    return VariantRecord(contig, pos, pos, len(alt) - len(ref), ref, alt, VariantType.INS)
