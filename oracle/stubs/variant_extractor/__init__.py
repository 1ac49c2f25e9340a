"""Stand-in for ``variant_extractor.VariantExtractor`` (TEST INFRASTRUCTURE ONLY, oracle/).

Reads a plain-text VCF and yields ``VariantRecord``s for SNV/MNV, DEL and INS rows; the
reference's windowing code (short_read_tumor_normal_anonymizer.py:71-131) consumes them.
"""
from .variants import VariantRecord, VariantType


class VariantExtractor:
    def __init__(self, path):
        self._path = path

    def __iter__(self):
        with open(self._path) as fh:
            for line in fh:
                if not line.strip() or line.startswith("#"):
                    continue
                f = line.rstrip("\n").split("\t")
                contig, pos, vid, ref, alt = f[0], int(f[1]), f[2], f[3], f[4]
                if len(ref) == len(alt):
                    yield VariantRecord(contig, pos, pos + len(ref) - 1, len(ref), vid, ref, alt,
                                        VariantType.SNV, None)
                elif len(ref) > len(alt):
                    yield VariantRecord(contig, pos, pos + len(ref) - 1, len(ref) - len(alt), vid,
                                        ref, alt, VariantType.DEL, None)
                else:
                    yield VariantRecord(contig, pos, pos, len(alt) - len(ref), vid, ref, alt,
                                        VariantType.INS, None)

    def close(self):
        pass
