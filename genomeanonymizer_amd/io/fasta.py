"""Reference FASTA: raw text per contig (for the host indel path and statistics) and the
whole genome packed to upper-cased nt16 nibbles for the device (include/ganon.h ref_nt16).

Mirrors what the reference reads through ``pysam.FastaFile``: ``references``, ``lengths``
and ``fetch(contig, start, end)`` (variation_classifier.py:89, :193; short_read_tumor_normal_
anonymizer.py:61-64, :245-250).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List

import numpy as np

from .. import native


class FastaRef:
    def __init__(self, path: str):
        self.filename = path
        names: List[str] = []
        chunks: List[List[bytes]] = []
        with open(path, "rb") as fh:
            for line in fh:
                line = line.rstrip(b"\r\n")
                if line.startswith(b">"):
                    names.append(line[1:].split()[0].decode())
                    chunks.append([])
                elif line:
                    chunks[-1].append(line)
        self.references = tuple(names)
        self._seq: Dict[str, bytes] = {n: b"".join(c) for n, c in zip(names, chunks)}
        self.lengths = tuple(len(self._seq[n]) for n in names)
        self.index = {n: i for i, n in enumerate(names)}
        self._packed = None
        self._nib_off = None

    def fetch(self, contig: str, start: int = None, end: int = None) -> str:
        s = self._seq[contig]
        start = 0 if start is None else start
        end = len(s) if end is None else end
        if start < 0:
            raise ValueError("start out of range")
        return s[start:end].decode()

    def raw(self, contig: str) -> bytes:
        return self._seq[contig]

    def packed(self):
        """(nt16 bytes of the whole genome, nibble offset of each contig). Each contig starts
        on a byte boundary; lower case is folded to upper case (ref_base.upper(), VC:194)."""
        if self._packed is None:
            lib = native.host_lib()
            offs = {}
            parts = []
            nib = 0
            for n in self.references:
                s = self._seq[n]
                buf = np.zeros((len(s) + 1) // 2, np.uint8)
                if len(s):
                    lib.ganon_pack_nt16(s, len(s), buf.ctypes.data_as(C.POINTER(C.c_uint8)))
                offs[n] = nib
                parts.append(buf)
                nib += 2 * len(buf)
            self._nib_off = offs      # before _packed: another thread may test _packed meanwhile
            self._packed = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
        return self._packed, self._nib_off
