"""Coordinate-sorted BAM -> structure-of-arrays read table (native decoder).

Stands in for what the reference reads through pysam ``AlignedSegment`` objects
(query_name, flags, reference_start/end, cigar, query_sequence, qualities, SA tag): one
numpy column per field, one packed-nt16 sequence blob in BAM layout (which is exactly the
device batch layout of include/ganon.h). ``fetch`` reproduces htslib region semantics:
records of a contig overlapping [start, stop) in file order, overlap computed with
``bam_endpos`` (pos + reference length, or pos + 1 for unmapped / zero-length records).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional

import numpy as np

from .. import native

FLAG_PAIRED = 0x1
FLAG_UNMAP = 0x4
FLAG_REVERSE = 0x10
FLAG_READ1 = 0x40
FLAG_READ2 = 0x80
FLAG_SECONDARY = 0x100
FLAG_SUPPLEMENTARY = 0x800


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


def _blob(ptr, n, dtype=np.uint8):
    if n == 0:
        return np.zeros(0, dtype)
    addr = ptr if isinstance(ptr, int) else C.cast(ptr, C.c_void_p).value
    return np.frombuffer(C.string_at(addr, n * np.dtype(dtype).itemsize), dtype=dtype).copy()


class ReadTable:
    """All records of one BAM file, in file order."""

    def __init__(self, path: str, threads: int = 8):
        lib = native.host_lib()
        h = C.c_void_p()
        rc = lib.ganon_bam_open(os.fsencode(path), int(threads), C.byref(h))
        if rc != 0:
            raise native.GanonError(f"cannot decode {path}: {lib.ganon_host_last_error().decode()}")
        try:
            v = native.BamView()
            lib.ganon_bam_view_get(h, C.byref(v))
            n = int(v.n_records)
            self.path = path
            self.n = n
            names_blob = _blob(v.names, int(v.names_bytes))
            self.ref_names: List[str] = []
            ref_name_off = _arr(v.ref_name_off, v.n_ref, np.int64)
            raw = int(v.ref_names)
            for o in ref_name_off:
                self.ref_names.append(C.string_at(raw + int(o)).decode())
            self.ref_lens = _arr(v.ref_len, v.n_ref, np.int64)
            self.tid = _arr(v.tid, n, np.int32)
            self.pos = _arr(v.pos, n, np.int32)
            self.end = _arr(v.end, n, np.int32)
            self.flag = _arr(v.flag, n, np.int32)
            self.mapq = _arr(v.mapq, n, np.int32)
            self.l_seq = _arr(v.l_seq, n, np.int32)
            self.n_cigar = _arr(v.n_cigar, n, np.int32)
            self.mate_tid = _arr(v.mate_tid, n, np.int32)
            self.mate_pos = _arr(v.mate_pos, n, np.int32)
            self.name_off = _arr(v.name_off, n, np.int64)
            self.name_len = _arr(v.name_len, n, np.int32)
            self.cig_off = _arr(v.cig_off, n, np.int64)
            self.seq_off = _arr(v.seq_off, n, np.int64)
            self.qual_off = _arr(v.qual_off, n, np.int64)
            self.aux_off = _arr(v.aux_off, n, np.int64)
            self.aux_len = _arr(v.aux_len, n, np.int32)
            self.names_blob = names_blob
            self.cigar = _blob(v.cigar, int(v.cigar_ops), np.uint32).copy()
            self.seq = _blob(v.seq, int(v.seq_bytes)).copy()
            self.qual = _blob(v.qual, int(v.qual_bytes)).copy()
            self.aux = _blob(v.aux, int(v.aux_bytes)).copy()
        finally:
            lib.ganon_bam_close(h)
        self._names: Optional[List[str]] = None
        self.is_unmapped = (self.flag & FLAG_UNMAP) != 0
        self.is_reverse = (self.flag & FLAG_REVERSE) != 0
        # pair slot as AnonymizedRead.get_pair_idx (anonymizer_methods.py:119-123): -1 = neither flag
        self.mate_idx = np.where(self.flag & FLAG_READ1, 0, np.where(self.flag & FLAG_READ2, 1, -1)).astype(np.int8)
        self.has_cigar = self.n_cigar > 0
        self._index: Dict[int, tuple] = {}

    @property
    def names(self) -> List[str]:
        """Read names as str (built on first use: the native planner and the formatters work on
        ``names_blob`` / ``name_off`` / ``name_len`` directly)."""
        if self._names is None:
            nb = self.names_blob.tobytes()
            self._names = [nb[o:o + l].decode() for o, l in zip(self.name_off.tolist(), self.name_len.tolist())]
        return self._names

    def name(self, i: int) -> str:
        o = int(self.name_off[i])
        return self.names_blob[o:o + int(self.name_len[i])].tobytes().decode()

    # -- htslib-style region query -----------------------------------------------------
    def _tid_index(self, tid: int):
        ix = self._index.get(tid)
        if ix is None:
            rows = np.nonzero(self.tid == tid)[0].astype(np.int64)
            # int64: searchsorted with a Python int would cast an int32 array on every call
            pos = self.pos[rows].astype(np.int64)
            if len(pos) > 1 and np.any(np.diff(pos) < 0):
                raise ValueError(f"{self.path}: records of contig {tid} are not coordinate sorted")
            span = int((self.end[rows] - pos).max()) if len(rows) else 1
            ix = (rows, pos, span)
            self._index[tid] = ix
        return ix

    def tid_of(self, contig: str) -> int:
        try:
            return self.ref_names.index(contig)
        except ValueError:
            raise ValueError(f"invalid contig `{contig}`") from None

    def fetch(self, contig: str, start: Optional[int] = None, stop: Optional[int] = None) -> np.ndarray:
        """Record indices overlapping [start, stop) of ``contig`` in file order.

        Region errors follow pysam's region parser (raised as ValueError), which the
        reference hits for windows closer than 2003 bp or starting before 1001.
        """
        tid = self.tid_of(contig)
        length = int(self.ref_lens[tid])
        rstart = 0 if start is None else int(start)
        rstop = length if stop is None else int(stop)
        if rstart > rstop:
            raise ValueError(f"invalid coordinates: start ({rstart}) > stop ({rstop})")
        if rstart < 0:
            raise ValueError(f"start out of range ({rstart})")
        rows, pos, span = self._tid_index(tid)
        lo = int(np.searchsorted(pos, rstart - span, side="left"))
        hi = int(np.searchsorted(pos, rstop, side="left"))
        cand = rows[lo:hi]
        return cand[self.end[cand] > rstart]

    def has_tag(self, i: int, tag: bytes) -> bool:
        a = self.aux[self.aux_off[i]:self.aux_off[i] + self.aux_len[i]].tobytes()
        j = 0
        sizes = {ord(c): s for c, s in zip("AcCsSiIf", (1, 1, 1, 2, 2, 4, 4, 4))}
        while j + 3 <= len(a):
            t, ty = a[j:j + 2], a[j + 2]
            if t == tag:
                return True
            j += 3
            if ty in sizes:
                j += sizes[ty]
            elif ty in (ord("Z"), ord("H")):
                j = a.index(b"\x00", j) + 1
            elif ty == ord("B"):
                sub = a[j]
                cnt = int.from_bytes(a[j + 1:j + 5], "little")
                j += 5 + sizes[sub] * cnt
            else:
                raise ValueError(f"bad aux type in record {i}")
        return False

    def cigar_of(self, i: int) -> np.ndarray:
        o = int(self.cig_off[i])
        return self.cigar[o:o + int(self.n_cigar[i])]
