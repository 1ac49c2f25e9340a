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


class _Decoded:
    """Owns one native ``ganon_bam`` (decoded records); released when the last array viewing its
    memory is gone."""
    __slots__ = ("h", "__weakref__")

    def __init__(self, h):
        self.h = h

    def __del__(self):
        if self.h:
            native.host_lib().ganon_bam_close(self.h)
            self.h = None


def _view(ptr, n, dtype, owner: _Decoded):
    """A writable numpy view of n elements of native memory (no copy); the view keeps `owner`, and
    with it the native buffers, alive."""
    if n == 0:
        return np.zeros(0, dtype)
    addr = ptr if isinstance(ptr, int) else C.cast(ptr, C.c_void_p).value
    buf = (C.c_char * (n * np.dtype(dtype).itemsize)).from_address(addr)
    buf._owner = owner
    return np.frombuffer(buf, dtype=dtype)


class ReadTable:
    """All records of one BAM file, in file order."""

    def __init__(self, path: str, threads: int = 8, handle=None):
        """Decode the whole file, or take the records of an open ``ganon_bam`` handle (one
        reference sequence from ``BamReader.contig``); the table owns the handle from here on."""
        lib = native.host_lib()
        if handle is None:
            h = C.c_void_p()
            rc = lib.ganon_bam_open(os.fsencode(path), int(threads), C.byref(h))
            if rc != 0:
                raise native.GanonError(f"cannot decode {path}: {lib.ganon_host_last_error().decode()}")
        else:
            h = handle
        owner = _Decoded(h)
        v = native.BamView()
        lib.ganon_bam_view_get(h, C.byref(v))
        self._load(path, v, owner)
        self._finish()

    def _load(self, path: str, v, owner: _Decoded) -> None:
        """Per-record columns are copied (small); the byte blobs (names, CIGAR words, sequences,
        qualities, aux) are views of the decoder's buffers, which `owner` frees with the last view."""
        n = int(v.n_records)
        self.path = path
        self.n = n
        self.ref_names: List[str] = []
        ref_name_off = _arr(v.ref_name_off, v.n_ref, np.int64)
        raw = int(v.ref_names) if v.n_ref else 0
        for o in ref_name_off:
            self.ref_names.append(C.string_at(raw + int(o)).decode())
        self.ref_lens = _arr(v.ref_len, v.n_ref, np.int64)
        for f in ("tid", "pos", "end", "flag", "mapq", "l_seq", "n_cigar", "mate_tid", "mate_pos", "tlen", "name_len",
                  "aux_len"):
            setattr(self, f, _arr(getattr(v, f), n, np.int32))
        for f in ("name_off", "cig_off", "seq_off", "qual_off", "aux_off"):
            setattr(self, f, _arr(getattr(v, f), n, np.int64))
        self.names_blob = _view(v.names, int(v.names_bytes), np.uint8, owner)
        self.cigar = _view(v.cigar, int(v.cigar_ops), np.uint32, owner)
        self.seq = _view(v.seq, int(v.seq_bytes), np.uint8, owner)
        self.qual = _view(v.qual, int(v.qual_bytes), np.uint8, owner)
        self.aux = _view(v.aux, int(v.aux_bytes), np.uint8, owner)

    def _finish(self) -> None:
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

    def may_be_complex(self) -> bool:
        """Any secondary / supplementary record or SA tag candidate (cheap pre-check)."""
        return bool(np.any(self.flag & (FLAG_SECONDARY | FLAG_SUPPLEMENTARY))) or self._sa_candidates().size > 0

    def _sa_candidates(self) -> np.ndarray:
        a = self.aux
        if len(a) < 3:
            return np.zeros(0, np.int64)
        hit = np.nonzero((a[:-2] == ord("S")) & (a[1:-1] == ord("A")) & (a[2:] == ord("Z")))[0]
        if not len(hit):
            return np.zeros(0, np.int64)
        rows = np.searchsorted(self.aux_off, hit, side="right") - 1
        return np.unique(rows[(rows >= 0)])

    def tag_value(self, i: int, tag: bytes):
        """The value of a Z/H/A or integer tag of record ``i`` (None without it)."""
        a = self.aux[self.aux_off[i]:self.aux_off[i] + self.aux_len[i]].tobytes()
        j = 0
        sizes = {ord(c): s for c, s in zip("AcCsSiIf", (1, 1, 1, 2, 2, 4, 4, 4))}
        while j + 3 <= len(a):
            t, ty = a[j:j + 2], a[j + 2]
            j += 3
            if ty in (ord("Z"), ord("H")):
                k = a.index(b"\x00", j)
                if t == tag:
                    return a[j:k].decode()
                j = k + 1
            elif ty in sizes:
                if t == tag:
                    return a[j:j + sizes[ty]]
                j += sizes[ty]
            elif ty == ord("B"):
                sub = a[j]
                cnt = int.from_bytes(a[j + 1:j + 5], "little")
                j += 5 + sizes[sub] * cnt
            else:
                raise ValueError(f"bad aux type in record {i}")
        return None

    def sa_count(self) -> np.ndarray:
        """Per record: entries of its SA tag (``len(tag.rstrip(';').split(';'))``, AM:103-106), -1
        without one (cached)."""
        c = getattr(self, "_sa", None)
        if c is None:
            c = np.full(self.n, -1, np.int32)
            if self.n and self._sa_candidates().size:
                aux = np.ascontiguousarray(self.aux)
                off = np.ascontiguousarray(self.aux_off, np.int64)
                ln = np.ascontiguousarray(self.aux_len, np.int32)
                native.host_lib().ganon_aux_sa_count(aux.ctypes.data_as(native._u8p), off.ctypes.data_as(native._i64p),
                                                     ln.ctypes.data_as(native._i32p), self.n,
                                                     c.ctypes.data_as(native._i32p))
            self._sa = c
        return c

    def cigar_of(self, i: int) -> np.ndarray:
        o = int(self.cig_off[i])
        return self.cigar[o:o + int(self.n_cigar[i])]


class BamReader:
    """One BAM file read a reference sequence at a time (``ganon_bam_reader``, include/
    ganon_host.h): the bounded-memory counterpart of ``ReadTable(path)``. ``contig(tid)`` returns a
    ReadTable of that sequence's records only (file order, full reference list); the reader seeks
    through ``<bam>.bai`` when present, else streams forward. ``inflater``: a native.GpuInflater
    that inflates the reader's BGZF block windows instead of its zlib threads."""

    def __init__(self, path: str, threads: int = 8, window: int = 0, inflater=None):
        lib = native.host_lib()
        h = C.c_void_p()
        rc = lib.ganon_bam_reader_open(os.fsencode(path), int(threads), C.byref(h))
        if rc != 0:
            raise native.GanonError(f"cannot open {path}: {lib.ganon_host_last_error().decode()}")
        self._h = h
        self.path = path
        if window:
            lib.ganon_bam_reader_set_window(h, int(window))
        self.inflater = None
        if inflater is not None:
            self.set_inflater(inflater)
        v = native.BamView()
        lib.ganon_bam_reader_header(h, C.byref(v))
        off = _arr(v.ref_name_off, v.n_ref, np.int64)
        raw = int(v.ref_names) if v.n_ref else 0
        self.ref_names: List[str] = [C.string_at(raw + int(o)).decode() for o in off]
        self.ref_lens = _arr(v.ref_len, v.n_ref, np.int64)
        self.has_index = bool(lib.ganon_bam_reader_has_index(h))

    def set_inflater(self, inflater) -> None:
        """Block windows inflate on the GPU from now on (a native.GpuInflater, kept alive here: the
        reader calls into its context)."""
        native.host_lib().ganon_bam_reader_set_inflater(self._h, inflater.fn, inflater.handle, inflater.min_blocks)
        self.inflater = inflater
        if isinstance(inflater, native.GpuInflater) and os.environ.get("GANON_PINNED_SCAN", "1") != "0":
            # the scans' inflated bytes in one page-locked buffer kept by the reader: the inflater's
            # device-to-host copies go by DMA instead of through the runtime's staging copies
            hl = native.hip_lib()
            native.host_lib().ganon_bam_reader_set_buffer_alloc(
                self._h, C.cast(hl.ganon_pinned_alloc, C.c_void_p), C.cast(hl.ganon_pinned_free, C.c_void_p))
            if os.environ.get("GANON_DEVICE_REGION", "1") != "0":
                # region reads: the first window inflated, walked and filtered on the device, the
                # kept records' columns back by DMA (no host record walk or column copies)
                native.host_lib().ganon_bam_reader_set_region_decoder(
                    self._h, inflater.region_fn, inflater.handle, inflater.min_blocks,
                    C.cast(hl.ganon_pinned_free, C.c_void_p))

    def tid_of(self, contig: str) -> int:
        try:
            return self.ref_names.index(contig)
        except ValueError:
            return -1

    def contig(self, tid: int) -> ReadTable:
        """The records of BAM sequence ``tid`` (an empty table for tid < 0)."""
        if tid < 0:
            return self.empty()
        lib = native.host_lib()
        h = C.c_void_p()
        rc = lib.ganon_bam_reader_contig(self._h, int(tid), C.byref(h))
        if rc != 0:
            raise native.GanonError(f"cannot decode {self.path} sequence {tid}: "
                                    f"{lib.ganon_host_last_error().decode()}")
        return ReadTable(self.path, handle=h)

    def region(self, tid: int, beg: int, end: int) -> ReadTable:
        """The records of BAM sequence ``tid`` overlapping [beg, end) (0-based, htslib's fetch
        semantics), through the index (``ganon_bam_reader_region``; an index is required)."""
        if tid < 0:
            return self.empty()
        lib = native.host_lib()
        h = C.c_void_p()
        rc = lib.ganon_bam_reader_region(self._h, int(tid), int(beg), int(end), C.byref(h))
        if rc != 0:
            raise native.GanonError(f"cannot decode {self.path} sequence {tid} [{beg}, {end}): "
                                    f"{lib.ganon_host_last_error().decode()}")
        return ReadTable(self.path, handle=h)

    def empty(self) -> ReadTable:
        """A table with no records and this file's reference list."""
        t = ReadTable.__new__(ReadTable)
        t.path, t.n = self.path, 0
        t.ref_names, t.ref_lens = list(self.ref_names), self.ref_lens.copy()
        for f in ("tid", "pos", "end", "flag", "mapq", "l_seq", "n_cigar", "mate_tid", "mate_pos", "tlen", "name_len",
                  "aux_len"):
            setattr(t, f, np.zeros(0, np.int32))
        for f in ("name_off", "cig_off", "seq_off", "qual_off", "aux_off"):
            setattr(t, f, np.zeros(0, np.int64))
        t.names_blob = np.zeros(0, np.uint8)
        t.cigar = np.zeros(0, np.uint32)
        t.seq = np.zeros(0, np.uint8)
        t.qual = np.zeros(0, np.uint8)
        t.aux = np.zeros(0, np.uint8)
        t._finish()
        return t

    def close(self) -> None:
        if self._h:
            native.host_lib().ganon_bam_reader_close(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
