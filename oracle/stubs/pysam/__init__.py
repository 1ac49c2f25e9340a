"""In-memory stand-in for the parts of pysam 0.22 / htslib that the reference touches.

TEST INFRASTRUCTURE ONLY (oracle/). Used by ``oracle/run_reference.py`` to execute the
unmodified reference Python in this container, where pysam is not installed.
Written from htslib's documented behaviour, not from pysam's source:

* ``AlignmentFile.fetch(contig, start, stop)``: records of that contig overlapping
  [start, stop) in file order; overlap uses htslib ``bam_endpos`` (pos + reference length,
  or pos + 1 for unmapped / zero-length records). ``start > stop`` or ``start < 0`` raise
  ``ValueError`` like pysam's region parser.
* ``AlignmentFile.pileup(...)`` with ``stepper='nofilter'``, ``truncate=False``: columns
  for every position covered by a *mapped* fetched record (htslib ``bam_plp_push`` skips
  BAM_FUNMAP), zero-depth positions skipped, reads in push (= file) order, and
  ``query_position = None`` on D/N positions.
* ``AlignedSegment``: the attributes the reference reads.
* ``FastaFile.fetch(name, start, end)``: plain slice of the stored sequence.

Parity with real htslib at this boundary is not pinned by the reference (it has no tests);
the build's own BAM reader and planner implement the same documented semantics.
"""
from __future__ import annotations

import array
import bisect
import gzip
import struct
from typing import Dict, List, Optional

NT16 = "=ACMGRSVTWYHKDBN"
CIGAR_OPS = "MIDNSHP=X"
_REF_CONSUMING = {0, 2, 3, 7, 8}
_QUERY_CONSUMING = {0, 1, 4, 7, 8}

_BAM_CACHE: Dict[str, tuple] = {}


class AlignedSegment:
    __slots__ = ("query_name", "flag", "reference_id", "reference_start", "mapping_quality",
                 "_cigar", "next_reference_id", "next_reference_start", "template_length",
                 "query_sequence", "_qual", "_tags", "_header", "_end", "_cigarstring")

    # -- flags ------------------------------------------------------------------------
    @property
    def is_paired(self): return bool(self.flag & 0x1)
    @property
    def is_unmapped(self): return bool(self.flag & 0x4)
    @property
    def is_mapped(self): return not (self.flag & 0x4)
    @property
    def is_reverse(self): return bool(self.flag & 0x10)
    @property
    def is_read1(self): return bool(self.flag & 0x40)
    @property
    def is_read2(self): return bool(self.flag & 0x80)
    @property
    def is_secondary(self): return bool(self.flag & 0x100)
    @property
    def is_supplementary(self): return bool(self.flag & 0x800)

    # -- coordinates ----------------------------------------------------------------
    @property
    def reference_name(self):
        return None if self.reference_id < 0 else self._header[self.reference_id][0]

    @property
    def reference_end(self):
        if (self.flag & 0x4) or not self._cigar:
            return None
        return self._end

    @property
    def cigarstring(self):
        if not self._cigar:
            return None
        cs = getattr(self, "_cigarstring", None)
        if cs is None:
            cs = self._cigarstring = "".join(f"{n}{CIGAR_OPS[op]}" for op, n in self._cigar)   # (never changes)
        return cs

    @property
    def cigartuples(self):
        return [(op, n) for op, n in self._cigar] if self._cigar else None

    # -- qualities --------------------------------------------------------------------
    @property
    def query_qualities(self):
        if self._qual is None:
            return None
        return array.array("B", self._qual)

    def get_forward_qualities(self):
        q = self.query_qualities
        if q is None:
            return None
        if self.is_reverse:
            q = q[::-1]
        return q

    # -- tags -------------------------------------------------------------------------
    def has_tag(self, tag):
        return tag in self._tags

    def get_tag(self, tag):
        return self._tags[tag]

    def to_string(self):
        return f"{self.query_name}\t{self.flag}\t{self.reference_name}\t{self.reference_start + 1}"


def _bam_endpos(pos: int, flag: int, cigar) -> int:
    rlen = 0
    if not (flag & 0x4):
        for op, n in cigar:
            if op in _REF_CONSUMING:
                rlen += n
    if rlen == 0:
        rlen = 1
    return pos + rlen


def _parse_tags(buf: bytes) -> Dict[str, object]:
    tags = {}
    i = 0
    sizes = {"A": 1, "c": 1, "C": 1, "s": 2, "S": 2, "i": 4, "I": 4, "f": 4}
    fmts = {"A": "c", "c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I", "f": "f"}
    while i + 3 <= len(buf):
        tag = buf[i:i + 2].decode(); typ = chr(buf[i + 2]); i += 3
        if typ in sizes:
            (v,) = struct.unpack_from("<" + fmts[typ], buf, i); i += sizes[typ]
            if typ == "A":
                v = v.decode()
        elif typ in "ZH":
            j = buf.index(b"\x00", i); v = buf[i:j].decode(); i = j + 1
        elif typ == "B":
            sub = chr(buf[i]); (cnt,) = struct.unpack_from("<i", buf, i + 1); i += 5
            v = list(struct.unpack_from("<" + fmts[sub] * cnt, buf, i)); i += sizes[sub] * cnt
        else:
            raise ValueError(f"bad tag type {typ}")
        tags[tag] = v
    return tags


def _load_bam(path: str):
    if path in _BAM_CACHE:
        return _BAM_CACHE[path]
    with gzip.open(path, "rb") as fh:
        data = fh.read()
    assert data[:4] == b"BAM\x01", "not a BAM file"
    (l_text,) = struct.unpack_from("<i", data, 4)
    off = 8 + l_text
    (n_ref,) = struct.unpack_from("<i", data, off); off += 4
    header = []
    for _ in range(n_ref):
        (l_name,) = struct.unpack_from("<i", data, off); off += 4
        name = data[off:off + l_name - 1].decode(); off += l_name
        (l_ref,) = struct.unpack_from("<i", data, off); off += 4
        header.append((name, l_ref))
    recs: List[AlignedSegment] = []
    while off < len(data):
        (bs,) = struct.unpack_from("<i", data, off)
        (tid, pos, l_rn, mapq, _bin, n_cig, flag, l_seq, ntid, npos, tlen) = struct.unpack_from(
            "<iiBBHHHiiii", data, off + 4)
        p = off + 36
        name = data[p:p + l_rn - 1].decode(); p += l_rn
        cig = []
        for k in range(n_cig):
            (c,) = struct.unpack_from("<I", data, p + 4 * k)
            cig.append((c & 0xF, c >> 4))
        p += 4 * n_cig
        sb = data[p:p + (l_seq + 1) // 2]; p += (l_seq + 1) // 2
        seq = "".join(NT16[(sb[i >> 1] >> (4 if (i & 1) == 0 else 0)) & 0xF] for i in range(l_seq))
        qual = data[p:p + l_seq]; p += l_seq
        tags = _parse_tags(data[p:off + 4 + bs])
        a = AlignedSegment()
        a.query_name = name; a.flag = flag; a.reference_id = tid; a.reference_start = pos
        a.mapping_quality = mapq; a._cigar = cig; a.next_reference_id = ntid
        a.next_reference_start = npos; a.template_length = tlen
        a.query_sequence = seq if l_seq else None
        a._qual = None if (l_seq == 0 or qual[0] == 0xFF) else bytes(qual)
        a._tags = tags; a._header = header
        a._end = _bam_endpos(pos, flag, cig)
        recs.append(a)
        off += 4 + bs
    _BAM_CACHE[path] = (header, recs)
    return _BAM_CACHE[path]


class PileupRead:
    __slots__ = ("alignment", "query_position")

    def __init__(self, aln, qpos):
        self.alignment = aln
        self.query_position = qpos


class _PileupCursor:
    """State shared by the columns of one pileup iterator. pysam's PileupColumn reads its reads
    from the pileup engine's live buffer, which the next step of the iterator overwrites: a column
    kept past that step shows other reads (or raises once the iterator finished). The stub makes
    that misuse loud: ``pileups`` of a column the iterator has moved past raises."""
    __slots__ = ("gen",)

    def __init__(self):
        self.gen = 0


class PileupColumn:
    __slots__ = ("reference_id", "reference_name", "reference_pos", "_pileups", "_cursor", "_gen")

    def __init__(self, tid, name, pos, pileups, cursor=None):
        self.reference_id = tid
        self.reference_name = name
        self.reference_pos = pos
        self._pileups = pileups
        self._cursor = cursor
        self._gen = cursor.gen if cursor is not None else 0

    @property
    def pileups(self):
        if self._cursor is not None and self._cursor.gen != self._gen:
            raise ValueError("PileupColumn accessed after its iterator moved on (pysam: live pileup buffer)")
        return self._pileups

    @property
    def nsegments(self):
        return len(self.pileups)


def _qpos_at(aln: AlignedSegment, refpos: int) -> Optional[int]:
    """Query position aligned to ``refpos`` (None on D/N), as htslib resolve_cigar2 does."""
    rp = aln.reference_start
    qp = 0
    for op, n in aln._cigar:
        if op in (0, 7, 8):
            if rp <= refpos < rp + n:
                return qp + (refpos - rp)
            rp += n; qp += n
        elif op in (1, 4):
            qp += n
        elif op in (2, 3):
            if rp <= refpos < rp + n:
                return None
            rp += n
    return None


class AlignmentFile:
    def __init__(self, path, mode="rb", reference_filename=None, threads=1, header=None, **kw):
        if "w" in str(mode):
            raise NotImplementedError("stub pysam cannot write alignment files")
        self.filename = path
        self._header, self._recs = _load_bam(path)
        self._by_tid: Dict[int, List[AlignedSegment]] = {}
        for r in self._recs:
            self._by_tid.setdefault(r.reference_id, []).append(r)
        self._starts = {t: [r.reference_start for r in rs] for t, rs in self._by_tid.items()}
        self._maxspan = {t: max(r._end - r.reference_start for r in rs) for t, rs in self._by_tid.items()}

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def close(self):
        pass

    @property
    def references(self):
        return tuple(n for n, _ in self._header)

    @property
    def lengths(self):
        return tuple(l for _, l in self._header)

    def _tid(self, name):
        for i, (n, _) in enumerate(self._header):
            if n == name:
                return i
        raise ValueError(f"invalid contig `{name}`")

    def _region(self, contig, start, stop):
        tid = self._tid(contig)
        length = self._header[tid][1]
        rstart = 0 if start is None else start
        rstop = length if stop is None else stop
        if rstart > rstop:
            raise ValueError(f"invalid coordinates: start ({rstart}) > stop ({rstop})")
        if rstart < 0:
            raise ValueError(f"start out of range ({rstart})")
        if rstop < 0:
            raise ValueError(f"stop out of range ({rstop})")
        return tid, rstart, rstop

    def fetch(self, reference=None, start=None, stop=None, until_eof=False, contig=None, end=None, **kw):
        contig = contig if contig is not None else reference
        stop = stop if stop is not None else end
        if contig is None:
            if until_eof:
                return iter(list(self._recs))
            raise ValueError("fetch called on bamfile without index")  # whole-file fetch
        tid, rstart, rstop = self._region(contig, start, stop)
        rs = self._by_tid.get(tid, [])
        if not rs:
            return iter(())
        st = self._starts[tid]
        lo = bisect.bisect_left(st, rstart - self._maxspan[tid])
        hi = bisect.bisect_left(st, rstop)
        out = [r for r in rs[lo:hi] if r._end > rstart]
        return iter(out)

    def pileup(self, reference=None, start=None, end=None, contig=None, stop=None, truncate=False,
               stepper="all", **kw):
        contig = contig if contig is not None else reference
        end = end if end is not None else stop
        if stepper != "nofilter" or truncate:
            raise NotImplementedError("stub pileup models stepper='nofilter', truncate=False only")
        reads = [r for r in self.fetch(contig, start, end) if not (r.flag & 0x4)]
        tid = self._tid(contig)
        return _pileup_columns(reads, tid, contig)


class _QposWalker:
    """_qpos_at for increasing reference positions of one read, walking its CIGAR once."""
    __slots__ = ("cig", "k", "rp", "qp")

    def __init__(self, aln):
        self.cig = aln._cigar
        self.k = 0
        self.rp = aln.reference_start
        self.qp = 0

    def at(self, refpos: int):
        while self.k < len(self.cig):
            op, n = self.cig[self.k]
            if op in (0, 7, 8):
                if refpos < self.rp + n:
                    return self.qp + (refpos - self.rp) if refpos >= self.rp else None
                self.rp += n
                self.qp += n
            elif op in (1, 4):
                self.qp += n
            elif op in (2, 3):
                if refpos < self.rp + n:
                    return None
                self.rp += n
            self.k += 1
        return None


def _pileup_columns(reads, tid, name):
    # reads are in file (= push) order; a read contributes to [start, end) columns
    i = 0
    active: List[AlignedSegment] = []
    walkers: Dict[int, _QposWalker] = {}
    n = len(reads)
    pos = reads[0].reference_start if reads else 0
    cur = _PileupCursor()
    try:
        while i < n or active:
            while i < n and reads[i].reference_start <= pos:
                active.append(reads[i]); walkers[id(reads[i])] = _QposWalker(reads[i]); i += 1
            active = [r for r in active if r._end > pos]
            if active:
                yield PileupColumn(tid, name, pos, [PileupRead(r, walkers[id(r)].at(pos)) for r in active], cur)
                cur.gen += 1     # the engine's buffer moves on
                pos += 1
            elif i < n:
                pos = reads[i].reference_start
            else:
                break
    finally:
        cur.gen += 1


class FastaFile:
    def __init__(self, path):
        self.filename = path
        names, seqs = [], []
        cur = None
        with open(path) as fh:
            for line in fh:
                line = line.rstrip("\n")
                if line.startswith(">"):
                    names.append(line[1:].split()[0]); seqs.append([])
                elif line:
                    seqs[-1].append(line)
        self._seqs = {n: "".join(s) for n, s in zip(names, seqs)}
        self.references = tuple(names)
        self.lengths = tuple(len(self._seqs[n]) for n in names)

    def fetch(self, reference=None, start=None, end=None, region=None):
        s = self._seqs[reference]
        start = 0 if start is None else start
        end = len(s) if end is None else end
        if start < 0:
            raise ValueError("start out of range")
        return s[start:end]

    def get_reference_length(self, ref):
        return len(self._seqs[ref])

    def close(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def get_include():  # pragma: no cover - build-time only in the real package
    return []


def get_defines():  # pragma: no cover
    return []
