"""Minimal BGZF/BAM, FASTA(+.fai) and VCF writers for the synthetic inputs.

Test and benchmark infrastructure only: the product never writes BAM (the reference
emits FASTQ only). Written from the SAM/BAM v1 specification
(BGZF blocks with the ``BC`` extra subfield, ``reg2bin`` binning, nt16 packed bases).
"""
from __future__ import annotations

import struct
import zlib
from typing import Iterable, List, Optional, Sequence, Tuple

NT16 = "=ACMGRSVTWYHKDBN"
_NT16_CODE = {c: i for i, c in enumerate(NT16)}
CIGAR_OPS = "MIDNSHP=X"
_CIGAR_CODE = {c: i for i, c in enumerate(CIGAR_OPS)}

_BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
_BGZF_MAX_INPUT = 0xFF00  # keep every block's payload below 64 KiB


def reg2bin(beg: int, end: int) -> int:
    """BAM bin of the 0-based half-open interval [beg, end) (SAM spec §5.3)."""
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


def _bgzf_block(payload: bytes, level: int) -> bytes:
    comp = zlib.compressobj(level, zlib.DEFLATED, -15)
    data = comp.compress(payload) + comp.flush()
    bsize = len(data) + 25  # header 18 + footer 8 - 1
    header = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize)
    footer = struct.pack("<II", zlib.crc32(payload) & 0xFFFFFFFF, len(payload))
    return header + data + footer


class BgzfWriter:
    def __init__(self, path: str, level: int = 6):
        self._fh = open(path, "wb")
        self._buf = bytearray()
        self._level = level

    def write(self, data: bytes) -> None:
        self._buf += data
        while len(self._buf) >= _BGZF_MAX_INPUT:
            self._fh.write(_bgzf_block(bytes(self._buf[:_BGZF_MAX_INPUT]), self._level))
            del self._buf[:_BGZF_MAX_INPUT]

    def tell_virtual(self) -> int:
        """BGZF virtual offset of the next byte written (compressed block offset << 16 | offset
        in the block's uncompressed payload)."""
        return (self._fh.tell() << 16) | len(self._buf)

    def close(self) -> None:
        if self._buf:
            self._fh.write(_bgzf_block(bytes(self._buf), self._level))
            self._buf.clear()
        self._fh.write(_BGZF_EOF)
        self._fh.close()


def cigar_ref_len(cigar: Sequence[Tuple[str, int]]) -> int:
    return sum(n for op, n in cigar if op in "MDN=X")


def cigar_query_len(cigar: Sequence[Tuple[str, int]]) -> int:
    return sum(n for op, n in cigar if op in "MIS=X")


class BamRecord:
    """One alignment record. ``cigar`` is a list of (op, length); ``seq`` a str over NT16."""

    __slots__ = ("name", "flag", "tid", "pos", "mapq", "cigar", "mate_tid", "mate_pos",
                 "tlen", "seq", "qual", "tags")

    def __init__(self, name: str, flag: int, tid: int, pos: int, mapq: int,
                 cigar: List[Tuple[str, int]], mate_tid: int, mate_pos: int, tlen: int,
                 seq: str, qual: Sequence[int], tags: Optional[List[Tuple[str, str, str]]] = None):
        self.name, self.flag, self.tid, self.pos, self.mapq = name, flag, tid, pos, mapq
        self.cigar, self.mate_tid, self.mate_pos, self.tlen = cigar, mate_tid, mate_pos, tlen
        self.seq, self.qual, self.tags = seq, qual, tags or []

    def end(self) -> int:
        rlen = 0 if (self.flag & 4) else cigar_ref_len(self.cigar)
        return self.pos + (rlen if rlen > 0 else 1)

    def encode(self) -> bytes:
        name = self.name.encode() + b"\x00"
        l_seq = len(self.seq)
        codes = [_NT16_CODE[c] for c in self.seq]
        if l_seq & 1:
            codes.append(0)
        packed = bytes((codes[i] << 4) | codes[i + 1] for i in range(0, len(codes), 2))
        cig = b"".join(struct.pack("<I", (n << 4) | _CIGAR_CODE[op]) for op, n in self.cigar)
        qual = bytes(self.qual) if len(self.qual) else b"\xff" * l_seq
        tags = b""
        for tag, typ, val in self.tags:
            if typ != "Z":
                raise ValueError("only Z tags are written")
            tags += tag.encode() + b"Z" + val.encode() + b"\x00"
        bin_ = reg2bin(self.pos, self.end()) if self.pos >= 0 else 4680
        body = struct.pack("<iiBBHHHiiii", self.tid, self.pos, len(name), self.mapq, bin_,
                           len(self.cigar), self.flag, l_seq, self.mate_tid, self.mate_pos,
                           self.tlen)
        body += name + cig + packed + qual + tags
        return struct.pack("<i", len(body)) + body


def write_bam(path: str, contigs: Sequence[Tuple[str, int]], records: Iterable[BamRecord],
              level: int = 6, index: bool = False) -> None:
    """Coordinate-sorted BAM; ``index`` also writes ``path + '.bai'`` (bins with their chunks, the
    16 kb linear index and the pseudo-bin 37450 of each reference, SAM spec §5.2)."""
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join(
        f"@SQ\tSN:{n}\tLN:{l}\n" for n, l in contigs)
    w = BgzfWriter(path, level)
    hdr = b"BAM\x01" + struct.pack("<i", len(text)) + text.encode() + struct.pack("<i", len(contigs))
    for n, l in contigs:
        nb = n.encode() + b"\x00"
        hdr += struct.pack("<i", len(nb)) + nb + struct.pack("<i", l)
    w.write(hdr)
    spans = []   # (tid, pos, end, voff_beg, voff_end, unmapped)
    for rec in records:
        b = rec.encode()
        v0 = w.tell_virtual()
        w.write(b)
        if index:
            spans.append((rec.tid, rec.pos, rec.end(), v0, w.tell_virtual(), bool(rec.flag & 4)))
    w.close()
    if index:
        _write_bai(path + ".bai", len(contigs), spans)


def _write_bai(path: str, n_ref: int, spans) -> None:
    per = [[] for _ in range(n_ref)]
    n_no_coor = 0
    for s in spans:
        if s[0] < 0:
            n_no_coor += 1
        else:
            per[s[0]].append(s)
    out = b"BAI\x01" + struct.pack("<i", n_ref)
    for recs in per:
        bins = {}
        lin = {}
        for tid, pos, end, v0, v1, unm in recs:
            ch = bins.setdefault(reg2bin(pos, end), [])
            if ch and ch[-1][1] == v0:
                ch[-1][1] = v1
            else:
                ch.append([v0, v1])
            for k in range(pos >> 14, ((end - 1) >> 14) + 1):
                lin.setdefault(k, v0)
        nb = len(bins) + (1 if recs else 0)
        out += struct.pack("<i", nb)
        for b in sorted(bins):
            out += struct.pack("<Ii", b, len(bins[b]))
            for v0, v1 in bins[b]:
                out += struct.pack("<QQ", v0, v1)
        if recs:
            n_unm = sum(1 for r in recs if r[5])
            out += struct.pack("<Ii", 37450, 2) + struct.pack("<QQ", recs[0][3], recs[-1][4]) + \
                struct.pack("<QQ", len(recs) - n_unm, n_unm)
        n_intv = (max(lin) + 1) if lin else 0
        out += struct.pack("<i", n_intv)
        last = 0
        for k in range(n_intv):
            last = lin.get(k, last)
            out += struct.pack("<Q", last)
    out += struct.pack("<Q", n_no_coor)
    with open(path, "wb") as fh:
        fh.write(out)


def write_fasta(path: str, contigs: Sequence[Tuple[str, str]], width: int = 60) -> None:
    """Write FASTA and a samtools-style ``.fai`` (name, length, offset, linebases, linewidth)."""
    fai = []
    with open(path, "wb") as fh:
        off = 0
        for name, seq in contigs:
            head = f">{name}\n".encode()
            fh.write(head)
            off += len(head)
            fai.append(f"{name}\t{len(seq)}\t{off}\t{width}\t{width + 1}\n")
            body = "".join(seq[i:i + width] + "\n" for i in range(0, len(seq), width)).encode()
            fh.write(body)
            off += len(body)
    with open(path + ".fai", "w") as fh:
        fh.write("".join(fai))


def write_vcf(path: str, contigs: Sequence[Tuple[str, int]],
              records: Iterable[Tuple[str, int, str, str, str]]) -> None:
    """records: (contig, 1-based pos, id, ref, alt)."""
    with open(path, "w") as fh:
        fh.write("##fileformat=VCFv4.2\n")
        for n, l in contigs:
            fh.write(f"##contig=<ID={n},length={l}>\n")
        fh.write("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n")
        for c, p, i, r, a in records:
            fh.write(f"{c}\t{p}\t{i}\t{r}\t{a}\t.\tPASS\t.\n")


def first_record_offset(d: bytes) -> int:
    """Offset of the first record of an inflated BAM stream (after magic, header text and the
    reference list, SAM spec §4.2)."""
    if d[:4] != b"BAM\x01":
        raise ValueError("not an inflated BAM stream")
    p = 8 + int.from_bytes(d[4:8], "little")
    n_ref = int.from_bytes(d[p:p + 4], "little")
    p += 4
    for _ in range(n_ref):
        p += 4 + int.from_bytes(d[p:p + 4], "little") + 4
    return p


def write_bgzf(path: str, data: bytes, level: int = 6) -> None:
    """``data`` as a BGZF file (level 0: stored blocks)."""
    w = BgzfWriter(path, level)
    w.write(data)
    w.close()

