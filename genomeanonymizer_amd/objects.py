"""Complex read names: the content of the reference's ``AnonymizedRead`` objects.

A name is *complex* when one of its records has an SA tag or is a secondary / supplementary
alignment. Its reads are then the reference's full object model (anonymizer_methods.py:84-287,
:320-389; short_read_tumor_normal_anonymizer.py:304-406, :603-622):

* an object is created by the first alignment of a read met in a scope (its *creator*: dataset,
  mate, orientation, SA count) and holds the sequence and forward qualities of its first
  non-supplementary alignment (``update_from_primary_mapping``, AM:142-149); the output keeps the
  creator's orientation (``is_reverse`` is never updated);
* a germline SNV found through any alignment of the read is written at that alignment's query
  position into the object's sequence (AM:548-554) — directly while the object holds a primary
  mapping, as a left-over while it is still supplementary; germline indels of the read's first
  alignment in the scope are left-overs too (AM:551-552, variation_classifier.py:196-207);
* ``mask_or_anonymize_left_over_variants`` (AM:254-270) applies the whole left-over list, stable by
  variant type; ``update_anonymized_read_from_other`` (AM:281-287) appends another object's list if
  that one is flagged and re-sets the flag when the list is non-empty.

Which objects meet, merge and get written is decided by the native planner and resolver
(csrc/ganon_plan.cpp, include/ganon_host.h ``objs`` and the resolver log); this module replays the
log over the masked sequences the device produced for each alignment (one device copy per
(alignment, scope), ``anonymizer_methods.build_batch``) and formats the written objects.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from .indels import apply_indel
from .variants import VariantType

NT16 = np.frombuffer(b"=ACMGRSVTWYHKDBN", np.uint8)
_REVERSES = {ord("A"): ord("T"), ord("C"): ord("G"), ord("G"): ord("C"), ord("T"): ord("A"), ord("N"): ord("N")}
_REF = (1 << 0) | (1 << 2) | (1 << 3) | (1 << 7) | (1 << 8)     # M D N = X
_QRY = (1 << 0) | (1 << 1) | (1 << 4) | (1 << 7) | (1 << 8)     # M I S = X
_TYPE_ORDER = {"S": VariantType.SNV.value, VariantType.DEL: VariantType.DEL.value,
               VariantType.INS: VariantType.INS.value}
_COMP = bytes.maketrans(b"ACGTN", b"TGCAN")
_PHRED = bytes((b + 33) & 0xFF for b in range(256))

Key = Tuple[int, int, int]            # (job, dataset, row)


class Record:
    """What the object model reads from one BAM record (pysam AlignedSegment fields)."""
    __slots__ = ("name", "flag", "pos", "cigar", "seq", "qual")

    def __init__(self, name: bytes, flag: int, pos: int, cigar: np.ndarray, seq: bytes, qual: Optional[bytes]):
        self.name, self.flag, self.pos, self.cigar, self.seq, self.qual = name, flag, pos, cigar, seq, qual

    @property
    def reverse(self) -> bool:
        return bool(self.flag & 0x10)

    def forward_qual(self) -> Optional[bytes]:
        """get_forward_qualities (bytes; a list once an indel edits it)."""
        if self.qual is None:
            return None
        return self.qual[::-1] if self.reverse else self.qual

    def columns(self, idx: np.ndarray) -> np.ndarray:
        """Reference column of each aligned query position (a CIGAR walk)."""
        out = np.full(len(idx), -1, np.int64)
        rp, qp = self.pos, 0
        for c in self.cigar.tolist():
            op, n = c & 0xF, c >> 4
            if (_REF >> op) & 1 and (_QRY >> op) & 1:
                m = (idx >= qp) & (idx < qp + n)
                out[m] = rp + (idx[m] - qp)
            if (_REF >> op) & 1:
                rp += n
            if (_QRY >> op) & 1:
                qp += n
        return out


def decode_nt16(buf: np.ndarray, nib0: int, n: int) -> bytes:
    i = nib0 + np.arange(n, dtype=np.int64)
    b = buf[i >> 1]
    return NT16[np.where(i & 1, b & 0xF, b >> 4)].tobytes()


def record_of(table, row: int) -> Record:
    return records_of(table, [row])[row]


def records_of(table, rows) -> Dict[int, Record]:
    """Records of many rows of a ReadTable, the sequences decoded in one pass."""
    rows = np.asarray(sorted(set(int(r) for r in rows)), np.int64)
    if not len(rows):
        return {}
    L = table.l_seq[rows].astype(np.int64)
    start = np.concatenate([[0], np.cumsum(L)[:-1]])
    nib = np.repeat(2 * table.seq_off[rows].astype(np.int64) - start, L) + np.arange(int(L.sum()), dtype=np.int64)
    b = table.seq[nib >> 1]
    blob = NT16[np.where(nib & 1, b & 0xF, b >> 4)].tobytes()
    qb = table.qual.tobytes()
    nb = table.names_blob.tobytes()
    cig = table.cigar
    out = {}
    for r, l, s0 in zip(rows.tolist(), L.tolist(), start.tolist()):
        qo = int(table.qual_off[r])
        qual = None if (l == 0 or qb[qo] == 0xFF) else qb[qo:qo + l]
        no, co = int(table.name_off[r]), int(table.cig_off[r])
        out[r] = Record(nb[no:no + int(table.name_len[r])], int(table.flag[r]), int(table.pos[r]),
                        cig[co:co + int(table.n_cigar[r])].copy(), blob[s0:s0 + l], qual)
    return out


def mask_diffs(rec: Record, masked: bytes) -> List[Tuple[int, int, int, int]]:
    """(column, query position, new base, read base) of every base the device changed."""
    a = np.frombuffer(rec.seq, np.uint8)
    b = np.frombuffer(masked, np.uint8)
    idx = np.nonzero(a != b)[0]
    if not len(idx):
        return []
    cols = rec.columns(idx)
    return list(zip(cols.tolist(), idx.tolist(), b[idx].tolist(), a[idx].tolist()))


class State:
    """One AnonymizedRead's mutable content."""
    __slots__ = ("seq", "qual", "left", "flag", "reverse", "name", "mate")

    def __init__(self, seq: bytearray, qual, reverse: bool, name: bytes, mate: int):
        self.seq, self.qual, self.reverse, self.name, self.mate = seq, qual, reverse, name, mate
        self.left: list = []
        self.flag = False

    def put(self, pos: int, base: int) -> None:
        """np.put(..., mode='raise') of mask_or_modify_base_pair (AM:170-176)."""
        n = len(self.seq)
        if not -n <= pos < n:
            raise IndexError(f"index {pos} is out of bounds for axis 0 with size {n}")
        self.seq[pos] = base

    def apply(self) -> None:
        """mask_or_anonymize_left_over_variants when flagged (AM:254-270)."""
        if not self.flag:
            return
        self.flag = False
        if self.seq is None:          # content never written (Replay._plain_object)
            return
        for kind, pos, x in sorted(self.left, key=lambda e: _TYPE_ORDER[e[0]]):
            if kind == "S":
                self.put(pos, x)
            else:
                self.seq, q = apply_indel(self.seq, list(self.qual), pos, x)
                self.qual = bytes(q)

    def absorb(self, other: "State") -> None:
        """update_anonymized_read_from_other (AM:281-287)."""
        if other.flag:
            self.left.extend(other.left)
        if self.left:
            self.flag = True

    def fastq(self) -> bytes:
        """get_anonymized_fastq_record (AM:215-243) with the creator's orientation."""
        if self.seq is None:
            # every masked copy a resolution can name is carried (stream.JobPrep._mask_instances)
            raise RuntimeError("internal: an object made from a masked copy that was not carried")
        seq = bytes(self.seq)
        if self.qual is None:
            raise TypeError(f"read {self.name.decode()!r} has no qualities")
        qual = bytes(self.qual)
        if self.reverse:
            if seq.translate(None, b"ACGTN"):
                raise TypeError(f"reverse read {self.name.decode()!r} has a base outside ACGTN (SURVEY Q7)")
            seq = seq[::-1].translate(_COMP)
            qual = qual[::-1]
        return (b"@" + self.name + b"/" + str(self.mate).encode() + b"\n" + seq + b"\n+\n" +
                qual.translate(_PHRED) + b"\n")


def decode_fastq(rec: bytes, reverse: bool) -> Tuple[bytes, bytes, int, bytes, List[int]]:
    """(name, sequence in BAM orientation, mate, BAM-order qualities) of a formatted plain record
    (writer.FastqFormatter: reverse reads complemented back; qualities in stored order, Q1)."""
    head, seq, _, qual = rec.rstrip(b"\n").split(b"\n")
    name, mate = head[1:].rsplit(b"/", 1)
    if reverse:
        seq = seq[::-1].translate(_COMP)
    return name, seq, int(mate), bytes((c - 33) & 0xFF for c in qual)


class Replay:
    """The objects of complex names across the contigs of a sample (stream.py): per job, the plan's
    object summaries and its records' ingredients; the resolver log turns them into FASTQ records
    (``written[serial]``)."""

    def __init__(self, carry: dict, carry_info: dict):
        self.carry = carry                 # stream.py's carried plain records (job, ds, scope, row, k)
        self.carry_info = carry_info       # (job, ds, row) -> flag; (job, ds, scope, row) -> left-over edits
        self.jobs: Dict[int, dict] = {}
        self.states: Dict[int, State] = {}
        self.written: Dict[int, bytes] = {}

    def add_job(self, job: int, cx: Optional[dict]) -> None:
        if cx is not None and len(cx["objs"]):
            cx = dict(cx, objs_l=cx["objs"].tolist(), rows_l=cx["obj_rows"].tolist())
            self.jobs[job] = cx

    # -- object creation ------------------------------------------------------------------------
    def _record(self, job: int, ds: int, row: int) -> Record:
        r = self.jobs[job]["rec"].get((ds, row)) if job in self.jobs else None
        if r is not None:
            return r
        flag = self.carry_info[(job, ds, row)]
        name, seq, _, qual = decode_fastq(self.carry[(job, ds, -1, row, 0)], bool(flag & 0x10))
        return Record(name, flag, -1, np.zeros(0, np.uint32), seq, qual)

    def _plan_object(self, gid: int) -> State:
        job, k = gid >> 32, gid & 0xFFFFFFFF
        cx = self.jobs[job]
        scope, ds, _, c, base, a_off, a_n = cx["objs_l"][k][:7]
        aligns = cx["rows_l"][a_off:a_off + a_n]
        crec = cx["rec"][(ds, c)]
        brec = cx["rec"][(ds, base)] if base >= 0 else crec
        q = brec.forward_qual()
        st = State(bytearray(brec.seq), q, crec.reverse, crec.name, 1 if crec.flag & 0x40 else 2)
        if scope < 0:
            return st
        lo = brec.pos if base >= 0 else None
        # supporting_reads is a dict per variant: at one column, the read's last alignment with that
        # allele (pileup = file order) holds the position (variants.py:64-65)
        best: Dict[Tuple[int, int], Tuple[int, int, int]] = {}
        for a in aligns:
            for col, idx, new, alt in cx["masks"].get((ds, a, scope), ()):
                key = (col, alt)
                if key not in best or a > best[key][0]:
                    best[key] = (a, idx, new)
        masks = sorted((col, a, idx, new) for (col, _), (a, idx, new) in best.items())
        for col, a, idx, new in masks:
            if lo is not None and col >= lo:
                st.put(idx, new)
            else:
                st.left.append(("S", idx, new))
        for irp, call in cx["indels"].get((ds, c, scope), ()):
            st.left.append((call.variant_type, irp, call))
        st.flag = bool(st.left)
        if base >= 0:
            st.apply()          # mask_left_over_variants_in_pair before the scope yields it (AM:495, 523)
        return st

    def _plain_object(self, job: int, ds: int, scope: int, row: int, upd: int) -> State:
        edits = self.carry_info.get((job, ds, scope, row), [])
        rec = self.carry.get((job, ds, scope, row, 2 if edits else 0))
        if rec is None:
            # not carried: only a copy no write can name (fastq() refuses it)
            st = State(None, None, False, b"", 0)
        else:
            flag = self.carry_info[(job, ds, row)]
            rev = bool(flag & 0x10)
            name, seq, mate, qual = decode_fastq(rec, rev)
            st = State(bytearray(seq), qual[::-1] if rev else qual, rev, name, mate)
        st.left = [(call.variant_type, irp, call) for irp, call in edits]
        st.flag = bool(st.left)
        if scope >= 0:
            st.apply()
        if upd:
            st.flag = bool(st.left)
        return st

    def state(self, gid: int) -> State:
        st = self.states.get(gid)
        if st is None:
            st = self._plan_object(gid)
            self.states[gid] = st
        return st

    # -- the resolver log -----------------------------------------------------------------------
    def run(self, log: np.ndarray) -> None:
        for op, gid, a, b, c, d, e, _ in log.tolist():
            if op == 1:
                self.states[gid] = self._plain_object(a, b, c, d, e)
            elif op == 2:
                self.state(gid).absorb(self.state(a))
            elif op == 3:
                self.state(gid).apply()
            elif op == 4:
                st = self.state(gid)
                rec = self._record(a, b, c)
                st.seq = bytearray(rec.seq)
                st.qual = rec.forward_qual()
            elif op == 5:
                self.written[a] = self.state(gid).fastq()
            else:
                raise RuntimeError(f"bad object log entry {op}")

    def settle(self, pending: np.ndarray) -> None:
        """After a round of jobs: create their objects still pending (the jobs' ingredients are
        dropped now) and forget the states no pending entry refers to."""
        live = set(pending[pending[:, 2] == -2, 3].tolist()) if len(pending) else set()
        for gid in live:
            if gid < (1 << 62) and (gid >> 32) in self.jobs:
                self.state(gid)
        for gid in [g for g in self.states if g not in live]:
            del self.states[gid]
        self.jobs.clear()
        self.written.clear()     # serials of other ranks' jobs (this rank's were taken)

    def take(self, serial: int) -> bytes:
        return self.written.pop(serial)


class NativeReplay:
    """The same replay in libganon_host.so (``native.ObjectStore``, csrc/ganon_objects.cpp): the
    product's; the job ingredients travel as the packed blob of ``native.objects_pack``."""

    native = True

    def __init__(self, carry: dict, carry_info: dict):
        from . import native
        self.carry, self.carry_info = carry, carry_info
        self.store = native.ObjectStore()
        self.written: Dict[int, bytes] = {}

    def add_job(self, job: int, cx: Optional[bytes]) -> None:
        if cx:
            self.store.add_job(job, cx)

    def run(self, log: np.ndarray) -> None:
        if not len(log):
            return
        # plain instances the log turns into objects (1) or promotes from (4): their carried records
        for op, _, a, b, c, d, _, _ in log[(log[:, 0] == 1) | (log[:, 0] == 4)].tolist():
            if op == 1:
                edits = self.carry_info.get((a, b, c, d), [])
                rec = self.carry.get((a, b, c, d, 2 if edits else 0))
                if rec is not None:
                    self.store.add_plain(a, b, c, d, self.carry_info[(a, b, d)], rec, edits)
            else:
                rec = self.carry.get((a, b, -1, c, 0))
                if rec is not None:
                    self.store.add_plain(a, b, -1, c, self.carry_info[(a, b, c)], rec, [])
        self.store.run(log)
        self.written.update(self.store.take_all())

    def settle(self, pending: np.ndarray) -> None:
        live = pending[pending[:, 2] == -2, 3] if len(pending) else np.zeros(0, np.int64)
        self.store.settle(live)
        self.written.clear()

    def take(self, serial: int) -> bytes:
        return self.written.pop(serial)
