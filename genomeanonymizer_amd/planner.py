"""Host scope scheduler: which reads meet in which scope, and which scope's masked copy of
each read is written where, in the reference's exact output order.

Restates (without masking anything) the control flow of
``anonymize_genome`` (short_read_tumor_normal_anonymizer.py:625-760) for one tumor/normal
pair:

* windows and sections: ``get_windows`` (SR:71-131), ``get_genome_sections`` (SR:245-276);
* variant windows: ``anonymize_window`` (SR:279-372) over a pileup of [first, last)
  (pileup_io.pyx:8-41, htslib ``nofilter`` stepper, ``truncate=False``);
* inter-window gaps: ``anonymize_inter_window_region`` (SR:498-558) driven by
  ``iter_fetch_pair`` (pileup_io.pyx:124-298) with its cluster rules;
* the yield order of ``CompleteGermlineAnonymizer.anonymize`` (anonymizer_methods.py:
  472-532) computed from coordinates: a complete pair is yielded at the first
  normal column beyond its rightmost end, pairs at one column in first-appearance order,
  leftovers at scope end in first-appearance order;
* pairing and de-duplication: ``write_pair``/``written_read_ids`` (SR:134-165),
  ``to_pair_anonymized_reads`` with first-object-wins (AM:320-389),
  ``pair_unmapped_or_non_pileup_pairs_and_write`` (SR:375-406), ``pair_unmapped_mates``
  (SR:561-600) and ``write_single_end_reads`` (SR:603-622);
* statistics bookkeeping (SR:175-242): the window rows and which scope counts into which.

The masking itself (the hot path) happens later, in one device batch over all scopes
(genomeanonymizer_amd/anonymizer_methods.py -> include/ganon.h). An output record is an
``Instance`` = (dataset, read row, scope): the read as masked by that scope's tally, or
unmasked when scope == -1 (reads written from a fetch pass-through).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from .io.bam import FLAG_SECONDARY, FLAG_SUPPLEMENTARY, ReadTable
from .io.fasta import FastaRef
from .variants import VariantRecord, VariantType, WindowVariant

DATASET_TUMORAL = 0
DATASET_NORMAL = 1
WINDOW_SIZE = 2000
LONG_SV = 100_000

Instance = Tuple[int, int, int]  # (dataset, row, scope id or -1)


class UnsupportedInput(NotImplementedError):
    """Input the reference handles through code paths this build does not restate yet."""


@dataclasses.dataclass
class Window:
    """SR:35-52."""
    sequence: str
    first: int
    last: int
    variant: Optional[WindowVariant] = None

    def is_variant_window(self) -> bool:
        return self.variant is not None

    def __str__(self) -> str:
        if self.variant is None:
            return ",".join(map(str, (self.sequence, self.first, self.last)))
        return ",".join(map(str, (self.sequence, self.first, self.last, self.variant)))


def get_windows(records: Sequence[VariantRecord], ref_index: Dict[str, int],
                window_size: int = WINDOW_SIZE) -> List[Window]:
    """One window (two for INV/TRA/long SVs) of +-window_size/2 around each record (SR:71-131)."""
    half = int(window_size / 2)
    windows: List[Window] = []
    for r in records:
        called = WindowVariant.from_record(r)
        end = r.end
        end_chrom = r.contig
        if r.alt_sv_breakend:
            end_chrom = r.alt_sv_breakend[0]
            if r.contig != end_chrom:
                end = r.alt_sv_breakend[1]
        vt = r.variant_type
        if vt is VariantType.INV:
            if r.pos + half > r.end - half:
                windows.append(Window(r.contig, r.pos - half, r.end + half + 1, called))
            else:
                windows.append(Window(r.contig, r.pos - half, r.pos + half + 1, called))
                windows.append(Window(r.contig, r.end - half, r.end + half + 1, called))
        elif vt is VariantType.TRA:
            windows.append(Window(r.contig, r.pos - half, r.pos + half + 1, called))
            windows.append(Window(end_chrom, end - half, end + half + 1, called))
        elif vt is VariantType.SNV:
            windows.append(Window(r.contig, r.pos - half, r.pos + half + 1, called))
        else:
            if r.length < LONG_SV:
                windows.append(Window(r.contig, r.pos - half, r.end + half + 1, called))
            else:
                windows.append(Window(r.contig, r.pos - half, r.pos + half + 1, called))
                windows.append(Window(end_chrom, end - half, end + half + 1, called))
    for w in windows:
        if w.sequence not in ref_index:
            raise ValueError(f"variant contig {w.sequence!r} is not in the reference FASTA")
    windows.sort(key=lambda w: (ref_index[w.sequence], w.first, w.last))
    return windows


def get_genome_sections(windows: Sequence[Window], fasta: FastaRef) -> List[Window]:
    """Alternating inter-window gaps and windows per contig; whole contigs without windows
    become Window(seq, 0, 0) (SR:245-276)."""
    sections: List[Window] = []
    by_seq: Dict[str, List[Window]] = {k: [] for k in fasta.references}
    for w in windows:
        by_seq[w.sequence].append(w)
    for seq, length in zip(fasta.references, fasta.lengths):
        ws = by_seq[seq]
        if not ws:
            sections.append(Window(seq, 0, 0))
            continue
        first = 1
        for w in ws:
            sections.append(Window(seq, first, w.first - 1))
            first = w.last + 1
            sections.append(w)
        sections.append(Window(seq, first, length - 1))
    idx = fasta.index
    sections.sort(key=lambda w: (idx[w.sequence], w.first, w.last))
    return sections


@dataclasses.dataclass
class Scope:
    """One pileup scope = one CompleteGermlineAnonymizer.anonymize call."""
    id: int
    contig: str
    tid_t: int
    tid_n: int
    first: int
    last: int
    t_rows: np.ndarray        # mapped tumor reads of the pileup, file order
    n_rows: np.ndarray        # mapped normal reads of the pileup, file order
    keep: Optional[WindowVariant]
    is_variant_window: bool
    span_start: int = 0
    span_end: int = 0


class Plan:
    """A sample's plan. The I/O log is kept as columns (``events``: kind 0 open / 1 write /
    2 close, handle, file dataset, file slot, instance dataset, instance scope, 0;
    ``event_rows``: instance row) by the native planner and as tuples by the Python one; each
    form is derived from the other on first use."""

    def __init__(self, scopes: List[Scope], io_log: Optional[List[tuple]], single_end: Dict[int, List[Instance]],
                 stats_events: List[Tuple[str, object]], write_single_end: bool,
                 events: Optional[np.ndarray] = None, event_rows: Optional[np.ndarray] = None,
                 single_reapply: Optional[Dict[int, List[int]]] = None):
        self.scopes = scopes
        self._io_log = io_log
        self.single_end = single_end
        # per single end: 1 when its left-overs are applied a second time (PairSlot::upd, ganon_plan.cpp)
        self.single_reapply = single_reapply or {d: [0] * len(single_end[d]) for d in (0, 1)}
        self.stats_events = stats_events
        self.write_single_end = write_single_end
        self._events = events
        self._event_rows = event_rows

    @property
    def io_log(self) -> List[tuple]:
        # ('open', hid) | ('write', hid, dataset, slot, Instance, reapply) | ('close', hid)
        if self._io_log is None:
            log = []
            for e, r in zip(self._events.tolist(), self._event_rows.tolist()):
                if e[0] == 1:
                    log.append(("write", e[1], e[2], e[3], (e[4], r, e[5]), e[6]))
                elif e[0] == 0:
                    log.append(("open", e[1]))
                else:
                    log.append(("close", e[1]))
            self._io_log = log
        return self._io_log

    def io_arrays(self) -> Tuple[np.ndarray, np.ndarray]:
        if self._events is None:
            n = len(self._io_log)
            ev = np.zeros((n, 7), np.int32)
            rows = np.full(n, -1, np.int64)
            for i, e in enumerate(self._io_log):
                if e[0] == "write":
                    ev[i, :7] = (1, e[1], e[2], e[3], e[4][0], e[4][2], e[5] if len(e) > 5 else 0)
                    rows[i] = e[4][1]
                else:
                    ev[i, :2] = (0 if e[0] == "open" else 2, e[1])
            self._events, self._event_rows = ev, rows
        return self._events, self._event_rows

    def written_arrays(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(dataset, row, scope) of every written record: pair writes, then single ends."""
        ev, rows = self.io_arrays()
        w = ev[:, 0] == 1
        se = [np.array(self.single_end[d], np.int64).reshape(-1, 3) for d in (0, 1)]
        ds = np.concatenate([ev[w, 4].astype(np.int64)] + [x[:, 0] for x in se])
        row = np.concatenate([rows[w]] + [x[:, 1] for x in se])
        sc = np.concatenate([ev[w, 5].astype(np.int64)] + [x[:, 2] for x in se])
        return ds, row, sc

    @property
    def streams(self) -> Dict[Tuple[int, int], List[Instance]]:
        """Records per (dataset, mate slot) in the order write_pair is called."""
        out: Dict[Tuple[int, int], List[Instance]] = {(d, s): [] for d in (0, 1) for s in (0, 1)}
        for ev in self.io_log:
            if ev[0] == "write":
                out[(ev[2], ev[3])].append(ev[4])
        return out

    def written_instances(self):
        for ev in self.io_log:
            if ev[0] == "write":
                yield ev[4]
        for recs in self.single_end.values():
            yield from recs


class SamplePlanner:
    """Plans one tumor/normal pair. Reads are referred to by (dataset, row)."""

    def __init__(self, tumor: ReadTable, normal: ReadTable, fasta: FastaRef, windows: Sequence[Window]):
        self.tables = (tumor, normal)
        self.fasta = fasta
        self.windows = list(windows)
        self.scopes: List[Scope] = []
        self.to_pair: Dict[str, List[Optional[Instance]]] = {}
        self.written: set = set()
        self.io_log: List[tuple] = []
        self._next_hid = 0
        self.stats_events: List[Tuple[str, object]] = []
        self._check_supported(names=not self.native)

    native = False
    # ---- input checks --------------------------------------------------------------------
    def _check_supported(self, names: bool = True) -> None:
        # the native planner plans complex names in contig mode and refuses them in whole-sample
        # mode itself (csrc/ganon_plan.cpp); this Python restatement does not plan them
        for ds, t in enumerate(self.tables if not self.native else ()):
            if np.any(t.flag & (FLAG_SECONDARY | FLAG_SUPPLEMENTARY)):
                raise UnsupportedInput("secondary/supplementary alignments are not supported yet "
                                       "(reference: AnonymizedRead supplementary bookkeeping, AM:98-137)")
            if b"SAZ" in t.aux.tobytes():
                rows = [i for i in range(t.n) if t.has_tag(i, b"SA")]
                if rows:
                    raise UnsupportedInput("reads with an SA tag are not supported yet (AM:100-108)")
        tn = set(self.tables[0].names) & set(self.tables[1].names) if names else None
        if tn:
            raise ValueError(f"{len(tn)} read names occur in both the tumor and the normal BAM; the "
                             "reference keys reads by name only and mixes such reads (SURVEY Q10)")

    # ---- read helpers ----------------------------------------------------------------------
    def name(self, ds: int, row: int) -> str:
        return self.tables[ds].names[row]

    def slot(self, ds: int, row: int) -> int:
        s = int(self.tables[ds].mate_idx[row])
        if s < 0:
            # list[None] in the reference (AM:119-123)
            raise TypeError(f"read {self.name(ds, row)!r} has neither the READ1 nor the READ2 flag; "
                            "the reference cannot store it (SURVEY Q8)")
        return s

    def _ref_end(self, ds: int, row: int) -> Optional[int]:
        t = self.tables[ds]
        if t.is_unmapped[row] or t.n_cigar[row] == 0:
            return None
        return int(t.end[row])

    # ---- pairing / writing (SR:134-165, AM:320-389, SR:375-406) ----------------------------
    # Each reference function that writes opens its own four append-mode handles and closes
    # them when it returns (SR:297-299/366, SR:516-518/558, SR:564-566/600); with Python's
    # buffered text I/O the records of nested handles land in the files in flush order, so
    # the opens, writes and closes are logged and replayed by writer.py.
    def _open(self) -> int:
        hid = self._next_hid
        self._next_hid += 1
        self.io_log.append(("open", hid))
        return hid

    def _close(self, hid: int) -> None:
        self.io_log.append(("close", hid))

    def write_pair(self, i0: Instance, i1: Instance, hid: int, r0: int = 0, r1: int = 0) -> None:
        name = self.name(i0[0], i0[1])
        if name in self.written:
            return
        self.written.add(name)
        ds = i0[0]
        self.io_log.append(("write", hid, ds, 0, i0, r0))
        self.io_log.append(("write", hid, ds, 1, i1, r1))

    def _store_first(self, inst: Instance, update: bool = False) -> List[Optional[Instance]]:
        """to_pair store; ``update``: from a scope's consumer (add_or_update_anonymized_read_from_other,
        AM:351-389), whose update_anonymized_read_from_other re-sets the stored object's left-over
        flag (AM:281-287): its already-applied left-overs are applied once more when it is written
        from to_pair or as a single end. pair = [inst0, inst1, reapply0, reapply1]."""
        name = self.name(inst[0], inst[1])
        slot = self.slot(inst[0], inst[1])
        pair = self.to_pair.get(name)
        if pair is None:
            pair = [None, None, 0, 0]
            self.to_pair[name] = pair
        if pair[slot] is None:
            pair[slot] = inst
        elif update:
            pair[2 + slot] = 1
        return pair

    def passthrough(self, ds: int, row: int, hid: int) -> None:
        """pair_unmapped_or_non_pileup_pairs_and_write: unmasked instance, first stored wins,
        write when both mates are known (never popped from to_pair)."""
        t = self.tables[ds]
        if t.l_seq[row] == 0:
            raise TypeError(f"read {t.names[row]!r} has no SEQ; the reference cannot upper-case it")
        pair = self._store_first((ds, row, -1))
        if pair[0] is not None and pair[1] is not None:
            self.write_pair(pair[0], pair[1], hid, pair[2], pair[3])

    # ---- scopes ------------------------------------------------------------------------------
    def _pileup_reads(self, ds: int, contig: str, first: int, last: int) -> np.ndarray:
        t = self.tables[ds]
        rows = t.fetch(contig, first, last)
        rows = rows[~t.is_unmapped[rows]]
        if len(rows) and np.any(t.n_cigar[rows] == 0):
            raise TypeError("mapped read without CIGAR in a pileup (reference_end is None)")
        return rows

    def new_scope(self, contig: str, first: int, last: int, keep: Optional[WindowVariant],
                  is_variant_window: bool) -> Scope:
        t_rows = self._pileup_reads(0, contig, first, last)
        n_rows = self._pileup_reads(1, contig, first, last)
        sc = Scope(len(self.scopes), contig, self.tables[0].tid_of(contig), self.tables[1].tid_of(contig),
                   first, last, t_rows, n_rows, keep, is_variant_window)
        starts, ends = [], []
        for ds, rows in ((0, t_rows), (1, n_rows)):
            if len(rows):
                starts.append(int(self.tables[ds].pos[rows].min()))
                ends.append(int(self.tables[ds].end[rows].max()))
        sc.span_start = min(starts) if starts else 0
        sc.span_end = max(ends) if ends else 0
        self.scopes.append(sc)
        self.stats_events.append(("scope", sc.id))
        return sc

    def registration_order(self, sc: Scope) -> List[Tuple[int, int]]:
        """(dataset, row) in the order the reference first meets each read: pileup columns by
        position, the tumor column before the normal one, reads in file order."""
        T, N = self.tables
        pos = np.concatenate([T.pos[sc.t_rows], N.pos[sc.n_rows]]).astype(np.int64)
        ds = np.concatenate([np.zeros(len(sc.t_rows), np.int64), np.ones(len(sc.n_rows), np.int64)])
        fo = np.concatenate([np.arange(len(sc.t_rows)), np.arange(len(sc.n_rows))])
        rows = np.concatenate([sc.t_rows, sc.n_rows]).astype(np.int64)
        order = np.lexsort((fo, ds, pos))
        return list(zip(ds[order].tolist(), rows[order].tolist()))

    def yield_sequence(self, sc: Scope) -> List[List[Optional[Instance]]]:
        """Pairs in the order CompleteGermlineAnonymizer.anonymize yields them (AM:472-532)."""
        reg = self.registration_order(sc)
        pairs: Dict[str, List[Optional[Instance]]] = {}
        max_end: Dict[str, int] = {}
        for ds, row in reg:
            name = self.name(ds, row)
            slot = self.slot(ds, row)
            p = pairs.get(name)
            if p is None:
                p = [None, None]
                pairs[name] = p
                max_end[name] = int(self.tables[ds].end[row])
            else:
                max_end[name] = max(max_end[name], int(self.tables[ds].end[row]))
            if p[slot] is not None:
                raise UnsupportedInput(f"two alignments of {name!r} with the same mate flag in one scope")
            p[slot] = (ds, row, sc.id)
        # normal columns: union of the normal reads' [pos, end)
        N = self.tables[1]
        if len(sc.n_rows):
            s = N.pos[sc.n_rows].astype(np.int64)
            e = N.end[sc.n_rows].astype(np.int64)
            o = np.argsort(s, kind="stable")
            s, e = s[o], e[o]
            run_end = np.maximum.accumulate(e)
            brk = np.nonzero(s[1:] > run_end[:-1])[0] + 1
            m_start = s[np.concatenate([[0], brk])]
            m_end = run_end[np.concatenate([brk - 1, [len(s) - 1]])]
        else:
            m_start = m_end = np.zeros(0, np.int64)
        scan, rest = [], []
        for rank, (name, p) in enumerate(pairs.items()):
            if p[0] is not None and p[1] is not None:
                x = max_end[name] + 1                      # first column with right_most_end < pos
                k = int(np.searchsorted(m_end, x, side="right"))
                if k < len(m_end):
                    scan.append((max(x, int(m_start[k])), rank, p))
                    continue
            rest.append(p)
        scan.sort(key=lambda t: (t[0], t[1]))
        return [t[2] for t in scan] + rest

    def anonymize_window(self, contig: str, first: int, last: int, keep: Optional[WindowVariant],
                         is_variant_window: bool) -> None:
        """SR:279-372 with the yielded pairs consumed as SR:304-361 does."""
        sc = self.new_scope(contig, first, last, keep, is_variant_window)
        hid = self._open()
        for p0, p1 in self.yield_sequence(sc):
            if p0 is not None and p1 is not None:
                self.write_pair(p0, p1, hid)
                continue
            name = None
            for inst in (p0, p1):
                if inst is not None:
                    self._store_first(inst, update=True)
                    name = self.name(inst[0], inst[1])
            upd = self.to_pair[name]
            if upd[0] is not None and upd[1] is not None:
                self.write_pair(upd[0], upd[1], hid, upd[2], upd[3])
                del self.to_pair[name]
        self._close(hid)

    # ---- inter-window clustering (pileup_io.pyx:124-298) --------------------------------------
    def iter_fetch_pair(self, contig: str, first: Optional[int], last: Optional[int]) -> Iterator[tuple]:
        T, N = self.tables
        it = [iter(T.fetch(contig, first, last).tolist()), iter(N.fetch(contig, first, last).tolist())]
        tabs = (T, N)

        def mapped(ds, r):
            return not tabs[ds].is_unmapped[r]

        def end_of(ds, r):
            return self._ref_end(ds, r)

        def cmp_reads(ds, a, b):
            ta = tabs[ds]
            fa, fb = int(ta.pos[a]), int(ta.pos[b])
            la = end_of(ds, a) if mapped(ds, a) else fa
            lb = end_of(ds, b) if mapped(ds, b) else fb
            from .variants import compare
            return compare(int(ta.tid[a]), fa, la, int(ta.tid[b]), fb, lb)

        def collect(ds, arr, unmapped):
            while True:
                nxt = next(it[ds], None)
                if nxt is None:
                    return None
                if not mapped(ds, nxt):
                    unmapped.append(nxt)
                    continue
                if not (-1 <= cmp_reads(ds, arr[-1], nxt) <= 1):
                    return nxt
                arr.append(nxt)

        def rightmost(ds, arr, prev):
            right = 0 if prev is None else prev
            for r in arr:
                if mapped(ds, r):
                    e = end_of(ds, r)
                    if e is None:
                        raise TypeError("mapped read without reference_end")
                    right = max(right, e)
            return right

        from .variants import compare
        arrs = [[], []]
        unm = [[], []]
        cur = [next(it[0], None), next(it[1], None)]
        yielded = [True, True]
        seqi = [None, None]
        left = [None, None]
        right = [None, None]
        if cur[0] is None and cur[1] is None:
            return
        for ds in (0, 1):
            if cur[ds] is not None:
                r = cur[ds]
                seqi[ds] = int(tabs[ds].tid[r])
                left[ds] = int(tabs[ds].pos[r])
                right[ds] = end_of(ds, r)
                arrs[ds].append(r)

        def restart(ds):
            r = cur[ds]
            yielded[ds] = True
            arrs[ds] = [r]
            seqi[ds] = int(tabs[ds].tid[r])
            left[ds] = int(tabs[ds].pos[r])
            right[ds] = end_of(ds, r)

        while True:
            for ds in (0, 1):
                if yielded[ds] and cur[ds] is not None:
                    cur[ds] = collect(ds, arrs[ds], unm[ds])
                    right[ds] = rightmost(ds, arrs[ds], right[ds])
                    yielded[ds] = False
            if cur[0] is None and cur[1] is None:
                yield arrs[0], None, None
                yield None, arrs[1], None
                break
            if cur[0] is not None and cur[1] is not None:
                c = compare(seqi[0], left[0], right[0], seqi[1], left[1], right[1])
                if c < -1:
                    yield arrs[0], None, None
                    restart(0)
                elif c > 1:
                    yield None, arrs[1], None
                    restart(1)
                else:
                    yield arrs[0], arrs[1], (contig, min(left[0], left[1]), max(right[0], right[1]))
                    restart(0)
                    restart(1)
            else:
                if cur[0] is not None:
                    yield arrs[0], None, None
                    restart(0)
                if cur[1] is not None:
                    yield None, arrs[1], None
                    restart(1)
        yield None, None, (unm[0], unm[1])

    def anonymize_inter_window_region(self, w: Window) -> None:
        """SR:498-558."""
        first, last = w.first, w.last
        if first + last == 0:
            first = last = None
        events = self.iter_fetch_pair(w.sequence, first, last)
        hid = self._open()
        for t_arr, n_arr, extra in events:
            if t_arr is not None and n_arr is not None:
                seq, lo, hi = extra
                self.anonymize_window(seq, lo, hi, None, False)
            elif t_arr is None and n_arr is None:
                for ds in (0, 1):
                    for r in extra[ds]:
                        self.passthrough(ds, r, hid)
            else:
                ds = 0 if t_arr is not None else 1
                for r in (t_arr if ds == 0 else n_arr):
                    self.passthrough(ds, r, hid)
        self._close(hid)

    def pair_unmapped_mates(self) -> None:
        """SR:561-600: re-fetch every window for placed-unmapped mates of unpaired reads."""
        hid = self._open()
        for w in self.windows:
            for ds in (0, 1):
                t = self.tables[ds]
                for r in t.fetch(w.sequence, w.first - 1, w.last).tolist():
                    if t.is_unmapped[r] and t.names[r] in self.to_pair:
                        self.passthrough(ds, r, hid)
        self._close(hid)

    # ---- whole sample (SR:625-760) -----------------------------------------------------------
    def run(self) -> Plan:
        sections = get_genome_sections(self.windows, self.fasta)
        for w in sections:
            if w.is_variant_window():
                self.stats_events.append(("window", str(w)))
                self.anonymize_window(w.sequence, w.first, w.last, w.variant, True)
            else:
                self.stats_events.append(("outside", None))
                self.anonymize_inter_window_region(w)
        if self.to_pair:
            self.pair_unmapped_mates()
        for k in self.written:
            self.to_pair.pop(k, None)
        single: Dict[int, List[Instance]] = {0: [], 1: []}
        reapply: Dict[int, List[int]] = {0: [], 1: []}
        for name, pair in self.to_pair.items():
            sl = 0 if pair[0] is not None else 1
            inst = pair[sl]
            single[inst[0]].append(inst)
            reapply[inst[0]].append(pair[2 + sl])
        return Plan(self.scopes, self.io_log, single, self.stats_events, bool(self.to_pair), single_reapply=reapply)


class NativeSamplePlanner(SamplePlanner):
    """The same plan from libganon_host.so (``ganon_plan_run``, csrc/ganon_plan.cpp): the
    control flow above restated in C++ over the read tables' columns. The product's planner;
    SamplePlanner (pure Python) is the second implementation the tests compare it with."""

    native = True
    only_contig: Optional[int] = None   # contig mode (ContigPlanner)
    force_names: Sequence[bytes] = ()   # contig mode: names planned as cross names (ContigPlanner)
    job: Optional[Tuple[int, int, int, int]] = None   # job mode: sections [lo, hi) of the contig, region

    def run(self) -> Plan:
        from . import native
        refs = list(self.fasta.references)
        cidx = {c: i for i, c in enumerate(refs)}
        w = self.windows
        res = native.plan_sample(self.tables, refs, list(self.fasta.lengths),
                                 [cidx[x.sequence] for x in w], [x.first for x in w], [x.last for x in w],
                                 only_contig=self.only_contig, force_names=self.force_names, job=self.job)
        self.contig_exports = {"left": res["left"], "cand": res["cand"], "objs": res["objs"],
                               "obj_rows": res["obj_rows"]}
        T, N = self.tables
        t_rows, n_rows = res["t_rows"], res["n_rows"]
        to, no = res["scope_t_off"], res["scope_n_off"]
        for k in range(len(res["scope_contig"])):
            contig = refs[int(res["scope_contig"][k])]
            wi = int(res["scope_window"][k])
            sc = Scope(k, contig, T.tid_of(contig), N.tid_of(contig), int(res["scope_first"][k]),
                       int(res["scope_last"][k]), t_rows[to[k]:to[k + 1]], n_rows[no[k]:no[k + 1]],
                       w[wi].variant if wi >= 0 else None, wi >= 0)
            sc.span_start = int(res["scope_span_start"][k])
            sc.span_end = int(res["scope_span_end"][k])
            self.scopes.append(sc)
        for kind, val in res["stats"].tolist():
            if kind == 0:
                self.stats_events.append(("window", str(w[val])))
            elif kind == 1:
                self.stats_events.append(("outside", None))
            else:
                self.stats_events.append(("scope", val))
        single = {d: [(d, r, s) for r, s, _ in res["single"][d].tolist()] for d in (0, 1)}
        reapply = {d: [x for _, _, x in res["single"][d].tolist()] for d in (0, 1)}
        plan = Plan(self.scopes, None, single, self.stats_events, res["write_single_end"], single_reapply=reapply,
                    events=res["events"], event_rows=res["event_rows"])
        plan.skip = res["skip"]
        return plan


class ContigPlanner(NativeSamplePlanner):
    """Contig mode of the native planner (include/ganon_host.h ``contig_mode``): plans one FASTA
    contig from tables holding only that contig's records. Pairing operations on names with a
    record on another sequence become placeholder events (kinds 3/4/5) for stream.py's resolver;
    ``contig_exports`` holds the contig's unwritten pairs and pair_unmapped_mates candidates.
    ``force_names``: names to plan as cross names although their records here say nothing of
    another sequence (secondary alignments elsewhere whose mate is on this contig, stream.py)."""

    def __init__(self, tumor: ReadTable, normal: ReadTable, fasta: FastaRef, windows: Sequence[Window],
                 contig_index: int, force_names: Sequence[bytes] = (), job: Optional[Tuple[int, int, int, int]] = None):
        """``job``: (first section, end section, region start, region end): job mode, a run of the
        contig's sections planned from the records overlapping the region (stream.py)."""
        self.only_contig = int(contig_index)
        self.force_names = sorted(force_names)
        self.job = job
        super().__init__(tumor, normal, fasta, windows)


def make_planner(tumor: ReadTable, normal: ReadTable, fasta: FastaRef, windows: Sequence[Window]) -> SamplePlanner:
    """The native planner; GANON_PLANNER=python selects the pure-Python one."""
    import os
    cls = SamplePlanner if os.environ.get("GANON_PLANNER") == "python" else NativeSamplePlanner
    return cls(tumor, normal, fasta, windows)
