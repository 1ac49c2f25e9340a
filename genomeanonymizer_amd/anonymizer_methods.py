"""The anonymizer plugin, MI355X edition.

Reference interface: the ``Anonymizer`` protocol selected with ``-m complete_germline``
(anonymizer_methods.py:290-309, genome_anonymizer.py:9-13, :73) and its one
implementation ``CompleteGermlineAnonymizer`` (anonymizer_methods.py:422-556), called once
per scope with a merged tumor/normal pileup and yielding anonymized read pairs.

Here the plugin receives the whole plan of a sample (all scopes, planner.py) and masks
every scope in ONE device batch through the C ABI of include/ganon.h (libganon_hip.so):
SNV tally -> TN classification -> overwrite, per scope, on the GPU; the germline indel tally
(process_indels + TN classification + normal-column check) runs on the GPU too
(``ganon_indel_*``), and its records become the reference's left-over edits, applied by the
host when a record is formatted (variable-length output, indels.py). There is no CPU
masking path: a missing HIP library or device raises ``GanonError``.
"""
from __future__ import annotations

import dataclasses
import threading
from typing import Callable, Dict, Optional, Tuple

import numpy as np

from . import native
from .indels import IndelCall, query_sequence
from .io.bam import ReadTable
from .io.fasta import FastaRef
from .planner import Plan, SamplePlanner
from .variants import VariantType, kept_snv


@dataclasses.dataclass
class MaskResult:
    _seq: Optional[np.ndarray]             # masked copy of the batch's seq blob (None: not fetched yet)
    seq_base: Tuple[int, int]              # byte offset of the tumor / normal blob in seq_out
    batch_index: Dict[Tuple[int, int], int]
    scope_snv_calls: np.ndarray            # [n_scopes] masked TN SNV calls
    scope_masked_bases: np.ndarray         # [n_scopes]
    scope_indel_counts: Dict[int, Dict[VariantType, int]]
    leftovers: Dict[Tuple[int, int, int], list]   # (ds, row, scope) -> indel edits
    totals: np.ndarray
    arrays: dict                           # the device batch (kept for tests/bench)
    dup_off: Dict[Tuple[int, int, int], int] = dataclasses.field(default_factory=dict)
    device_gen: int = -1                   # the engine's job batch holding this result (format_fastq_batch)
    seq_fetch: Optional[Callable[[], np.ndarray]] = None   # downloads _seq while that batch holds it

    @property
    def seq_out(self) -> np.ndarray:
        """The masked bases; fetched from the device on first use when the mask left them there."""
        if self._seq is None:
            if self.seq_fetch is None:
                raise RuntimeError("masked bases were not kept")
            self._seq = self.seq_fetch()
            self.seq_fetch = None
        return self._seq

    def masked_nib(self, tables, ds: int, row: int, scope: int) -> int:
        """Nibble offset in seq_out of read (ds, row) as masked by ``scope``."""
        o = self.dup_off.get((ds, row, scope))
        if o is None:
            o = self.seq_base[ds] + int(tables[ds].seq_off[row])
        return 2 * o


def _seq_buffer(parts, extra=None) -> np.ndarray:
    """The batch's bases (the tables' blobs back to back, then the further copies) in one page-locked
    block when the GPU engine is loaded (native.PINNED: the batch upload then goes by DMA instead of
    through the runtime's staging copies), else in fresh memory."""
    parts = [np.asarray(p, np.uint8) for p in parts] + ([np.asarray(extra, np.uint8)] if extra is not None else [])
    n = sum(len(p) for p in parts)
    out = native.PINNED.take(n) if n >= (8 << 20) and native.hip_loaded() else np.empty(n, np.uint8)
    at = 0
    for p in parts:
        out[at:at + len(p)] = p
        at += len(p)
    return out


def build_batch(plan: Plan, tables: Tuple[ReadTable, ReadTable], fasta: FastaRef,
                scope_ids=None, written=None) -> Tuple[dict, dict]:
    """Lay the plan's scopes (all, or the subset ``scope_ids`` of one contig shard) out as
    one ganon_batch (include/ganon.h). Batch scope k is plan scope ``meta['scope_ids'][k]``.
    ``written``: (dataset, row, scope) arrays of the instances to mask (default: the plan's written
    records). A read masked in a second scope (the alignments of complex names, objects.py) gets a
    copy of its record in the batch, the one that scope's incidence points at."""
    T, N = tables
    packed, nib_off = fasta.packed()
    scopes = plan.scopes if scope_ids is None else [plan.scopes[i] for i in scope_ids]
    # batch reads: every read of every scope, tumor rows then normal rows
    in_scope = [np.zeros(T.n, bool), np.zeros(N.n, bool)]
    for sc in scopes:
        in_scope[0][sc.t_rows] = True
        in_scope[1][sc.n_rows] = True
    rows = [np.nonzero(in_scope[0])[0], np.nonzero(in_scope[1])[0]]
    bidx = [np.full(T.n, -1, np.int64), np.full(N.n, -1, np.int64)]
    bidx[0][rows[0]] = np.arange(len(rows[0]))
    bidx[1][rows[1]] = len(rows[0]) + np.arange(len(rows[1]))
    n_reads = len(rows[0]) + len(rows[1])
    seq_base = (0, len(T.seq))
    cig_base = (0, len(T.cigar))
    arr = {}
    cat = lambda f, dt: np.concatenate([getattr(T, f)[rows[0]], getattr(N, f)[rows[1]]]).astype(dt)
    arr["ref_start"] = cat("pos", np.int32)
    arr["read_len"] = cat("l_seq", np.int32)
    arr["seq_off"] = np.concatenate([T.seq_off[rows[0]] + seq_base[0], N.seq_off[rows[1]] + seq_base[1]]).astype(np.int64)
    arr["cig_off"] = np.concatenate([T.cig_off[rows[0]] + cig_base[0], N.cig_off[rows[1]] + cig_base[1]]).astype(np.int64)
    arr["n_cig"] = cat("n_cigar", np.int32)
    arr["cigar"] = np.ascontiguousarray(np.concatenate([T.cigar, N.cigar]).astype(np.uint32))
    arr["dataset"] = np.concatenate([np.zeros(len(rows[0]), np.uint8), np.ones(len(rows[1]), np.uint8)])
    ws = np.full(n_reads, -1, np.int32)
    w_ds, w_row, w_sc = plan.written_arrays() if written is None else written
    w_ds, w_row, w_sc = (np.asarray(x, np.int64) for x in (w_ds, w_row, w_sc))
    loc = np.full(len(plan.scopes) + 1, -1, np.int64)
    loc[[sc.id for sc in scopes]] = np.arange(len(scopes))
    sel = (w_sc >= 0) & (loc[np.where(w_sc >= 0, w_sc, len(plan.scopes))] >= 0)
    w_ds, w_row, w_sc = w_ds[sel], w_row[sel], w_sc[sel]
    b = np.where(w_ds == 0, bidx[0][np.where(w_ds == 0, w_row, 0)], bidx[1][np.where(w_ds == 1, w_row, 0)])
    first = np.ones(len(b), bool)
    if len(b):
        _, fi = np.unique(b, return_index=True)
        first[:] = False
        first[fi] = True
    ws[b[first]] = loc[w_sc[first]]
    counts = np.array([len(sc.t_rows) + len(sc.n_rows) for sc in scopes], np.int64)
    incid_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    incid = (np.concatenate([np.concatenate([bidx[0][sc.t_rows], bidx[1][sc.n_rows]]) for sc in scopes]).astype(np.int32)
             if scopes else np.zeros(0, np.int32))
    # the same read masked in another scope: a copy of its record, the one that scope's
    # incidence points at (first occurrence per (dataset, row, scope); vectorised)
    cand = np.nonzero(~first)[0]
    cand = cand[ws[b[cand]] != loc[w_sc[cand]]]
    if len(cand):
        trip = np.stack([w_ds[cand], w_row[cand], w_sc[cand]], axis=1)
        _, fi = np.unique(trip, axis=0, return_index=True)
        cand = cand[np.sort(fi)]
    d_ds, d_row, d_sc = w_ds[cand], w_row[cand], w_sc[cand]
    nd = len(cand)
    d0 = d_ds == 0
    r0, r1 = np.where(d0, d_row, 0), np.where(d0, 0, d_row)
    pick = lambda f: np.where(d0, getattr(T, f)[r0] if T.n else 0, getattr(N, f)[r1] if N.n else 0).astype(np.int64)
    d_len = pick("l_seq")
    nbytes = (d_len + 1) // 2
    n_seq = len(T.seq) + len(N.seq)
    d_seq = n_seq + np.concatenate([[0], np.cumsum(nbytes)[:-1]]).astype(np.int64) if nd else np.zeros(0, np.int64)
    d_k = loc[d_sc]
    d_idx = n_reads + np.arange(nd, dtype=np.int64)          # batch read index of each copy
    if nd:
        src = np.repeat(np.where(d0, 0, len(T.seq)) + pick("seq_off"), nbytes) + \
            (np.arange(int(nbytes.sum())) - np.repeat(np.concatenate([[0], np.cumsum(nbytes)[:-1]]), nbytes))
        seq_all = _seq_buffer([T.seq, N.seq], np.concatenate([T.seq, N.seq])[src])
        # re-point the copy's scope incidences at the copy
        inc_k = np.repeat(np.arange(len(scopes), dtype=np.int64), counts)
        M = n_reads + nd + 1
        dkey = d_k * M + b[cand]
        order = np.argsort(dkey, kind="stable")
        ikey = inc_k * M + incid
        pos = np.minimum(np.searchsorted(dkey[order], ikey), nd - 1)
        hit = dkey[order][pos] == ikey
        incid = incid.copy()
        incid[hit] = d_idx[order][pos[hit]].astype(np.int32)
        for f, v, dt in (("ref_start", pick("pos"), np.int32), ("read_len", d_len, np.int32), ("seq_off", d_seq, np.int64),
                         ("cig_off", pick("cig_off") + np.where(d0, cig_base[0], cig_base[1]), np.int64),
                         ("n_cig", pick("n_cigar"), np.int32), ("dataset", d_ds, np.uint8)):
            arr[f] = np.concatenate([arr[f], v.astype(dt)])
        ws = np.concatenate([ws, d_k.astype(np.int32)])
    else:
        seq_all = _seq_buffer([T.seq, N.seq])
    dup_off = dict(zip(zip(d_ds.tolist(), d_row.tolist(), d_sc.tolist()), d_seq.tolist()))
    dup_rows = list(zip(d_ds.tolist(), d_row.tolist()))
    arr["seq_nt16"] = seq_all
    arr["write_scope"] = ws
    arr["scope_incid_off"] = incid_off
    arr["incid_read"] = incid
    skip = getattr(plan, "skip", None)
    if skip is not None and len(skip):
        # seen_read_alns (variation_classifier.py:196-207): later alignments of a read in a scope
        # are tallied for SNVs but not for indels
        s_sc, s_ds, s_row = (np.asarray(skip[:, j], np.int64) for j in range(3))
        ok = s_sc < len(plan.scopes)
        s_sc, s_ds, s_row = s_sc[ok], s_ds[ok], s_row[ok]
        s_k = loc[s_sc]
        ok = s_k >= 0
        s_sc, s_ds, s_row, s_k = s_sc[ok], s_ds[ok], s_row[ok], s_k[ok]
        br = np.where(s_ds == 0, bidx[0][np.where(s_ds == 0, s_row, 0)] if T.n else -1,
                      bidx[1][np.where(s_ds == 1, s_row, 0)] if N.n else -1)
        if nd:    # a read copied into that scope: the copy
            key3 = lambda a, b_, c: (c * 2 + a) * (max(T.n, N.n) + 1) + b_
            dk3 = key3(d_ds, d_row, d_sc)
            o3 = np.argsort(dk3)
            sk3 = key3(s_ds, s_row, s_sc)
            p3 = np.minimum(np.searchsorted(dk3[o3], sk3), nd - 1)
            h3 = dk3[o3][p3] == sk3
            br = np.where(h3, d_idx[o3][p3], br)
        inc_k = np.repeat(np.arange(len(scopes), dtype=np.int64), counts)
        M = n_reads + nd + 1
        drop = np.isin(inc_k * M + incid, s_k * M + br)
        kept = np.diff(np.concatenate([[0], np.cumsum(~drop)])[incid_off])
        arr["indel_incid_off"] = np.concatenate([[0], np.cumsum(kept)]).astype(np.int64)
        arr["indel_incid_read"] = incid[~drop]
    arr["scope_span_start"] = np.array([sc.span_start for sc in scopes], np.int32)
    arr["scope_span_len"] = np.array([sc.span_end - sc.span_start for sc in scopes], np.int32)
    arr["scope_ref_off"] = np.array([nib_off[sc.contig] + sc.span_start for sc in scopes], np.int64)
    arr["ref_nt16"] = np.ascontiguousarray(packed)
    keep = [kept_snv(sc.keep) if sc.is_variant_window else (-1, 0) for sc in scopes]
    arr["keep_pos"] = np.array([k[0] for k in keep], np.int32)
    arr["keep_code"] = np.array([k[1] for k in keep], np.uint8)
    meta = {"bidx": bidx, "rows": rows, "seq_base": seq_base, "dup_off": dup_off, "dup_rows": dup_rows,
            "scope_ids": np.array([sc.id for sc in scopes], np.int64)}
    return arr, meta


def indel_results(recs: np.ndarray, meta: dict, plan: Plan, tables: Tuple[ReadTable, ReadTable],
                  fasta: FastaRef):
    """Device indel records (``native.INDEL_REC``, sorted by scope, pos, rank) -> the reference's
    per-scope statistics counts (``stats_recorder.count_variant``, anonymizer_methods.py:555-556)
    and left-over lists ``(ds, row, scope) -> [(in_read_pos, IndelCall)]`` in the order
    ``mask_germline_variants`` appends them (by normal column, then call order at the column).
    The kept window variant (AM:546-547) is excluded here: its identity includes the allele."""
    rows = meta["rows"]
    n_t = len(rows[0])
    n_p = n_t + len(rows[1])
    dups = meta.get("dup_rows", [])

    def ds_row(r: int) -> Tuple[int, int]:
        if r >= n_p:
            return dups[r - n_p]
        return (0, int(rows[0][r])) if r < n_t else (1, int(rows[1][r - n_t]))

    indel_counts: Dict[int, Dict[VariantType, int]] = {}
    leftovers: Dict[Tuple[int, int, int], list] = {}
    live: Dict[Tuple[int, int, int], Optional[IndelCall]] = {}
    for rec in recs.tolist():
        b_scope, pos, length, vtype, rank, kind, read, irp = rec
        sid = int(meta["scope_ids"][b_scope])
        key = (sid, pos, rank)
        ds, row = ds_row(read)
        if kind == native.INDEL_CALL:
            sc = plan.scopes[sid]
            vt = VariantType(vtype)
            end = pos + 1 if vt is VariantType.INS else pos + length - 1
            alen = length if vt is VariantType.INS else 2
            allele = query_sequence(tables[ds], row)[irp:irp + alen]
            if sc.is_variant_window and sc.keep is not None and \
                    (sc.contig, vt, pos, end, length, allele) == sc.keep.identity():
                live[key] = None
                continue
            counts = indel_counts.setdefault(sid, {VariantType.DEL: 0, VariantType.INS: 0})
            counts[vt] += 1
            live[key] = IndelCall(pos, end, vt, length, allele, fasta.fetch(sc.contig, pos, end + 1).upper())
        else:
            call = live[key]
            if call is not None:
                leftovers.setdefault((ds, row, sid), []).append((irp, call))
    return indel_counts, leftovers


class CompleteGermlineAnonymizer:
    """Masks every germline (tumor AND normal) SNV of every scope on the GPU and tallies its
    germline indels there; keeps the window's own variant; indel edits are left-overs applied
    when a pair is yielded, like the reference."""

    name = "complete_germline"

    def __init__(self, device: int = 0, engine=None):
        self.device = device
        self._engine = engine
        # one caller of the engine at a time (the streamed path formats on a writer thread while the
        # next contig masks; the engine's context is not thread-safe)
        self.lock = threading.RLock()

    @property
    def engine(self):
        if self._engine is None:
            self._engine = native.HipMasker(self.device)
        return self._engine

    def format_fastq(self, recs: dict) -> bytes:
        """FASTQ records on the masking engine's device (``ganon_fastq_format_hip``); an engine
        without a formatter (none in the product) leaves them to libganon_host.so."""
        fmt = getattr(self.engine, "format_fastq", None)
        if fmt is None:
            return native.host_format_fastq(recs)
        with self.lock:
            return fmt(recs)

    def format_fastq_batch(self, recs: dict, gen: int):
        """The same records formatted from the engine's resident job batch (its masked output and
        input bases, no upload of the sequences), or None when that batch has moved on."""
        fmt = getattr(self.engine, "format_fastq_batch", None)
        if fmt is None:
            return None
        with self.lock:
            return fmt(recs, gen)

    def anonymize(self, planner: SamplePlanner, plan: Plan, scope_ids=None, written=None, batch=None,
                  lazy_seq: bool = False) -> MaskResult:
        """Mask all scopes of ``plan`` (or the contig shard ``scope_ids``) in one device batch
        (``batch``: build_batch's result when the caller built it already). Per-scope counts come
        back indexed by plan scope id (zero outside the shard). ``lazy_seq``: leave the masked bases
        on the device (MaskResult.seq_out downloads them on first use, valid until the engine's next
        job; the streamed path formats from the device and rarely needs them)."""
        tables = planner.tables
        fasta = planner.fasta
        arrays, meta = batch if batch is not None else build_batch(plan, tables, fasta, scope_ids, written)
        fetch = None
        with self.lock:
            if lazy_seq and hasattr(self.engine, "job_seq"):
                out, b_calls, b_bases, totals, irecs = self.engine.mask(arrays, indels=True, fetch_seq=False)
                gen = self.engine.job_gen
                eng, lock = self.engine, self.lock

                def fetch():
                    with lock:
                        return eng.job_seq(gen)
            else:
                out, b_calls, b_bases, totals, irecs = self.engine.mask(arrays, indels=True)
                gen = getattr(self.engine, "job_gen", -1)
        calls = np.zeros(len(plan.scopes), np.int32)
        bases = np.zeros(len(plan.scopes), np.int32)
        calls[meta["scope_ids"]] = b_calls
        bases[meta["scope_ids"]] = b_bases
        indel_counts, leftovers = indel_results(irecs, meta, plan, tables, fasta)
        return MaskResult(out, meta["seq_base"], {}, calls, bases, indel_counts, leftovers, totals, arrays,
                          meta["dup_off"], gen, fetch)


ANONYMIZER_ALGORITHMS = {CompleteGermlineAnonymizer.name: CompleteGermlineAnonymizer}
