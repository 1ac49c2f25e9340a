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
from typing import Dict, Optional, Tuple

import numpy as np

from . import native
from .indels import IndelCall, query_sequence
from .io.bam import ReadTable
from .io.fasta import FastaRef
from .planner import Plan, SamplePlanner
from .variants import VariantType, kept_snv


@dataclasses.dataclass
class MaskResult:
    seq_out: np.ndarray                    # masked copy of the batch's seq blob
    seq_base: Tuple[int, int]              # byte offset of the tumor / normal blob in seq_out
    batch_index: Dict[Tuple[int, int], int]
    scope_snv_calls: np.ndarray            # [n_scopes] masked TN SNV calls
    scope_masked_bases: np.ndarray         # [n_scopes]
    scope_indel_counts: Dict[int, Dict[VariantType, int]]
    leftovers: Dict[Tuple[int, int, int], list]   # (ds, row, scope) -> indel edits
    totals: np.ndarray
    arrays: dict                           # the device batch (kept for tests/bench)
    dup_off: Dict[Tuple[int, int, int], int] = dataclasses.field(default_factory=dict)

    def masked_nib(self, tables, ds: int, row: int, scope: int) -> int:
        """Nibble offset in seq_out of read (ds, row) as masked by ``scope``."""
        o = self.dup_off.get((ds, row, scope))
        if o is None:
            o = self.seq_base[ds] + int(tables[ds].seq_off[row])
        return 2 * o


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
    seq_parts = [T.seq, N.seq]
    dup_off: Dict[Tuple[int, int, int], int] = {}
    dup_rows = []
    extra = {k: [] for k in ("ref_start", "read_len", "seq_off", "cig_off", "n_cig", "dataset")}
    n_seq = len(T.seq) + len(N.seq)
    ex_ws = []
    for i in np.nonzero(~first)[0].tolist():        # the same read masked in another scope
        d, r, sid = int(w_ds[i]), int(w_row[i]), int(w_sc[i])
        if (d, r, sid) in dup_off or ws[b[i]] == loc[sid]:
            continue
        t = tables[d]
        nbytes = (int(t.l_seq[r]) + 1) // 2
        o = int(t.seq_off[r])
        seq_parts.append(t.seq[o:o + nbytes])
        dup_off[(d, r, sid)] = n_seq
        k = int(loc[sid])
        seg = incid[incid_off[k]:incid_off[k + 1]]
        hit = np.nonzero(seg == b[i])[0]
        seg[hit] = n_reads + len(dup_rows)
        extra["ref_start"].append(int(t.pos[r]))
        extra["read_len"].append(int(t.l_seq[r]))
        extra["seq_off"].append(n_seq)
        extra["cig_off"].append(int(t.cig_off[r]) + cig_base[d])
        extra["n_cig"].append(int(t.n_cigar[r]))
        extra["dataset"].append(d)
        ex_ws.append(k)
        dup_rows.append((d, r))
        n_seq += nbytes
    if dup_rows:
        for f, dt in (("ref_start", np.int32), ("read_len", np.int32), ("seq_off", np.int64), ("cig_off", np.int64),
                      ("n_cig", np.int32), ("dataset", np.uint8)):
            arr[f] = np.concatenate([arr[f], np.array(extra[f], dt)])
        ws = np.concatenate([ws, np.array(ex_ws, np.int32)])
    arr["seq_nt16"] = np.ascontiguousarray(np.concatenate(seq_parts).astype(np.uint8))
    arr["write_scope"] = ws
    arr["scope_incid_off"] = incid_off
    arr["incid_read"] = incid
    skip = getattr(plan, "skip", None)
    if skip is not None and len(skip):
        # seen_read_alns (variation_classifier.py:196-207): later alignments of a read in a scope
        # are tallied for SNVs but not for indels
        drop = np.zeros(len(incid), bool)
        for sid, d, r in skip.tolist():
            k = int(loc[sid]) if sid < len(plan.scopes) else -1
            if k < 0:
                continue
            br = n_reads + dup_rows.index((d, r)) if (d, r, sid) in dup_off else int(bidx[d][r])
            seg = incid[incid_off[k]:incid_off[k + 1]]
            drop[incid_off[k] + np.nonzero(seg == br)[0]] = True
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

    @property
    def engine(self):
        if self._engine is None:
            self._engine = native.HipMasker(self.device)
        return self._engine

    def format_fastq(self, recs: dict) -> bytes:
        """FASTQ records on the masking engine's device (``ganon_fastq_format_hip``); an engine
        without a formatter (none in the product) leaves them to libganon_host.so."""
        fmt = getattr(self.engine, "format_fastq", None)
        return fmt(recs) if fmt is not None else native.host_format_fastq(recs)

    def anonymize(self, planner: SamplePlanner, plan: Plan, scope_ids=None, written=None) -> MaskResult:
        """Mask all scopes of ``plan`` (or the contig shard ``scope_ids``) in one device batch.
        Per-scope counts come back indexed by plan scope id (zero outside the shard)."""
        tables = planner.tables
        fasta = planner.fasta
        arrays, meta = build_batch(plan, tables, fasta, scope_ids, written)
        out, b_calls, b_bases, totals, irecs = self.engine.mask(arrays, indels=True)
        calls = np.zeros(len(plan.scopes), np.int32)
        bases = np.zeros(len(plan.scopes), np.int32)
        calls[meta["scope_ids"]] = b_calls
        bases[meta["scope_ids"]] = b_bases
        indel_counts, leftovers = indel_results(irecs, meta, plan, tables, fasta)
        return MaskResult(out, meta["seq_base"], {}, calls, bases, indel_counts, leftovers, totals, arrays,
                          meta["dup_off"])


ANONYMIZER_ALGORITHMS = {CompleteGermlineAnonymizer.name: CompleteGermlineAnonymizer}
