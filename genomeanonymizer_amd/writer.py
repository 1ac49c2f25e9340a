"""FASTQ and statistics output.

* FASTQ records as ``write_pair`` / ``write_single_end_reads`` write them
  (short_read_tumor_normal_anonymizer.py:134-165, :603-622) with the per-read encoding of
  ``AnonymizedRead.get_anonymized_fastq_record`` (anonymizer_methods.py:205-243):
  ``@name/1|2``, the upper-cased (masked) sequence, reverse-complemented for reverse reads,
  and the qualities printed in the BAM's stored order for every read (they are
  loaded forward-oriented and reversed once more on output). Bulk formatting runs on the
  GPU (``ganon_fastq_format_hip`` through the masking engine) or in libganon_host.so; the
  rare indel-edited records get their left-overs applied by ``native.fastq_edit``.
* the statistics file of ``AnonymizedVariantsStatistics.write_statistics`` (SR:175-242).
"""
from __future__ import annotations

import itertools
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import native
from .anonymizer_methods import MaskResult
from .variants import VariantType
from .io.bam import ReadTable
from .planner import Plan

OUTSIDE_WINDOWS = "outside_windows,-,-,-"
STAT_HEADER = ["#SEQ", "#FIRST", "#LAST", "#SNV", "#DEL", "#INS", "#DUP", "#INV", "#CNV", "#TRA", "#SGL"]


class _Pre:
    """A job's pre-formatted records (FastqFormatter.preformat): ``base`` (or None) the masked scope
    of every read's own copy, in row order (tumor then normal), its record at index row (+ the tumor
    rows); ``keys`` the sorted instance keys of the other records, at indices len(base) + rank;
    ``off`` / ``len`` each record's range in ``data`` (bytes, or a page-locked uint8 array)."""
    __slots__ = ("base", "keys", "off", "len", "data")

    def __init__(self, base, keys, off, ln, data):
        self.base, self.keys, self.off, self.len, self.data = base, keys, off, ln, data


class FastqFormatter:
    """Formats record runs through ``backend`` (a ``native.fastq_records`` dict -> bytes): the
    HIP formatter of the masking engine's device (``HipMasker.format_fastq``) in the product,
    the host library's ``ganon_fastq_format`` when no engine formatter is given."""

    def __init__(self, tables: Tuple[ReadTable, ReadTable], res: MaskResult, backend=None, device_backend=None):
        """``device_backend(recs, gen)``: formats from the engine's resident job batch while it still
        holds ``res`` (preformat only; None = not available)."""
        self.tables = tables
        self.res = res
        self.backend = backend or native.host_format_fastq
        self.device_backend = device_backend
        self._qual_bufs = [tables[0].qual, tables[1].qual]
        self._names = np.concatenate([np.asarray(tables[0].names_blob, np.uint8), np.asarray(tables[1].names_blob, np.uint8)])
        self._name_base = (0, len(tables[0].names_blob))
        self.edited: Dict[Tuple[int, int, int], bytes] = {}   # indel-edited records (write_fastqs)
        self.edited2: Dict[Tuple[int, int, int], bytes] = {}  # the same with the left-overs applied twice
        self._pre = None     # preformat()'s blob: _Pre
        self._left_keys = None   # sorted keys of the instances with left-over edits

    def _seq_bufs(self, masked: bool = True) -> list:
        """Sequence buffers: 0 = the masked output (fetched from the device on first use, only when
        some record reads it: ``masked``), 1 / 2 = the tumor / normal BAM bases."""
        m = self.res.seq_out if masked else np.zeros(1, np.uint8)
        return [m, self.tables[0].seq, self.tables[1].seq]

    @staticmethod
    def _key(ds, row, sc):
        return ((np.asarray(sc, np.int64) + 1) << 33) | (np.asarray(ds, np.int64) << 32) | np.asarray(row, np.int64)

    def records_arrays(self, ds: np.ndarray, row: np.ndarray, sc: np.ndarray, seq_bufs: bool = True) -> dict:
        """The record arrays of instances ``(dataset, row, write scope | -1)`` (``seq_bufs`` False:
        without the host sequence buffers, for the device formatter that reads them in place)."""
        n = len(ds)
        T, N = self.tables
        ds = np.asarray(ds, np.int64)
        row = np.asarray(row, np.int64)
        sc = np.asarray(sc, np.int64)
        t0 = ds == 0
        g = row + ds * T.n          # row in the concatenated tumor + normal columns
        pick = lambda f, dt: self._column(f, dt)[g]
        seq_sel = np.where(sc >= 0, 0, 1 + ds).astype(np.uint8)
        seq_off_t = pick("seq_off", np.int64)
        base = np.where(t0, self.res.seq_base[0], self.res.seq_base[1])
        byte_off = np.where(sc >= 0, base + seq_off_t, seq_off_t)
        if getattr(self.res, "dup_off", None) and n:   # a read masked in a further scope: that scope's copy
            dk, dv = self._dup_index()
            k = self._key(ds, row, sc)
            pos = np.minimum(np.searchsorted(dk, k), len(dk) - 1)
            hit = (dk[pos] == k) & (sc >= 0)
            byte_off = np.where(hit, dv[pos], byte_off)
        seq_len = pick("l_seq", np.int32)
        flag = pick("flag", np.int64)
        name_off = pick("name_off", np.int64) + np.where(t0, self._name_base[0], self._name_base[1])
        return {
            "seq_bufs": self._seq_bufs(bool((seq_sel == 0).any())) if seq_bufs else None, "seq_sel": seq_sel,
            "seq_nib_off": (2 * byte_off).astype(np.int64),
            "seq_len": seq_len, "reverse": pick("is_reverse", np.uint8),
            "qual_bufs": self._qual_bufs, "qual_sel": ds.astype(np.uint8), "qual_off": pick("qual_off", np.int64),
            "qual_len": seq_len.copy(), "qual_rev": np.zeros(n, np.uint8),   # stored order for every read (Q1)
            "names": self._names, "name_len": pick("name_len", np.int32), "name_off": name_off,
            "mate": np.where(flag & 0x40, 1, 2).astype(np.uint8),
        }

    def _column(self, f: str, dt) -> np.ndarray:
        """Column f of the tumor then the normal table, as dt (made once per job)."""
        cols = self.__dict__.setdefault("_cols", {})
        c = cols.get(f)
        if c is None:
            T, N = self.tables
            c = np.concatenate([np.asarray(getattr(T, f)), np.asarray(getattr(N, f))]).astype(dt, copy=False)
            cols[f] = c
        return c

    def _dup_index(self):
        """Sorted instance keys of the further masked copies and their byte offsets in seq_out."""
        if getattr(self, "_dup", None) is None:
            k = np.array(list(self.res.dup_off.keys()), np.int64).reshape(-1, 3)
            v = np.array(list(self.res.dup_off.values()), np.int64)
            key = self._key(k[:, 0], k[:, 1], k[:, 2])
            o = np.argsort(key)
            self._dup = (key[o], v[o])
        return self._dup

    def records(self, recs: Sequence[Tuple[int, int, int]]) -> dict:
        a = np.array(recs, np.int64).reshape(-1, 3)
        return self.records_arrays(a[:, 0], a[:, 1], a[:, 2])

    def _edited_index(self, ds, row, sc) -> np.ndarray:
        """Indices of the instances that carry left-over edits."""
        left = self.res.leftovers
        if not left or len(ds) == 0:
            return np.zeros(0, np.int64)
        if self._left_keys is None or len(self._left_keys) != len(left):
            a = np.array(list(left.keys()), np.int64).reshape(-1, 3)
            self._left_keys = np.sort(self._key(a[:, 0], a[:, 1], a[:, 2]))
        lk = self._left_keys
        k = self._key(ds, row, sc)
        pos = np.minimum(np.searchsorted(lk, k), len(lk) - 1)
        return np.nonzero(lk[pos] == k)[0]

    def _locate(self, ds, row, sc) -> Optional[np.ndarray]:
        """Indices in the pre-formatted blob of the records (ds, row, sc), or None when one is not in it.
        A read's own copy (its masked scope, or unmasked) is found by its row directly; other copies by
        a search of the few extra keys."""
        pre = self._pre
        if pre is None or len(ds) == 0:
            return None
        ds = np.asarray(ds, np.int64)
        row = np.asarray(row, np.int64)
        sc = np.asarray(sc, np.int64)
        if pre.base is None:
            k = self._key(ds, row, sc)
            pos = np.minimum(np.searchsorted(pre.keys, k), len(pre.keys) - 1)
            return pos if np.array_equal(pre.keys[pos], k) else None
        g = row + ds * self.tables[0].n
        idx = g.copy()
        miss = np.nonzero(pre.base[g] != sc)[0]
        if len(miss):
            if not len(pre.keys):
                return None
            k = self._key(ds[miss], row[miss], sc[miss])
            pos = np.minimum(np.searchsorted(pre.keys, k), len(pre.keys) - 1)
            if not np.array_equal(pre.keys[pos], k):
                return None
            idx[miss] = len(pre.base) + pos
        return idx

    def _native(self, ds, row, sc) -> bytes:
        if len(ds) == 0:
            return b""
        idx = self._locate(ds, row, sc)
        if idx is not None:      # slices of the job's pre-formatted records
            pre = self._pre
            return native.gather_ranges(pre.data, pre.off[idx], pre.len[idx])
        return self._format(ds, row, sc)

    def _format(self, ds, row, sc) -> bytes:
        try:
            return self.backend(self.records_arrays(ds, row, sc))
        except native.FastqBadRecord as e:
            d, r = int(ds[e.index]), int(row[e.index])
            raise TypeError(f"reverse read {self.tables[d].name(r)!r} has a base outside ACGTN: the "
                            "reference's reverse complement fails on it (SURVEY Q7)") from None

    def preformat(self, ds, row, sc, n_base: int = 0) -> bool:
        """Format the instances a job can write in ONE formatter call (the device round trip costs
        more than the bytes); later record runs are sliced out of it. A reverse read with a base
        outside ACGTN is left out (its error is raised only if it is written, as in the
        reference); after a few such reads the job formats on demand. True when every instance was
        formatted (no later record run needs the masked bases on the host).

        ``n_base``: the first n_base instances are every read of the tumor then the normal table once,
        in row order (Job._format_instances): they are formatted in that order and found by row, the
        rest are de-duplicated against them and searched by key (sorting every instance key of a job
        and searching them cost the 30x line ~0.8 CPU-s, tools/cpu_sampler.py)."""
        ds, row, sc = (np.asarray(x, np.int64) for x in (ds, row, sc))
        T, N = self.tables
        if n_base and n_base == T.n + N.n and len(ds) >= n_base and self._preformat_base(ds, row, sc, n_base):
            return True
        key = self._key(ds, row, sc)
        key, first = np.unique(key, return_index=True)
        ds, row, sc = ds[first], row[first], sc[first]
        n_all = len(ds)
        for _ in range(4):
            if len(ds) == 0:
                return n_all == 0
            try:
                data = None
                if self.device_backend is not None:   # the bases in place on the device
                    recs = self.records_arrays(ds, row, sc, seq_bufs=False)
                    recs["seq_base1"] = len(self.tables[0].seq)
                    data = self.device_backend(recs, self.res.device_gen)
                if data is None:
                    data = self.backend(self.records_arrays(ds, row, sc))
            except native.FastqBadRecord as e:
                keep = np.ones(len(ds), bool)
                keep[e.index] = False
                ds, row, sc, key = ds[keep], row[keep], sc[keep], key[keep]
                continue
            ln = self._plain_lengths(ds, row)
            self._pre = _Pre(None, key, np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.int64), ln, data)
            return len(ds) == n_all
        return False

    def _preformat_base(self, ds, row, sc, nb: int) -> bool:
        """preformat's structured case (no record refused by the formatter; else False, nothing kept)."""
        base_sc = sc[:nb]
        e_ds, e_row, e_sc = ds[nb:], row[nb:], sc[nb:]
        if len(e_ds):   # extras that are not a read's own copy, once each, by key
            own = base_sc[e_row + e_ds * self.tables[0].n] == e_sc
            e_ds, e_row, e_sc = e_ds[~own], e_row[~own], e_sc[~own]
            ekey, first = np.unique(self._key(e_ds, e_row, e_sc), return_index=True)
            e_ds, e_row, e_sc = e_ds[first], e_row[first], e_sc[first]
        else:
            ekey = np.zeros(0, np.int64)
        a_ds = np.concatenate([ds[:nb], e_ds])
        a_row = np.concatenate([row[:nb], e_row])
        a_sc = np.concatenate([base_sc, e_sc])
        try:
            data = None
            if self.device_backend is not None:
                recs = self.records_arrays(a_ds, a_row, a_sc, seq_bufs=False)
                recs["seq_base1"] = len(self.tables[0].seq)
                data = self.device_backend(recs, self.res.device_gen)
            if data is None:
                data = self.backend(self.records_arrays(a_ds, a_row, a_sc))
        except native.FastqBadRecord:
            return False
        ln = self._plain_lengths(a_ds, a_row)
        self._pre = _Pre(base_sc.copy(), ekey, np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.int64), ln, data)
        return True

    def edited_bytes(self, inst, reapply: int = 0) -> bytes:
        """Record of an instance with left-over edits, applied once or (reapply) twice (cached)."""
        cache = self.edited2 if reapply else self.edited
        b = cache.get(inst)
        if b is None:
            self.prepare_edited([inst], [reapply])
            b = cache[inst]
        return b

    def prepare_edited(self, insts: Sequence[Tuple[int, int, int]], reapply: Sequence[int]) -> None:
        """Format the edited records of ``insts`` not cached yet in one batch: the unedited records
        in one formatter call, the left-overs applied by ``native.fastq_edit`` (AM:178-203, 254-270)."""
        todo, seen = [], set()
        for inst, re_ in zip(insts, reapply):
            k = (inst, int(bool(re_)))
            if k not in seen and inst not in (self.edited2 if re_ else self.edited):
                seen.add(k)
                todo.append(k)
        if not todo:
            return
        a = np.array([x[0] for x in todo], np.int64).reshape(-1, 3)
        ds, row, sc = a[:, 0], a[:, 1], a[:, 2]
        plain = self._native(ds, row, sc)
        rec_off = np.concatenate([[0], np.cumsum(self._plain_lengths(ds, row))])
        T, N = self.tables
        rev = np.where(ds == 0, T.is_reverse[np.where(ds == 0, row, 0)] if T.n else 0,
                       N.is_reverse[np.where(ds == 1, row, 0)] if N.n else 0).astype(np.uint8)
        times = np.array([2 if r else 1 for _, r in todo], np.int32)
        edits, alleles, edit_off, allele_off, extra = [], [], [0], [0], 0
        left = self.res.leftovers
        for (inst, r) in todo:
            for irp, c in left[inst]:
                al = c.ref_allele.encode() if c.variant_type is VariantType.DEL else b""
                edits.append((irp, c.variant_type.value, c.length))
                alleles.append(al)
                allele_off.append(allele_off[-1] + len(al))
                extra += (2 if r else 1) * (len(al) + max(c.length, 0))
            edit_off.append(len(edits))
        try:
            data, lens = native.fastq_edit(plain, rec_off, rev, times, np.array(edit_off, np.int64),
                                           np.array(edits, np.int64).reshape(-1, 3), b"".join(alleles),
                                           np.array(allele_off, np.int64), len(plain) + extra)
        except native.FastqEditError as e:
            (d, r_, _), _r = todo[e.index]
            if e.code == 1:
                raise TypeError(f"reverse read {self.tables[d].name(r_)!r} has a base outside ACGTN (SURVEY Q7)") from None
            if e.code == 3:
                raise ValueError("cannot convert float NaN to integer") from None
            raise ValueError("Length of the modified qualities does not match the length of the modified sequence") from None
        off = np.concatenate([[0], np.cumsum(lens)]).tolist()
        for j, (inst, r) in enumerate(todo):
            (self.edited2 if r else self.edited)[inst] = data[off[j]:off[j + 1]]

    def _plain_lengths(self, ds, row) -> np.ndarray:
        T, N = self.tables
        r0, r1 = np.where(ds == 0, row, 0), np.where(ds == 1, row, 0)
        nl = np.where(ds == 0, T.name_len[r0] if T.n else 0, N.name_len[r1] if N.n else 0).astype(np.int64)
        ls = np.where(ds == 0, T.l_seq[r0] if T.n else 0, N.l_seq[r1] if N.n else 0).astype(np.int64)
        return nl + 8 + 2 * ls

    def unedited(self, insts: Sequence[Tuple[int, int, int]]) -> List[bytes]:
        """The records of ``insts`` before their left-over edits, one formatter call."""
        if not insts:
            return []
        a = np.array(insts, np.int64).reshape(-1, 3)
        data = self._native(a[:, 0], a[:, 1], a[:, 2])
        off = np.concatenate([[0], np.cumsum(self._plain_lengths(a[:, 0], a[:, 1]))]).tolist()
        return [data[off[j]:off[j + 1]] for j in range(len(a))]

    def format_arrays(self, ds: np.ndarray, row: np.ndarray, sc: np.ndarray, reapply=None) -> bytes:
        """Records in the given order: every unedited record in ONE formatter call, the rare
        indel-edited ones (variable length, formatted on the host; ``reapply``: left-overs applied
        twice) spliced in."""
        ds = np.asarray(ds, np.int64)
        row = np.asarray(row, np.int64)
        sc = np.asarray(sc, np.int64)
        reapply = np.zeros(len(ds), np.int64) if reapply is None else np.asarray(reapply, np.int64)
        ed = self._edited_index(ds, row, sc)
        if len(ed) == 0:
            return self._native(ds, row, sc)
        keep = np.ones(len(ds), bool)
        keep[ed] = False
        insts = list(zip(ds[ed].tolist(), row[ed].tolist(), sc[ed].tolist()))
        re_ = reapply[ed].tolist()
        self.prepare_edited(insts, re_)
        eb = [(self.edited2 if r else self.edited)[inst] for inst, r in zip(insts, re_)]
        # ONE copy of every record into its place: the unedited ones straight out of the job's
        # pre-formatted blob (or of one formatter call), the edited ones out of their small
        # concatenation (slicing and joining the whole output in Python copied it twice more: the
        # writer thread's largest CPU cost at 30x, tools/cpu_sampler.py)
        sel = np.zeros(len(ds), np.uint8)
        sel[ed] = 1
        off = np.zeros(len(ds), np.int64)
        ln = np.zeros(len(ds), np.int64)
        e_len = np.array([len(b) for b in eb], np.int64)
        off[ed] = np.concatenate([[0], np.cumsum(e_len)[:-1]])
        ln[ed] = e_len
        kd, kr, ks = ds[keep], row[keep], sc[keep]
        src, k_off, k_len = self._ranges(kd, kr, ks)
        off[keep] = k_off
        ln[keep] = k_len
        return native.gather_ranges2(src, b"".join(eb), sel, off, ln)

    def _ranges(self, ds, row, sc):
        """(source bytes, offsets, lengths) of the records of ``ds, row, sc`` (unedited): ranges of
        the pre-formatted blob when it holds every one, else one formatter call's output."""
        idx = self._locate(ds, row, sc)
        if idx is not None:
            pre = self._pre
            return pre.data, pre.off[idx], pre.len[idx]
        data = self._format(ds, row, sc) if len(ds) else b""
        ln = self._plain_lengths(ds, row)
        return data, np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.int64) if len(ds) else ln, ln

    def format(self, recs: Sequence[Tuple[int, int, int]], reapply=None) -> bytes:
        a = np.array(recs, np.int64).reshape(-1, 3)
        return self.format_arrays(a[:, 0], a[:, 1], a[:, 2], reapply)

    def record_lengths(self, ds, row, sc, reapply=None) -> np.ndarray:
        """Byte length of each record (edited ones included)."""
        T, N = self.tables
        ds = np.asarray(ds, np.int64)
        row = np.asarray(row, np.int64)
        sc = np.asarray(sc, np.int64)
        r0, r1 = np.where(ds == 0, row, 0), np.where(ds == 1, row, 0)
        nl = np.where(ds == 0, T.name_len[r0] if T.n else 0, N.name_len[r1] if N.n else 0).astype(np.int64)
        ls = np.where(ds == 0, T.l_seq[r0] if T.n else 0, N.l_seq[r1] if N.n else 0).astype(np.int64)
        out = nl + 8 + 2 * ls
        ed = self._edited_index(ds, row, sc)
        if len(ed):
            re_ = np.zeros(len(ds), np.int64) if reapply is None else np.asarray(reapply, np.int64)
            insts = list(zip(ds[ed].tolist(), row[ed].tolist(), sc[ed].tolist()))
            rl = re_[ed].tolist()
            self.prepare_edited(insts, rl)
            out[ed] = [len((self.edited2 if r else self.edited)[inst]) for inst, r in zip(insts, rl)]
        return out


TEXT_CHUNK = 8192  # TextIOWrapper._CHUNK_SIZE of CPython


class AppendHandle:
    """One ``open(path, 'a')`` text handle of CPython (TextIOWrapper over a BufferedWriter
    of ``block`` = st_blksize bytes) writing into a shared O_APPEND file: records become
    visible in the file only when a flush reaches the raw layer. The reference opens a
    fresh set of such handles in every scope / section function (SR:297-299, :516-518,
    :564-566), so nested handles interleave in the files at flush granularity."""

    def __init__(self, sink: list, block: int):
        self.sink = sink
        self.block = block
        self.pending: list = []
        self.pending_len = 0
        self.buf: list = []
        self.buf_len = 0

    def write(self, rec, n: int) -> None:
        # textio.c write(): never concatenate more than chunk_size, flush once >= chunk_size
        if self.pending_len + n > TEXT_CHUNK:
            self._text_flush()
            self.pending = [rec]
            self.pending_len = n
        else:
            self.pending.append(rec)
            self.pending_len += n
        if self.pending_len >= TEXT_CHUNK:
            self._text_flush()

    def _text_flush(self) -> None:
        if not self.pending:
            return
        recs, n = self.pending, self.pending_len
        self.pending, self.pending_len = [], 0
        # bufferedio.c write(): buffer if it fits, else flush the buffer and write through
        if n <= self.block - self.buf_len:
            self.buf.extend(recs)
            self.buf_len += n
            return
        self._raw_flush()
        if n > self.block:
            self.sink.extend(recs)
        else:
            self.buf, self.buf_len = list(recs), n

    def _raw_flush(self) -> None:
        if self.buf:
            self.sink.extend(self.buf)
            self.buf, self.buf_len = [], 0

    def close(self) -> None:
        self._text_flush()
        self._raw_flush()


def replay_io(io_log, rec_len, block: int) -> Dict[Tuple[int, int], list]:
    """Order in which the records of each output file reach the disk."""
    files: Dict[Tuple[int, int], list] = {(d, s): [] for d in (0, 1) for s in (0, 1)}
    handles: Dict[int, Dict[Tuple[int, int], AppendHandle]] = {}
    for ev in io_log:
        if ev[0] == "open":
            handles[ev[1]] = {k: AppendHandle(files[k], block) for k in files}
        elif ev[0] == "write":
            inst = ev[4]
            handles[ev[1]][(ev[2], ev[3])].write(inst, rec_len(inst))
        else:
            for h in handles.pop(ev[1]).values():
                h.close()
    if handles:
        raise RuntimeError("unclosed handles in the I/O log")
    return files


def io_block_size(directory: str) -> int:
    """st_blksize CPython would use for a buffered file in ``directory`` (override with the
    environment variable GANON_IO_BLOCK to reproduce files written on another filesystem)."""
    import os
    if os.environ.get("GANON_IO_BLOCK"):
        return int(os.environ["GANON_IO_BLOCK"])
    try:
        st = os.stat(directory).st_blksize
        return st if st > 1 else 8192
    except OSError:
        return 8192


def write_fastqs(plan: Plan, res: MaskResult, tables, prefixes: Tuple[str, str],
                 block_size: int = None, backend=None) -> Dict[str, int]:
    import os
    fmt = FastqFormatter(tables, res, backend)
    if block_size is None:
        block_size = io_block_size(os.path.dirname(os.path.abspath(prefixes[0])))
    ev, rows = plan.io_arrays()
    ids = ev[:, 4].astype(np.int64)
    isc = ev[:, 5].astype(np.int64)
    wr = ev[:, 0] == 1
    reapply = np.where(wr, ev[:, 6], 0).astype(np.int64)
    rec_len = np.zeros(len(ev), np.int64)
    wi = np.nonzero(wr)[0]
    rec_len[wi] = fmt.record_lengths(ids[wi], rows[wi], isc[wi], reapply[wi])
    order = native.io_replay(ev, rec_len, block_size)
    sizes = {}
    for ds in (0, 1):
        for slot in (0, 1):
            path = f"{prefixes[ds]}.{slot + 1}.fastq"
            e = order[2 * ds + slot]
            data = fmt.format_arrays(ids[e], rows[e], isc[e], reapply[e])
            with open(path, "wb") as fh:
                fh.write(data)
            sizes[path] = len(data)
    if plan.write_single_end:
        for ds in (0, 1):
            path = f"{prefixes[ds]}.single_end.fastq"
            data = fmt.format(plan.single_end[ds], plan.single_reapply[ds])
            with open(path, "wb") as fh:
                fh.write(data)
            sizes[path] = len(data)
    return sizes


def statistics_rows(plan: Plan, res: MaskResult) -> Dict[str, List[int]]:
    """Replay the recorder events (SR:175-210) with the per-scope counts."""
    from .variants import VariantType
    rows: Dict[str, List[int]] = {OUTSIDE_WINDOWS: [0] * 8}
    current = ""
    for kind, val in plan.stats_events:
        if kind == "window":
            rows[val] = [0] * 8
            current = val
        elif kind == "outside":
            current = OUTSIDE_WINDOWS
        else:
            s = int(val)
            ic = res.scope_indel_counts.get(s, {})
            add = [int(res.scope_snv_calls[s]), ic.get(VariantType.DEL, 0), ic.get(VariantType.INS, 0)]
            if any(add):
                row = rows[current]
                for k in range(3):
                    row[k] += add[k]
    return rows


def write_statistics(path: str, rows: Dict[str, List[int]]) -> None:
    """AnonymizedVariantsStatistics.write_statistics (SR:212-242)."""
    cols = [[] for _ in range(8)]
    with open(path, "w") as fh:
        fh.write("\t".join(STAT_HEADER) + "\n")
        for key, counts in rows.items():
            fields = key.split(",")[:-1]
            fh.write("\t".join(map(str, itertools.chain(fields, counts))) + "\n")
            for k, v in enumerate(counts):
                cols[k].append(v)
        fh.write("### Overall statistics:\n")
        fh.write("\t".join(STAT_HEADER[3:]) + "\n")
        arrays = [np.array(c, dtype=np.int64) for c in cols]
        for stat in ("total_counts", "average_counts", "median_counts", "max_counts", "min_counts"):
            fh.write(f"#{stat}\t")
            if stat == "total_counts":
                vals = [np.sum(a) for a in arrays]
            elif stat == "average_counts":
                vals = [a.mean() for a in arrays]
            elif stat == "median_counts":
                vals = [np.median(a) for a in arrays]
            elif stat == "max_counts":
                vals = [a.max() for a in arrays]
            else:
                vals = [a.min() for a in arrays]
            fh.write("\t".join(map(str, vals)) + "\n")
