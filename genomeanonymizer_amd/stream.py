"""Bounded-memory, contig-sharded anonymization of one tumor/normal pair.

The reference walks a sample section by section through region queries
(``anonymize_genome``, short_read_tumor_normal_anonymizer.py:625-760) and never holds a BAM in
memory; its only state that outlives a contig is the pairing state — ``to_pair_anonymized_reads``,
``written_read_ids`` (SR:134-165, :304-406, AM:351-389) — and the end-of-sample passes
(``pair_unmapped_mates`` SR:561-600, ``write_single_end_reads`` SR:603-622). This module runs the
same flow one FASTA contig ("job") at a time:

1. decode the job's records only (``io.bam.BamReader``: .bai seek or forward stream);
2. plan it in contig mode (``planner.ContigPlanner``): every name whose records all lie on this
   contig is planned exactly; operations on "cross" names (a record whose mate is on another
   sequence, or unplaced) become placeholder events;
3. mask its scopes in one device batch (``CompleteGermlineAnonymizer``: HIP SNV + indel tally);
4. resolve the placeholders, contig after contig in FASTA order, against the sample-wide pairing
   state (``native.Resolver``, C++), and carry the records those names may still need (their
   formatted FASTQ bytes) to later contigs;
5. replay the job's I/O log (the reference's per-section append handles) and write its
   bytes at the job's offset of each output file; the files grow in contig order.

Steps 1-3 and the formatting run on the job's owner rank; step 4 runs in a coordinator thread of
rank 0 (``_Coordinator``) that takes the contigs in FASTA order as their exports arrive and answers
the owner with its resolved writes and its offsets in the files; the owner assembles and writes its
bytes (step 5) itself. Multi-GPU (distributed.py): the contigs are sharded over the
ranks (round-robin or LPT), each rank works through its own contigs with no lock-step; only the
cross-contig pairing state and the records it may write travel, to rank 0 and back to the owner.
No data-path collective touches the masked bases. Memory: GANON_PENDING jobs per rank waiting for
their resolution plus the prefetched ones, and the carried records of names still unpaired.
"""
from __future__ import annotations

import dataclasses
import os
import threading
import time
from concurrent.futures import Future, ThreadPoolExecutor, wait
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import native
from . import objects
from .anonymizer_methods import CompleteGermlineAnonymizer, MaskResult, build_batch
from .io.bam import BamReader, ReadTable
from .io.fasta import FastaRef
from .planner import ContigPlanner, Plan, Window, get_genome_sections
from . import writer as _writer
from .writer import OUTSIDE_WINDOWS, FastqFormatter, statistics_rows, write_statistics

Key = Tuple[int, int, int, int, int]   # (job, dataset, scope, row, reapply)


def _names(table: ReadTable, rows: np.ndarray) -> List[bytes]:
    nb = table.names_blob
    return [nb[o:o + n].tobytes() for o, n in zip(table.name_off[rows].tolist(), table.name_len[rows].tolist())]


_NK = (np.uint64(0x9E3779B97F4A7C15), np.uint64(0xC2B2AE3D27D4EB4F), np.uint64(0x165667B19E3779F9))


def _name_keys(blob: np.ndarray, off: np.ndarray, ln: np.ndarray) -> np.ndarray:
    """A 64-bit key per name (blob[off:off + ln]): its length with its first and last eight bytes
    (shorter names: their bytes, zero-padded). Equal names have equal keys; the rare unequal names with
    equal keys are told apart by the caller's byte comparison."""
    buf = np.zeros(len(blob) + 16, np.uint8)
    buf[:len(blob)] = blob
    off = off.astype(np.int64)
    ln = ln.astype(np.int64)
    idx = np.arange(8, dtype=np.int64)
    first = buf[off[:, None] + idx]
    first[idx[None, :] >= ln[:, None]] = 0
    last = buf[np.maximum(off, off + ln - 8)[:, None] + idx]
    last[idx[None, :] >= ln[:, None]] = 0
    w0 = first.view(np.uint64).ravel()
    w1 = last.view(np.uint64).ravel()
    with np.errstate(over="ignore"):
        return (w0 * _NK[0]) ^ (w1 * _NK[1]) ^ (ln.astype(np.uint64) * _NK[2])


def _names_present(table: ReadTable, names: Sequence[bytes]) -> set:
    """The names of ``names`` that some record of ``table`` carries: one vectorized pass over the
    table's names (keys, then a byte comparison of the key hits) instead of a search of the names
    blob per name (5,362 blob searches took 14.9 s of a 2-rank CPU run's 22.8 s, `redo_needed`)."""
    if not len(names) or table.n == 0:
        return set()
    cand = list(names)
    cb = np.frombuffer(b"".join(cand), np.uint8)
    cl = np.array([len(x) for x in cand], np.int64)
    co = np.concatenate([[0], np.cumsum(cl)[:-1]]).astype(np.int64)
    ck = _name_keys(cb, co, cl)
    tk = _name_keys(table.names_blob, table.name_off, table.name_len)
    hit = np.isin(ck, tk)
    if not hit.any():
        return set()
    order = np.argsort(tk, kind="stable")
    sk = tk[order]
    nb = table.names_blob
    out = set()
    for i in np.nonzero(hit)[0].tolist():
        lo, hi = np.searchsorted(sk, ck[i], "left"), np.searchsorted(sk, ck[i], "right")
        for r in order[lo:hi].tolist():
            o, n = int(table.name_off[r]), int(table.name_len[r])
            if nb[o:o + n].tobytes() == cand[i]:
                out.add(cand[i])
                break
    return out


def _names_ds(tables, ds: np.ndarray, rows: np.ndarray) -> List[bytes]:
    out: List[bytes] = [b""] * len(ds)
    for d in (0, 1):
        sel = np.nonzero(ds == d)[0]
        for i, nm in zip(sel.tolist(), _names(tables[d], rows[sel])):
            out[i] = nm
    return out


def _pwrite_all(fd: int, data, offset: int) -> None:
    """Write ``data`` (a bytes-like object, or a list of them written back to back with pwritev, no
    join) at ``offset`` until every byte is written (a single call may write fewer bytes)."""
    parts = [memoryview(x).cast("B") for x in (data if isinstance(data, list) else [data])]
    parts = [x for x in parts if len(x)]
    while parts:
        batch = parts[:512]   # (IOV_MAX is 1024)
        n = os.pwritev(fd, batch, offset)
        if n <= 0:
            raise OSError(f"pwritev wrote nothing at offset {offset}")
        offset += n
        k = 0
        while k < len(batch) and n >= len(batch[k]):
            n -= len(batch[k])
            k += 1
        parts = ([batch[k][n:]] if k < len(batch) else []) + batch[k + 1:] + parts[len(batch):]


@dataclasses.dataclass(frozen=True)
class JobSpec:
    """One unit of the streamed sample: a FASTA contig, or a run of consecutive sections of it (job
    mode). The reference's unit of work is the section (anonymize_genome, SR:660-697); a run of
    sections is planned from the records overlapping ``region``, the union of its sections' region
    queries (the jobs of a contig tile it)."""
    index: int
    contig: str
    cidx: int                                   # FASTA index of the contig
    sections: Optional[Tuple[int, int]] = None  # [first, end) in the contig's section order; None = all
    region: Optional[Tuple[int, int]] = None    # [beg, end), 0-based: the records decoded
    length: int = 0                             # bases (sharding weight)

    def label(self) -> str:
        return self.contig if self.region is None else f"{self.contig}:{self.region[0]}-{self.region[1]}"


DECODE_TIMES = {"decode_s": 0.0}   # per process (one decode thread per streamed run)
_SAMPLE_POOL: list = []


def _sample_pool():
    """Two threads reading a job's tumor and normal BAM at once (one per process)."""
    if not _SAMPLE_POOL:
        _SAMPLE_POOL.append(ThreadPoolExecutor(2, thread_name_prefix="ganon-sample"))
    return _SAMPLE_POOL[0]
_INFLATERS: Dict[Tuple[int, int, int], "native.GpuInflater"] = {}   # (device, min blocks, sample) -> inflater


def _map_samples(fn, readers) -> list:
    """``fn`` over the samples' readers on the sample pool. Every call finishes before the first error
    is raised: a failing sample must not leave the other sample's native read running inside a reader
    (or an inflater context) that the failure path then closes or hands to the next run."""
    futs = [_sample_pool().submit(fn, r) for r in readers]
    wait(futs)
    return [f.result() for f in futs]


def _close_all(objs) -> None:
    for o in objs:
        o.close()


def auto_job_bp(genome_len: int, world: int) -> int:
    """Job size when GANON_JOB_BP is unset: 4 Mb, or less so that each of the ``world`` ranks gets
    about GANON_JOBS_PER_RANK (3) jobs, but at least 256 kb. (The 30x chromosome-scale line, 8
    ranks: 3 jobs per rank 6.67e6 reads/s, 6 6.42e6, 12 6.55e6 — more jobs add plan waits for the
    decode frontier of the jobs before them; the 24-contig line keeps one job per 2 Mb contig.)"""
    per_rank = max(1, int(os.environ.get("GANON_JOBS_PER_RANK", "3")))
    return int(min(4_000_000, max(256_000, genome_len // max(1, per_rank * world))))


def job_targets(genome_len: int, job_bp: int, world: int, taper: float):
    """Target length of job k (a function): ``job_bp`` each, except that with several ranks the first
    and the last ``world`` jobs — every rank's first and last job under round-robin ownership — are
    ``taper`` x shorter and the jobs between them longer by what those give up. A rank's first job's
    decode + plan is waited for with nothing to overlap it, and its last job's format + write drains
    alone: shorter ones shorten both ends of every rank's pipeline (GANON_JOB_TAPER, default 1 = equal
    jobs). Measured on the 30x line (8 ranks, 3 jobs each, round 6): equal jobs 1.14e7 reads/s, taper
    0.5 9.8e6, 0.7 1.0e7 — the longer middle jobs put their decode on the critical path instead."""
    n = max(1, int(round(genome_len / max(1, job_bp))))
    if world <= 1 or taper >= 1.0 or n < 3 * world:
        return lambda k: job_bp
    small = max(1, int(job_bp * taper))
    mid = max(small, (genome_len - 2 * world * small) // max(1, n - 2 * world))
    return lambda k: small if k < world or k >= n - world else mid


def plan_jobs(fasta: FastaRef, windows: Sequence[Window], job_bp: int, indexed: bool, target=None) -> List[JobSpec]:
    """The sample's jobs in FASTA then section order. ``job_bp`` > 0 and indexed BAMs: each contig
    longer than job_bp is cut at section boundaries into runs of about job_bp bases (a short tail
    joins the run before it); else one job per contig. A contig whose sections do not tile it (the
    reference's region errors) stays whole."""
    refs, lens = list(fasta.references), list(fasta.lengths)
    if job_bp <= 0 or not indexed:
        return [JobSpec(i, c, i, None, None, int(L)) for i, (c, L) in enumerate(zip(refs, lens))]
    by: Dict[str, List[Window]] = {c: [] for c in refs}
    for w in get_genome_sections(windows, fasta):
        by[w.sequence].append(w)
    out: List[JobSpec] = []
    for ci, (c, L) in enumerate(zip(refs, lens)):
        ss = by[c]
        tiles = (len(ss) > 1 and ss[0].first == 1 and ss[-1].last == L - 1 and
                 all(w.first <= w.last for w in ss) and
                 all(ss[k].first == ss[k - 1].last + 1 for k in range(1, len(ss))))
        cuts = [0]
        tgt = target or (lambda k: job_bp)     # (job_targets: the k-th job's length)
        if tiles and L > job_bp:
            acc = 0
            for k, w in enumerate(ss):
                acc += w.last - w.first + 1
                if acc >= tgt(len(out) + len(cuts) - 1) and k + 1 < len(ss):
                    cuts.append(k + 1)
                    acc = 0
            if len(cuts) > 1 and ss[-1].last - ss[cuts[-1]].first + 1 < tgt(len(out) + len(cuts) - 1) // 2:
                cuts.pop()
        if len(cuts) == 1:
            out.append(JobSpec(len(out), c, ci, None, None, int(L)))
            continue
        cuts.append(len(ss))
        for a, b in zip(cuts[:-1], cuts[1:]):
            lo = 0 if a == 0 else ss[a].first - 1
            hi = int(L) if b == len(ss) else ss[b - 1].last
            out.append(JobSpec(len(out), c, ci, (a, b), (lo, hi), hi - lo))
    return out


def decode_job(readers, spec: JobSpec, secondaries: "Optional[SecondaryIndex]" = None):
    """The job's records of both BAMs (io.bam.BamReader.contig, or .region in job mode); with
    ``secondaries``, the secondary alignments among them whose mate another job reads are published
    there before the tables are handed on (the decode runs in job order, so every later job's plan
    sees them)."""
    t0 = time.time()
    # the two samples' BAMs are read at once (round 5: the decode thread bounded the 30x line's ranks;
    # each reader has its own threads and, with GPU inflate, its own inflater context; the native
    # reads drop the GIL)
    both = _map_samples if len(readers) == 2 and os.environ.get("GANON_DECODE_PAIR", "1") != "0" else map
    if spec.region is None:
        tables = tuple(both(lambda r: r.contig(r.tid_of(spec.contig)), readers))
    else:
        # the scopes of a gap section pile up the union of its read clusters (pileup_io.pyx:124-298,
        # SR:523-534), which reaches past the job's range by a read's extent: the records overlapping
        # [lo, hi) fix the range the job's pileups can touch; read with a margin, again if it was short
        lo, hi = spec.region
        m = int(os.environ.get("GANON_JOB_MARGIN", "4096"))
        tables = tuple(both(lambda r: r.region(r.tid_of(spec.contig), max(0, lo - m), hi + m), readers))
        need_lo, need_hi = lo, hi
        for t in tables:
            if t.n:
                sel = (np.asarray(t.pos) < hi) & (np.asarray(t.end) > lo) & ((np.asarray(t.flag) & 4) == 0)
                if sel.any():
                    need_lo = min(need_lo, int(np.asarray(t.pos)[sel].min()))
                    need_hi = max(need_hi, int(np.asarray(t.end)[sel].max()))
        if need_lo < lo - m or need_hi > hi + m:
            tables = tuple(both(lambda r: r.region(r.tid_of(spec.contig), need_lo, need_hi), readers))
    if secondaries is not None:
        secondaries.publish(spec.index, secondaries.scan(tables, spec.index)[0])
    DECODE_TIMES["decode_s"] += time.time() - t0   # (the decode thread's busy time)
    return tables


def content_ids(table: ReadTable, rows: np.ndarray) -> np.ndarray:
    """A record's identity for the supplementary records an object recorded
    (get_supplementary_hash_from_aln: reference, start, CIGAR, sequence, qualities, flag; AM:61-62):
    a 63-bit mix of its sequence, position, flag, length and CIGAR words, so that a record two jobs'
    tables both hold is one record (vectorised)."""
    rows = np.asarray(rows, np.int64)
    if not len(rows):
        return np.zeros(0, np.int64)
    M = np.uint64(0xFFFFFFFFFFFFFFFF)

    def mix(x):
        x = (x + np.uint64(0x9E3779B97F4A7C15)) & M
        x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M
        x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M
        return x ^ (x >> np.uint64(31))

    with np.errstate(over="ignore"):
        u = lambda a: np.asarray(a, np.int64).astype(np.uint64)
        h = mix(u(table.tid[rows]) << np.uint64(32) | (u(table.pos[rows]) & np.uint64(0xFFFFFFFF)))
        h = mix(h ^ (u(table.flag[rows]) << np.uint64(40) | u(table.l_seq[rows])))
        nc = np.asarray(table.n_cigar[rows], np.int64)
        co = np.asarray(table.cig_off[rows], np.int64)
        tot = int(nc.sum())
        if tot:
            idx = np.repeat(co - np.concatenate([[0], np.cumsum(nc)[:-1]]), nc) + np.arange(tot)
            w = mix(u(table.cigar[idx]) + u(np.arange(tot) - np.repeat(np.concatenate([[0], np.cumsum(nc)[:-1]]), nc)))
            acc = np.zeros(len(rows), np.uint64)
            np.add.at(acc, np.repeat(np.arange(len(rows)), nc), w)
            h = mix(h ^ acc)
    return (h >> np.uint64(1)).astype(np.int64)


class SecondaryIndex:
    """Secondary alignments whose mate another job reads (flag 0x100; the mate on another contig,
    or in job mode in another run of sections). Their name's other records say nothing of them, so
    the job holding the mate plans that name locally unless told (the reference keeps one pairing
    state per name for the whole sample, SR:134-165, AM:320-389): a job planned after such a
    secondary's job plans the name as a cross name (``forced_for``); a job planned before it wrote
    the name itself, which the coordinator marks in the resolver when it meets the secondary
    (``ganon_resolver_mark_written``). The coordinator checks every export against the secondaries
    of the jobs before it and asks the owner to plan a job again when one was published too late
    (another rank decoded it)."""

    def __init__(self, readers, jobs: Sequence[JobSpec]):
        contigs: Dict[str, int] = {}
        for j in jobs:
            contigs.setdefault(j.contig, j.cidx)
        # FASTA contig of every BAM tid, per sample (-1: not a FASTA contig)
        self.contig_of_tid = [np.array([contigs.get(n, -1) for n in r.ref_names] + [-1], np.int64) for r in readers]
        n_c = max(contigs.values()) + 1 if contigs else 0
        self.starts: List[np.ndarray] = [np.zeros(0, np.int64)] * n_c   # per contig: its jobs' region starts
        self.ids: List[np.ndarray] = [np.zeros(0, np.int64)] * n_c
        by_c: Dict[int, list] = {}   # one pass over the jobs (a scaffold-level FASTA has ~1e5 contigs)
        for j in jobs:
            by_c.setdefault(j.cidx, []).append(j)
        for c, js in by_c.items():
            self.starts[c] = np.array([j.region[0] if j.region else 0 for j in js], np.int64)
            self.ids[c] = np.array([j.index for j in js], np.int64)
        self.lock = threading.Lock()
        self.by_mate: Dict[int, Dict[bytes, int]] = {}   # mate job -> name -> lowest source job
        # several ranks: distributed.SecondaryExchange — every job's secondaries reach every later
        # job's plan whichever rank decodes them (a plan waits until every earlier job is decoded)
        self.remote = None
        # speculative plans checked against their permit, and how many had to be planned again:
        # when at least half of them were (secondaries common in the data), later jobs wait for
        # their permit before planning instead (GANON_SPEC_PLAN=1 / 0 forces either way)
        self.spec_checked = 0
        self.spec_redone = 0

    def speculate(self) -> bool:
        """Plan the next job at once with the names known here (True) or wait for its permit."""
        mode = os.environ.get("GANON_SPEC_PLAN", "auto")
        if mode in ("0", "1"):
            return mode == "1"
        with self.lock:
            return self.spec_checked < 2 or 2 * self.spec_redone < self.spec_checked

    def note_spec(self, redone: bool) -> None:
        with self.lock:
            self.spec_checked += 1
            self.spec_redone += bool(redone)

    def job_of(self, ds: int, tid: np.ndarray, pos: np.ndarray) -> np.ndarray:
        """The job reading position pos of BAM tid (-1: none)."""
        ct = self.contig_of_tid[ds]
        c = ct[np.where((tid >= 0) & (tid < len(ct) - 1), tid, len(ct) - 1)]
        out = np.full(len(tid), -1, np.int64)
        for ci in np.unique(c[c >= 0]).tolist():
            sel = np.nonzero(c == ci)[0]
            k = np.searchsorted(self.starts[ci], pos[sel], side="right") - 1
            out[sel] = self.ids[ci][np.maximum(k, 0)]
        return out

    def scan(self, tables, job: int) -> Tuple[List[Tuple[bytes, int]], List[bytes]]:
        """(name, mate job) of each secondary alignment of ``tables`` whose mate another job reads,
        and the names of all its secondary alignments (complex names of the job already)."""
        out: List[Tuple[bytes, int]] = []
        own: List[bytes] = []
        for d, t in enumerate(tables):
            if not t.n:
                continue
            sec = np.nonzero((t.flag & 0x100) != 0)[0]
            if not len(sec):
                continue
            own.extend(_names(t, sec))
            sel = sec[np.asarray(t.mate_tid[sec]) >= 0]
            if not len(sel):
                continue
            mj = self.job_of(d, np.asarray(t.mate_tid[sel], np.int64), np.asarray(t.mate_pos[sel], np.int64))
            keep = (mj >= 0) & (mj != job)
            for nm, j in zip(_names(t, sel[keep]), mj[keep].tolist()):
                out.append((nm, int(j)))
        return out, own

    def publish(self, job: int, pairs: List[Tuple[bytes, int]]) -> None:
        with self.lock:
            for nm, mj in pairs:
                d = self.by_mate.setdefault(mj, {})
                if d.get(nm, 1 << 62) > job:
                    d[nm] = job
        if self.remote is not None:
            self.remote.report(job, pairs)

    def forced_local(self, job: int) -> List[bytes]:
        """The names ``forced_for`` would return that this rank knows already (no wait): a
        speculative plan's, checked against the permit before its export (the stream loop)."""
        with self.lock:
            return sorted({nm for nm, src in self.by_mate.get(job, {}).items() if src < job})

    def forced_for(self, job: int) -> List[bytes]:
        """Names of published secondaries of earlier jobs whose mate this job reads (several ranks:
        once every earlier job is decoded, on any rank)."""
        remote = self.remote.permit(job) if self.remote is not None else []
        with self.lock:
            return sorted(set(remote) | {nm for nm, src in self.by_mate.get(job, {}).items() if src < job})


class JobPrep:
    """The host stage of one contig before the device: decode (io.bam), plan (ganon_plan_run), the
    masked instance of every read and the device batch (anonymizer_methods.build_batch). The
    streamed loop runs it for the next contig in a prefetch thread while the current one masks,
    formats and writes (the BGZF inflate and the planner are native and drop the GIL)."""

    def __init__(self, spec: JobSpec, readers, fasta: FastaRef, windows: Sequence[Window], tables=None,
                 secondaries: Optional[SecondaryIndex] = None, force: Optional[Sequence[bytes]] = None):
        """``tables``: the decoded records when a decode thread produced them (a Future);
        ``secondaries``: the run's SecondaryIndex; ``force``: names to plan as cross names (a job
        planned again), else the secondaries published for this job."""
        self.spec = spec
        self.job = spec.index
        self.contig = spec.label()
        t0 = time.time()
        self.tables = decode_job(readers, spec, secondaries) if tables is None else tables.result()
        t1 = time.time()
        # several ranks: plan at once with the names known here, and take the permit — every
        # earlier job decoded, on any rank — only before the export (stream loop: a job whose
        # permitted names change its plan is planned again there). Waiting for it here put the decode
        # frontier of all earlier jobs on every plan's critical path (up to 0.6 s per rank on the 30x
        # line's later ranks, with no secondary in the data).
        self.speculative = force is None and secondaries is not None and secondaries.remote is not None and \
            secondaries.speculate()
        if force is None:
            force = (secondaries.forced_local(self.job) if self.speculative else secondaries.forced_for(self.job)) \
                if secondaries is not None else []
        self.forced = sorted(set(force))
        self.offsec, self.own_sec = secondaries.scan(self.tables, self.job) if secondaries is not None else ([], [])
        job_arg = None if spec.sections is None else (spec.sections[0], spec.sections[1], spec.region[0], spec.region[1])
        self.planner = ContigPlanner(self.tables[0], self.tables[1], fasta, windows, spec.cidx, self.forced, job_arg)
        self.plan: Plan = self.planner.run()
        ex = self.planner.contig_exports
        t2 = time.time()
        ev, rows = self.plan.io_arrays()
        self.events, self.event_rows = ev, rows
        self.ph = np.nonzero(ev[:, 0] >= 3)[0]
        self.plain_ph = self.ph[ev[self.ph, 0] <= 5]   # kinds 6 / 7 carry objects of complex names
        self.left = ex["left"]
        self.cand = ex["cand"]
        self.objs, self.obj_rows = ex["objs"], ex["obj_rows"]
        self.masked_scope = [np.full(t.n, -1, np.int64) for t in self.tables]
        self.written = self._mask_instances()
        self.batch = build_batch(self.plan, self.tables, fasta, None, self.written)
        self.prep_timing = (t1 - t0, t2 - t1, time.time() - t2)

    # -- which masked copy of each read the device produces --------------------------------------
    def _mask_instances(self):
        """Every masked copy a write of this job or of the sample-wide resolution may name: each
        read's local write, its placeholders and unwritten-pair entries (a cross name's read met in
        two scopes of the contig: one copy per scope, build_batch). ``masked_scope`` per read is the
        first of them (its local write, else its first placeholder, else its unwritten-pair entry):
        the copy formatted when nothing names another."""
        ev, rows = self.events, self.event_rows
        parts = []
        w = ev[:, 0] == 1
        parts.append((ev[w, 4].astype(np.int64), rows[w], ev[w, 5].astype(np.int64)))
        p = self.plain_ph
        parts.append((ev[p, 4].astype(np.int64), rows[p], ev[p, 5].astype(np.int64)))
        L = self.left
        for s in (0, 1):
            h = L[:, 1 + 4 * s] == 1 if len(L) else np.zeros(0, bool)
            parts.append((L[h, 2 + 4 * s], L[h, 4 + 4 * s], L[h, 3 + 4 * s]))
        ds = np.concatenate([x[0] for x in parts]).astype(np.int64)
        rw = np.concatenate([x[1] for x in parts]).astype(np.int64)
        sc = np.concatenate([x[2] for x in parts]).astype(np.int64)
        m = sc >= 0
        ds, rw, sc = ds[m], rw[m], sc[m]
        for d in (0, 1):
            sel = ds == d
            r, s = rw[sel][::-1], sc[sel][::-1]        # reversed: the first occurrence wins
            self.masked_scope[d][r] = s
        keep = np.zeros(len(ds), bool)
        if len(ds):
            _, first = np.unique(FastqFormatter._key(ds, rw, sc), return_index=True)
            keep[np.sort(first)] = True     # every distinct copy, first occurrences first
        ds, rw, sc = ds[keep], rw[keep], sc[keep]
        self.masked_keys = np.unique(FastqFormatter._key(ds, rw, sc))
        c = self._complex_incidences()      # every (alignment, scope) of a complex name: one copy each
        if len(c):
            ds, rw, sc = np.concatenate([ds, c[:, 0]]), np.concatenate([rw, c[:, 1]]), np.concatenate([sc, c[:, 2]])
        return ds, rw, sc

    def _complex_incidences(self) -> np.ndarray:
        """(dataset, row, scope) of every alignment of a complex name's object in a scope, [n, 3]."""
        c = getattr(self, "_cx_inc", None)
        if c is not None:
            return c
        O = self.objs
        if not len(O):
            c = np.zeros((0, 3), np.int64)
        else:
            O = O[O[:, 0] >= 0]
            n = O[:, 6]
            idx = np.repeat(O[:, 5] - np.concatenate([[0], np.cumsum(n)[:-1]]), n) + np.arange(int(n.sum()))
            trip = np.stack([np.repeat(O[:, 1], n), self.obj_rows[idx], np.repeat(O[:, 0], n)], axis=1)
            c = np.unique(trip, axis=0) if len(trip) else np.zeros((0, 3), np.int64)
        self._cx_inc = c
        return c


class Job(JobPrep):
    """One contig: its JobPrep stage, then mask + format on the device; once resolved, its output
    bytes."""

    def __init__(self, spec: JobSpec, readers, fasta: FastaRef, windows: Sequence[Window],
                 anonymizer: CompleteGermlineAnonymizer, prepared=None, secondaries: Optional[SecondaryIndex] = None):
        """``prepared``: a ``concurrent.futures.Future`` of this job's JobPrep when the caller
        prefetched it; decode_s is then the time spent waiting for it and prefetch_s the time the
        thread spent (decode + plan + batch)."""
        t0 = time.time()
        if prepared is None:
            JobPrep.__init__(self, spec, readers, fasta, windows, secondaries=secondaries)
            t_dec, t_pl, t_b = self.prep_timing
            hidden = 0.0
        else:
            self.__dict__.update(prepared.result().__dict__)
            t_dec, t_pl, t_b = time.time() - t0, 0.0, 0.0
            hidden = sum(self.prep_timing)
        t2 = time.time()
        # the device part in one hold of the engine: a job planned again on the writer thread
        # (SecondaryIndex) must not take the engine's job batch between this mask and its format
        with anonymizer.lock:
            self.res: MaskResult = anonymizer.anonymize(self.planner, self.plan, written=self.written,
                                                        batch=self.batch, lazy_seq=True)
            self.batch = None
            t3 = time.time()
            self.fmt = FastqFormatter(self.tables, self.res, anonymizer.format_fastq,
                                      getattr(anonymizer, "format_fastq_batch", None))
            # every read once, as its masked copy (or unmasked): the records this job can write. The
            # masked bases stay on the device unless a later stage needs them on the host (records
            # left to on-demand formatting, complex names' objects): fetched now, while the engine's
            # job batch still holds them
            nb = self.tables[0].n + self.tables[1].n   # (_format_instances: every read once first)
            if not self.fmt.preformat(*self._format_instances(), n_base=nb) or len(self.objs):
                _ = self.res.seq_out
        t4 = time.time()
        self.cx = self._complex_ingredients()
        self.timing = {"decode_s": t_dec, "plan_s": t_pl, "mask_s": t3 - t2 + t_b, "format_s": t4 - t3,
                       "prefetch_s": hidden}
        # the prefetch thread's parts: waiting for the decode thread, the plan, the batch build
        self.prep_parts = self.prep_timing if prepared is not None else (0.0, 0.0, 0.0)

    def _format_instances(self):
        """Every read once as its masked copy (or unmasked), plus the unmasked records the events,
        unwritten pairs and candidates name for reads masked elsewhere."""
        ds, rw, sc = [], [], []
        for d in (0, 1):
            n = self.tables[d].n
            ds.append(np.full(n, d, np.int64))
            rw.append(np.arange(n, dtype=np.int64))
            sc.append(self.masked_scope[d])
        ev, rows = self.events, self.event_rows
        m = ((ev[:, 0] == 1) | ((ev[:, 0] >= 3) & (ev[:, 0] <= 5))) & (ev[:, 5] < 0)
        ds.append(ev[m, 4].astype(np.int64))
        rw.append(rows[m].astype(np.int64))
        L = self.left
        for s_ in (0, 1):
            h = (L[:, 1 + 4 * s_] == 1) & (L[:, 3 + 4 * s_] < 0) if len(L) else np.zeros(0, bool)
            ds.append(L[h, 2 + 4 * s_].astype(np.int64))
            rw.append(L[h, 4 + 4 * s_].astype(np.int64))
        C = self.cand
        cm = C[:, 1] >= 0 if len(C) else np.zeros(0, bool)
        ds.append(C[cm, 1].astype(np.int64))
        rw.append(C[cm, 2].astype(np.int64))
        n_extra = sum(len(x) for x in ds[2:])
        sc.append(np.full(n_extra, -1, np.int64))
        # the further masked copies of reads met in two scopes (cross names)
        mk = self.masked_keys
        if len(mk):
            m_sc = (mk >> 33) - 1
            m_ds = (mk >> 32) & 1
            m_rw = mk & 0xFFFFFFFF
            other = np.nonzero(np.where(m_ds == 0, self.masked_scope[0][np.where(m_ds == 0, m_rw, 0)] if self.tables[0].n else -1,
                                        self.masked_scope[1][np.where(m_ds == 1, m_rw, 0)] if self.tables[1].n else -1)
                               != m_sc)[0]
            ds.append(m_ds[other])
            rw.append(m_rw[other])
            sc.append(m_sc[other])
        return np.concatenate(ds), np.concatenate(rw), np.concatenate(sc)

    def is_masked(self, ds, row, sc) -> np.ndarray:
        """Whether the device masked copy (dataset, row, scope) (vectorised; scope -1: unmasked)."""
        k = FastqFormatter._key(ds, row, sc)
        mk = self.masked_keys
        if not len(mk):
            return np.asarray(sc) < 0
        pos = np.minimum(np.searchsorted(mk, k), len(mk) - 1)
        return (np.asarray(sc) < 0) | (mk[pos] == k)

    def _masked_nibs(self, I: np.ndarray) -> np.ndarray:
        """MaskResult.masked_nib of every (dataset, row, scope) row of ``I``, vectorised."""
        T = self.tables
        d0 = I[:, 0] == 0
        r0, r1 = np.where(d0, I[:, 1], 0), np.where(d0, 0, I[:, 1])
        off = np.where(d0, T[0].seq_off[r0] if T[0].n else 0, T[1].seq_off[r1] if T[1].n else 0).astype(np.int64)
        nib = 2 * (np.where(d0, self.res.seq_base[0], self.res.seq_base[1]) + off)
        dup = self.res.dup_off
        if dup and len(I):
            k = np.array(list(dup.keys()), np.int64).reshape(-1, 3)
            v = np.array(list(dup.values()), np.int64)
            M = max(T[0].n, T[1].n) + 1
            dk = (k[:, 2] * 2 + k[:, 0]) * M + k[:, 1]
            o = np.argsort(dk)
            ik = (I[:, 2] * 2 + I[:, 0]) * M + I[:, 1]
            p = np.minimum(np.searchsorted(dk[o], ik), len(dk) - 1)
            hit = dk[o][p] == ik
            nib[hit] = 2 * v[o][p[hit]]
        return nib

    def _complex_ingredients(self):
        """What the object replay needs of this job's complex names: their records and, per
        (alignment, scope), the bases the device masked and the indel left-overs — the packed blob of
        ``native.objects_pack`` (objects.NativeReplay), or Python objects (objects.Replay,
        GANON_OBJECTS=python)."""
        O = self.objs
        if not len(O):
            return None
        if os.environ.get("GANON_OBJECTS", "native") != "python":
            I = self._complex_incidences()
            T = self.tables
            nib = self._masked_nibs(I)
            incs = set(map(tuple, I.tolist()))
            left = {k: v for k, v in self.res.leftovers.items() if v and k in incs}
            return native.objects_pack(T, O, self.obj_rows, I, nib, self.res.seq_out, left)
        rec = {}
        for ds in (0, 1):
            m = O[:, 1] == ds
            if not np.any(m):
                continue
            rows = [O[m, 3], O[m, 4][O[m, 4] >= 0]]
            rows += [self.obj_rows[a:a + n] for a, n in zip(O[m, 5].tolist(), O[m, 6].tolist())]
            for r, v in objects.records_of(self.tables[ds], np.concatenate(rows)).items():
                rec[(ds, r)] = v
        masks, indels = {}, {}
        I = self._complex_incidences()
        if len(I):
            # every incidence's masked copy against its record, one vectorised compare
            T = self.tables
            d0 = I[:, 0] == 0
            r0, r1 = np.where(d0, I[:, 1], 0), np.where(d0, 0, I[:, 1])
            pick = lambda f: np.where(d0, getattr(T[0], f)[r0] if T[0].n else 0,
                                      getattr(T[1], f)[r1] if T[1].n else 0).astype(np.int64)
            L = pick("l_seq")
            onib = 2 * pick("seq_off")
            mnib = self._masked_nibs(I)
            start = np.concatenate([[0], np.cumsum(L)[:-1]])
            k = np.arange(int(L.sum()), dtype=np.int64) - np.repeat(start, L)
            src = np.concatenate([T[0].seq, T[1].seq]) if T[1].n else T[0].seq
            base1 = len(T[0].seq)
            on = np.repeat(onib + 2 * base1 * (I[:, 0] == 1), L) + k
            mn = np.repeat(mnib, L) + k
            ob = src[on >> 1]
            ov = np.where(on & 1, ob & 0xF, ob >> 4)
            mb = self.res.seq_out[mn >> 1]
            mv = np.where(mn & 1, mb & 0xF, mb >> 4)
            hit = np.nonzero(ov != mv)[0]
            owner = np.searchsorted(start, hit, side="right") - 1
            inc = I.tolist()
            for i in np.unique(owner).tolist():
                ds, a, sc = inc[i]
                sel = hit[owner == i]
                idx = sel - start[i]
                cols = rec[(ds, a)].columns(idx)
                masks[(ds, a, sc)] = list(zip(cols.tolist(), idx.tolist(), objects.NT16[mv[sel]].tolist(),
                                              objects.NT16[ov[sel]].tolist()))
            if self.res.leftovers:
                incset = set(map(tuple, inc))
                for k, e in self.res.leftovers.items():
                    if e and k in incset:
                        indels[k] = list(e)
        return {"objs": O, "obj_rows": self.obj_rows, "rec": rec, "masks": masks, "indels": indels}

    def check_instance(self, ds: int, row: int, scope: int) -> None:
        if scope >= 0 and not bool(self.is_masked(np.array([ds]), np.array([row]), np.array([scope]))[0]):
            raise RuntimeError(f"internal: read {self.tables[ds].name(row)!r} written from scope {scope} of "
                               f"{self.contig!r}, a copy the device did not mask")

    # -- exports for the resolution ---------------------------------------------------------------
    def record_lengths(self, ds, row, sc, reapply=None) -> np.ndarray:
        return self.fmt.record_lengths(ds, row, sc, reapply)

    def format_records(self, ds, row, sc, reapply=None) -> List[bytes]:
        ds = np.asarray(ds, np.int64)
        row = np.asarray(row, np.int64)
        sc = np.asarray(sc, np.int64)
        if len(ds) == 0:
            return []
        data = self.fmt.format_arrays(ds, row, sc, reapply)
        off = np.concatenate([[0], np.cumsum(self.record_lengths(ds, row, sc, reapply))])
        return [data[off[i]:off[i + 1]] for i in range(len(ds))]

    def exports(self) -> dict:
        ev, rows = self.events, self.event_rows
        p = self.ph
        ops = ev[p]
        op_rows = rows[p]
        op_ds = ops[:, 4].astype(np.int64)
        plain = ops[:, 0] <= 5
        O = self.objs
        op_name_rows = op_rows.copy()
        if len(O) and not np.all(plain):   # objects: the name of their creator
            op_name_rows[~plain] = O[op_rows[~plain], 3]
        L = self.left
        left_ds = np.where(L[:, 1] == 1, L[:, 2], L[:, 6]) if len(L) else np.zeros(0, np.int64)
        left_row = np.where(L[:, 1] == 1, L[:, 4], L[:, 8]) if len(L) else np.zeros(0, np.int64)
        C = self.cand
        cm = C[:, 1] >= 0 if len(C) else np.zeros(0, bool)
        cand = np.zeros((len(C), 8), np.int64)
        if len(C):
            cand[:, 0] = self.job
            cand[:, 1:7] = C
            cand[:, 7] = -1
            for d in (0, 1):   # identities of the records that create objects with supplementary state
                sel = np.nonzero((C[:, 1] == d) & (C[:, 5] != 0))[0]
                if len(sel):
                    cand[sel, 7] = content_ids(self.tables[d], C[sel, 2])
        cand_names = [b""] * len(C)
        idx = np.nonzero(cm)[0]
        for i, nm in zip(idx.tolist(), _names_ds(self.tables, C[idx, 1], C[idx, 2])):
            cand_names[i] = nm
        # carried records: every instance the resolution may write outside this job
        inst = [(ops[plain, 4].astype(np.int64), op_rows[plain], ops[plain, 5].astype(np.int64))]
        for s in (0, 1):
            h = L[:, 1 + 4 * s] == 1 if len(L) else np.zeros(0, bool)
            inst.append((L[h, 2 + 4 * s], L[h, 4 + 4 * s], L[h, 3 + 4 * s]))
        inst.append((C[idx, 1], C[idx, 2], np.full(len(idx), -1, np.int64)))
        ds = np.concatenate([x[0] for x in inst]).astype(np.int64)
        rw = np.concatenate([x[1] for x in inst]).astype(np.int64)
        sc = np.concatenate([x[2] for x in inst]).astype(np.int64)
        carry: Dict[Key, bytes] = {}
        info: dict = {}
        if len(ds):
            _, first = np.unique(FastqFormatter._key(ds, rw, sc), return_index=True)
            first = np.sort(first)
            first = first[self.is_masked(ds[first], rw[first], sc[first])] if len(first) else first
            recs = self.format_records(ds[first], rw[first], sc[first])
            edited = []
            for i, b in zip(first.tolist(), recs):
                inst = (int(ds[i]), int(rw[i]), int(sc[i]))
                carry[(self.job, inst[0], inst[2], inst[1], 0)] = b
                info[(self.job, inst[0], inst[1])] = int(self.tables[inst[0]].flag[inst[1]])
                if inst in self.res.leftovers:
                    edited.append(inst)
            # written later with its left-overs applied twice; the record before its edits and the
            # edits (objects.Replay, complex names)
            self.fmt.prepare_edited(edited, [1] * len(edited))
            for inst, b in zip(edited, self.fmt.unedited(edited)):
                carry[(self.job, inst[0], inst[2], inst[1], 1)] = self.fmt.edited_bytes(inst, 1)
                carry[(self.job, inst[0], inst[2], inst[1], 2)] = b
                info[(self.job, inst[0], inst[2], inst[1])] = list(self.res.leftovers[inst])
        op_names = _names_ds(self.tables, op_ds, op_name_rows)
        left_names = _names_ds(self.tables, left_ds, left_row)
        # (redo_needed) names planned as cross names here: those of plain placeholder events (kinds
        # 3-5; the object events 6/7 and the unwritten pairs can be local names)
        self.cross_names = {nm for nm, pl in zip(op_names, plain.tolist()) if pl}
        return {
            "job": self.job, "ops": ops, "op_rows": op_rows,
            "op_names": op_names,
            "left": L, "left_names": left_names,
            "cand": cand, "cand_names": cand_names, "carry": carry, "carry_info": info,
            "objs": O, "obj_rows": self.obj_rows, "cx": self.cx,
            "obj_ids": self._obj_ids(), "forced": self.forced, "offsec": self.offsec, "own_sec": self.own_sec,
        }

    def _obj_ids(self) -> Optional[np.ndarray]:
        """content_ids of every obj_rows entry (the records of each object: alignments, then the
        supplementary records it recorded; all of its dataset)."""
        O = self.objs
        if not len(O):
            return None
        ds = np.repeat(O[:, 1], O[:, 6] + O[:, 8])
        ids = np.zeros(len(self.obj_rows), np.int64)
        for d in (0, 1):
            sel = np.nonzero(ds == d)[0]
            if len(sel):
                ids[sel] = content_ids(self.tables[d], self.obj_rows[sel])
        return ids

    # -- output ----------------------------------------------------------------------------------
    def local_sizes(self) -> List[int]:
        """Bytes of the job's own (non-placeholder) writes per output file (tumor .1, .2, normal .1,
        .2): with the resolved placeholder writes, the coordinator places the job in the files."""
        ev, rows = self.events, self.event_rows
        w = np.nonzero(ev[:, 0] == 1)[0]
        if not len(w):
            return [0, 0, 0, 0]
        ln = self.record_lengths(ev[w, 4], rows[w], ev[w, 5], ev[w, 6])
        f = 2 * ev[w, 2].astype(np.int64) + ev[w, 3]
        return [int(x) for x in np.bincount(f, weights=ln, minlength=4).astype(np.int64)[:4]]

    def output(self, out_n: np.ndarray, out_w: np.ndarray, ext_list: List[bytes], block: int) -> List[bytes]:
        """The job's bytes per output file (tumor .1, .2, normal .1, .2) with the resolved writes of
        its placeholder events spliced into its I/O log, each as a list of buffers written back to back
        (no join); ``ext_list``: the bytes of the resolved writes of records of other contigs (and
        objects of complex names), in event order (the coordinator's ``resolve``)."""
        ev, rows = self.events, self.event_rows
        n = len(ev)
        is_ph = ev[:, 0] >= 3
        k = np.ones(n, np.int64)
        k[is_ph] = 0
        if len(self.ph):
            k[self.ph] = out_n
        src = np.repeat(np.arange(n), k)                 # source event of each final event
        nf = len(src)
        fin = ev[src].copy()
        frow = rows[src].copy()
        fjob = np.full(nf, self.job, np.int64)
        # the resolved writes: placeholder op i contributes out_w[i, :out_n[i]]
        ph_pos = np.nonzero(is_ph[src])[0]
        if len(ph_pos):
            which = np.concatenate([np.arange(c) for c in out_n[out_n > 0]]) if np.any(out_n > 0) else np.zeros(0, np.int64)
            opi = np.repeat(np.arange(len(self.ph)), out_n)
            w = out_w[opi, which]
            fin[ph_pos, 0] = 1
            fin[ph_pos, 2] = w[:, 0]
            fin[ph_pos, 3] = w[:, 1]
            fin[ph_pos, 4] = w[:, 3]
            fin[ph_pos, 5] = w[:, 4]
            fin[ph_pos, 6] = w[:, 6]
            frow[ph_pos] = w[:, 5]
            fjob[ph_pos] = w[:, 2]
        wr = fin[:, 0] == 1
        fin[~wr, 6] = 0
        reap = fin[:, 6].astype(np.int64)
        gen = wr & (fin[:, 5] == -2)        # an object of a complex name (objects.Replay)
        ext = wr & ((fjob != self.job) | gen)
        loc = wr & ~ext
        chk = np.nonzero(loc & (fin[:, 5] >= 0))[0]   # plain local writes only (gen is ext)
        if len(chk):
            d, r, sc = fin[chk, 4].astype(np.int64), frow[chk], fin[chk, 5].astype(np.int64)
            bad = np.nonzero(~self.is_masked(d, r, sc))[0]
            if len(bad):
                i = int(chk[bad[0]])
                self.check_instance(int(fin[i, 4]), int(frow[i]), int(fin[i, 5]))
        rec_len = np.zeros(nf, np.int64)
        li = np.nonzero(loc)[0]
        rec_len[li] = self.record_lengths(fin[li, 4], frow[li], fin[li, 5], reap[li])
        xi = np.nonzero(ext)[0]
        if len(xi) != len(ext_list):
            raise RuntimeError(f"job {self.job}: {len(xi)} writes from other contigs, {len(ext_list)} resolved")
        ext_bytes: Dict[int, bytes] = dict(zip(xi.tolist(), ext_list))
        if len(xi):
            rec_len[xi] = [len(b) for b in ext_list]
        order = native.io_replay(fin[:, :7].astype(np.int32), np.where(wr, rec_len, 0), block)
        # every local record of the four files in ONE formatter call, then split per file
        les = [order[f][~ext[order[f]]] for f in range(4)]
        allr = np.concatenate(les)
        blob = self.fmt.format_arrays(fin[allr, 4], frow[allr], fin[allr, 5], reap[allr]) if len(allr) else b""
        cut = np.concatenate([[0], np.cumsum([int(rec_len[x].sum()) for x in les])])
        out = []
        mv = memoryview(blob)
        for f in range(4):
            e = order[f]
            is_ext = ext[e]
            le = les[f]
            data = mv[cut[f]:cut[f + 1]]
            if not np.any(is_ext):
                out.append([data])
                continue
            off = np.concatenate([[0], np.cumsum(rec_len[le])])
            parts, prev_local = [], 0
            pos = np.nonzero(is_ext)[0]
            offl = off.tolist()
            for j, (p, ei) in enumerate(zip(pos.tolist(), e[pos].tolist())):
                n_local_before = p - j
                parts.append(data[offl[prev_local]:offl[n_local_before]])
                parts.append(ext_bytes[ei])
                prev_local = n_local_before
            parts.append(data[offl[prev_local]:])
            out.append(parts)
        return out

    def stats(self) -> Dict[str, List[int]]:
        return statistics_rows(self.plan, self.res)

    def release_device(self) -> None:
        """The job's exports are out: nothing on the device is needed to write it any more."""
        self.batch = None

    def redo_needed(self, force: Sequence[bytes]) -> List[bytes]:
        """The names of ``force`` whose forcing changes this job's plan: not forced already, present in
        its records (a name it never meets plans the same), and planned as a local name (a name already
        cross here — a placeholder event or an unwritten pair of its export — plans the same).
        Call after exports()."""
        new = sorted(set(force) - set(self.forced) - getattr(self, "cross_names", set()))
        if not new:
            return []
        out = []
        for t in self.tables:
            if not len(new) or t.n == 0:
                continue
            found = _names_present(t, new)
            out.extend(nm for nm in new if nm in found)
            new = [nm for nm in new if nm not in found]
        return sorted(out)


class _Comm:
    """Host-side gathers for the per-round exchange (gloo group over torch.distributed)."""

    def __init__(self, dist=None):
        self.dist = dist
        self.group = None
        self.rank, self.world = 0, 1
        if dist is not None:
            self.rank, self.world = dist.get_rank(), dist.get_world_size()
            self.group = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else None

    def allgather(self, obj) -> list:
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def barrier(self) -> None:
        if self.dist is not None:
            self.dist.barrier(group=self.group)

    def allreduce_totals(self, totals: np.ndarray) -> np.ndarray:
        """The one collective on the data path's results: int64 totals, summed over the ranks (RCCL
        over xGMI on the default nccl group, gloo otherwise)."""
        if self.dist is None:
            return totals
        import torch
        dev = torch.device("cuda", torch.cuda.current_device()) if self.dist.get_backend() == "nccl" \
            else torch.device("cpu")
        t = torch.from_numpy(totals.astype(np.int64)).to(dev)
        self.dist.all_reduce(t)
        return t.cpu().numpy()


class _Coordinator:
    """The sample-wide pairing state (rank 0): resolves the contigs in FASTA order as their exports
    arrive — ``native.Resolver`` over the placeholder events, the object replay of complex names,
    the carried records — and answers each job's owner with its resolved writes, the bytes of those
    writing records of other contigs, and the offsets of the job's bytes in the four files (their
    sizes follow from the owner's own write sizes and the resolved writes: no round trip). At the
    end it writes the tail (``pair_unmapped_mates``) and the single ends (SR:561-622)."""

    def __init__(self, fds, paths_single, block_size: int):
        self.fds = fds
        self.paths_single = paths_single
        self.block = block_size
        self.resolver = native.Resolver()
        self.carry: Dict[Key, bytes] = {}
        self.carry_info: dict = {}
        self.replay = (objects.Replay if os.environ.get("GANON_OBJECTS") == "python" else objects.NativeReplay)(
            self.carry, self.carry_info)
        self.cands: List[np.ndarray] = []
        self.cand_live: set = set()
        self.cand_names: List[bytes] = []
        self.carry_floor = 0
        self.prune_min = int(os.environ.get("GANON_CARRY_PRUNE_MIN", "200000"))   # carried records before a prune
        self.base = [0, 0, 0, 0]
        self.prunes = 0
        self.resolve_s = 0.0
        self.need_force: Dict[int, set] = {}   # job -> names its plan must treat as cross (SecondaryIndex)
        self.redos = 0
        self.redos_unchanged = 0   # redo requests the owner answered without planning again
        self.marked = 0

    def missing_force(self, exp: dict, k: int) -> List[bytes]:
        """Names job k's plan had to plan as cross names but did not (a secondary of an earlier job,
        decoded on another rank after this job was planned): the owner plans it again with them."""
        need = self.need_force.get(k)
        if not need:
            return []
        return sorted(need - set(exp.get("forced", ())) - set(exp.get("own_sec", ())))

    def _bytes_of(self, jb: int, d: int, sc: int, r: int, re_: int) -> bytes:
        if sc == -2:        # an object of a complex name (objects.Replay)
            return self.replay.take(r)
        b = self.carry.get((jb, d, sc, r, re_))
        if b is None and re_:   # a carried record without left-overs: the same bytes
            b = self.carry.get((jb, d, sc, r, 0))
        if b is None:
            raise RuntimeError(f"internal: record {(jb, d, sc, r)} written across contigs was not carried")
        return b

    def resolve(self, exp: dict, k: int) -> dict:
        t0 = time.time()
        e = exp
        # off-contig secondaries of this job: a mate's contig before it planned the name locally and
        # wrote it (unless the resolver holds the name: pending, or planned as cross there); a mate's
        # contig after it must plan the name as a cross name
        before = [nm for nm, mj in e.get("offsec", ()) if mj < k]
        if before:
            self.marked += self.resolver.mark_written(sorted(set(before)))
        for nm, mj in e.get("offsec", ()):
            if mj > k:
                self.need_force.setdefault(mj, set()).add(nm)
        self.need_force.pop(k, None)
        self.carry.update(e["carry"])
        self.carry_info.update(e["carry_info"])
        self.replay.add_job(e["job"], e["cx"])
        out_n, out_w = self.resolver.contig(e["job"], e["ops"], e["op_rows"], e["op_names"], e["left"],
                                            e["left_names"], e["objs"], e["obj_rows"], e.get("obj_ids"))
        self.replay.run(self.resolver.take_log())
        c = e["cand"]
        self.cands.append(c)
        if len(c):      # candidates stay live to the end of the sample
            self.cand_live.update((r[0], r[2], -1, r[3]) for r in c[c[:, 2] >= 0].tolist())
        self.cand_names.extend(e["cand_names"])
        # the job's resolved writes: bytes of those from other contigs (in event order), file sizes
        sizes = list(e["local_sizes"])
        ext: List[bytes] = []
        job = e["job"]
        for i in range(len(out_n)):
            for w in out_w[i, :int(out_n[i])].tolist():
                f, jb, d, sc, r, re_ = 2 * w[0] + w[1], w[2], w[3], w[4], w[5], w[6]
                b = self._bytes_of(jb, d, sc, r, re_)
                if jb != job or sc == -2:
                    ext.append(b)
                sizes[f] += len(b)
        offsets = list(self.base)
        for f in range(4):
            self.base[f] += sizes[f]
        # carried records still reachable: pending pairs and the end-of-sample candidates (pruned
        # when the carry has doubled; the objects of complex names are settled every 16 jobs)
        grow = len(self.carry) > max(self.prune_min, 2 * self.carry_floor)
        if grow or k % 16 == 15:
            pend = self.resolver.pending()
            self.replay.settle(pend)
            if grow:
                live = set(map(tuple, pend.tolist()))
                live |= self.cand_live
                for key in [key for key in self.carry if key[:4] not in live]:
                    del self.carry[key]
                live_rows = {(x[0], x[1], x[3]) for x in live}
                for key in [key for key in self.carry_info
                            if (key if len(key) == 3 else (key[0], key[1], key[3])) not in live_rows
                            or (len(key) == 4 and key not in live)]:
                    del self.carry_info[key]
                self.carry_floor = len(self.carry)
                self.prunes += 1
        self.resolve_s += time.time() - t0
        return {"job": job, "out_n": out_n, "out_w": out_w, "ext": ext, "offsets": offsets, "sizes": sizes,
                "err": None}

    def finish(self, rank0_fds) -> None:
        """End of the sample: pair_unmapped_mates, single ends (SR:561-622)."""
        cand = np.concatenate(self.cands) if self.cands else np.zeros((0, 8), np.int64)
        tail, single, wse = self.resolver.finish(cand, self.cand_names)
        self.replay.run(self.resolver.take_log())
        per_file: List[List[bytes]] = [[], [], [], []]

        def carried(k):
            if k[2] == -2:
                return self.replay.take(k[3])
            b = self.carry.get(k)
            return b if b is not None else self.carry[k[:4] + (0,)]
        for w in tail.tolist():
            per_file[2 * w[0] + w[1]].append(carried((w[2], w[3], w[4], w[5], w[6])))
        for f in range(4):
            blob = b"".join(per_file[f])
            if blob:
                _pwrite_all(rank0_fds[f], blob, self.base[f])
        if wse:
            for d, path in enumerate(self.paths_single):
                with open(path, "wb") as fh:
                    fh.write(b"".join(carried(tuple(x)) for x in single[d].tolist()))

    def close(self) -> None:
        self.resolver.close()


def anonymize_genome_streaming(windows: List[Window], tumor_bam: str, normal_bam: str, fasta: FastaRef,
                               anonymizer: CompleteGermlineAnonymizer, tumor_out: str, normal_out: str,
                               record_statistics: bool, threads: int = 8, dist=None,
                               normal_stats_path: Optional[str] = None, block_size: Optional[int] = None,
                               window_bytes: int = 0) -> dict:
    """One tumor/normal pair, contig by contig (single rank when ``dist`` is None, else the
    ranks of the initialised torch.distributed world, each on its own contigs: distributed.py).
    Output files, statistics and errors are the reference's (SR:625-760)."""
    from .distributed import Link, assign_contigs
    t_start = time.time()
    comm = _Comm(dist)
    rank, world = comm.rank, comm.world
    paths = [f"{tumor_out}.1.fastq", f"{tumor_out}.2.fastq", f"{normal_out}.1.fastq", f"{normal_out}.2.fastq"]
    if block_size is None:
        block_size = _writer.io_block_size(os.path.dirname(os.path.abspath(tumor_out)))
    timing = {"decode_s": 0.0, "plan_s": 0.0, "mask_s": 0.0, "format_s": 0.0, "prefetch_s": 0.0, "resolve_s": 0.0,
              "write_s": 0.0, "wait_s": 0.0, "writer_wait_s": 0.0, "prunes": 0, "jobs": 0, "reads": 0, "bases": 0}
    failure: Optional[BaseException] = None
    if rank == 0:
        for p in paths:
            open(p, "wb").close()
    comm.barrier()
    fds = [os.open(p, os.O_WRONLY) for p in paths]
    readers = (BamReader(tumor_bam, threads, window_bytes), BamReader(normal_bam, threads, window_bytes))
    # jobs: contigs, or runs of sections of about GANON_JOB_BP bases (default 4 Mb; 0 = whole
    # contigs) when both BAMs are indexed
    # (unset: 4 Mb, or smaller so that every rank gets about GANON_JOBS_PER_RANK jobs (default 3, at
    # least 256 kb each): 2 x 20 Mb over 8 ranks made 10 jobs of 4 Mb, two ranks ran two each and
    # the rest idled half the wall — round 5's 30x chromosome-scale line)
    job_bp = int(os.environ.get("GANON_JOB_BP", "0") or 0) if "GANON_JOB_BP" in os.environ else \
        auto_job_bp(sum(int(L) for L in fasta.lengths), world)
    genome_len = sum(int(L) for L in fasta.lengths)
    jobs = plan_jobs(fasta, windows, job_bp, all(r.has_index for r in readers),
                     job_targets(genome_len, job_bp, world, float(os.environ.get("GANON_JOB_TAPER", "1"))))
    # The readers' BGZF windows inflate on this rank's GPU (a context of its own per reader: the two
    # samples decode at once) when the masking engine is the GPU's and a job's reads come in windows of at least GANON_GPU_INFLATE_MIN blocks (default 512,
    # ~18 MB compressed: a block takes milliseconds on its wave, so only large windows pay off, and
    # the context costs its setup) — round 5: the token-round kernel made it the faster decoder at
    # chromosome scale (30x line: 6.28e6 -> 6.93e6 and 5.87e6 -> 8.04e6 reads/s on two boxes, 22 %
    # less host CPU). GANON_GPU_INFLATE=0 / 1 forces it off / on.
    inflater = None
    gi = os.environ.get("GANON_GPU_INFLATE", "auto")
    min_blocks = int(os.environ.get("GANON_GPU_INFLATE_MIN", "512"))
    gpu_engine = anonymizer._engine is None or isinstance(anonymizer._engine, native.HipMasker)
    big_jobs = max(os.path.getsize(p) for p in (tumor_bam, normal_bam)) / max(1, len(jobs)) >= min_blocks * 36_000
    if gi == "1" or (gi == "auto" and gpu_engine and big_jobs):
        # (per device, sample and process, kept for the next run: their teardown was part of every
        # run's tail)
        for i, r in enumerate(readers):
            inflater = _INFLATERS.get((anonymizer.device, min_blocks, i))
            if inflater is None:
                inflater = _INFLATERS[(anonymizer.device, min_blocks, i)] = native.GpuInflater(anonymizer.device,
                                                                                             min_blocks)
            r.set_inflater(inflater)
    owner = assign_contigs([j.length for j in jobs], world)
    mine = [j for j in range(len(jobs)) if owner[j] == rank]
    t_g = time.time()
    link = Link(dist)
    timing_groups = time.time() - t_g
    coord = _Coordinator(fds, (f"{tumor_out}.single_end.fastq", f"{normal_out}.single_end.fastq"), block_size) \
        if rank == 0 else None
    coord_exc: List[Optional[BaseException]] = [None]
    stats_rows: List[Tuple[int, Dict[str, List[int]]]] = []
    totals = np.zeros(8, np.int64)
    totals_lock = threading.Lock()
    secondaries = SecondaryIndex(readers, jobs)
    xchg = None
    if world > 1 and os.environ.get("GANON_SEC_EXCHANGE", "1") != "0":
        from .distributed import SecondaryExchange
        t_g = time.time()
        xchg = SecondaryExchange(dist, owner)
        timing_groups += time.time() - t_g
        secondaries.remote = xchg

    stash: Dict[int, list] = {}      # exports an owner sent after the job it is planning again

    def recv_export(o: int) -> dict:
        q = stash.get(o)
        return q.pop(0) if q else link.recv_export(o)

    def recv_redo(o: int, k: int) -> dict:
        while True:
            m = link.recv_export(o)
            if m.get("err") is not None or m.get("redo_of") == k:
                return m
            stash.setdefault(o, []).append(m)

    def coordinate() -> None:
        """Rank 0's coordinator thread: every job in FASTA order, as its export arrives. When it
        stops on an error, every rank with a job still unresolved gets the error and answers with
        an error export of its own (stream loop below); the exports it sent in between are received
        and dropped, so no send is left without its receive."""
        err = None
        k = 0
        failed_owner = -1
        try:
            for k in range(len(jobs)):
                o = owner[k]
                exp = recv_export(o)
                while exp.get("err") is None:
                    miss = coord.missing_force(exp, k)
                    if not miss:
                        break
                    coord.redos += 1
                    link.send_resolution(o, {"job": k, "redo": sorted(set(miss) | set(exp.get("forced", ()))),
                                             "err": None})
                    re_exp = recv_redo(o, k)
                    if re_exp.get("unchanged") and re_exp.get("err") is None:
                        # the owner found nothing to plan again: the first export stands
                        coord.redos_unchanged += 1
                        exp["forced"] = re_exp["forced"]
                    else:
                        exp = re_exp
                if exp.get("err") is not None:   # the owner failed: its error is its own to report
                    err = exp["err"]
                    failed_owner = o
                    break
                link.send_resolution(o, coord.resolve(exp, k))
                k += 1
            if err is None:
                coord.finish(fds)
        except BaseException as e:   # reported to every owner still waiting
            coord_exc[0] = e
            err = repr(e)
        if err is not None:
            waiting = sorted({owner[j] for j in range(k, len(jobs))})
            for r in waiting:        # every worker with a job not resolved stops
                link.send_resolution(r, {"err": err})
            for r in waiting:        # ... and answers with its error: drop what it sent before
                if r == failed_owner:
                    continue
                while recv_export(r).get("err") is None:
                    pass

    coord_thread = threading.Thread(target=coordinate, name="ganon-coordinator", daemon=True) if rank == 0 else None
    if coord_thread is not None:
        coord_thread.start()
    # look-ahead: a decode thread reads this rank's next contigs in order (one BamReader stream) and
    # `depth` threads plan and batch them (JobPrep) while the current one masks, formats and writes;
    # GANON_PREFETCH = depth (default 2, 0: everything in line). At most `pend_max` jobs wait for
    # their resolution (GANON_PENDING, default 4): memory is bounded by them and the prefetched jobs.
    depth = int(os.environ.get("GANON_PREFETCH", "2"))
    pend_max = max(1, int(os.environ.get("GANON_PENDING", "4")))
    dec_pool = ThreadPoolExecutor(1) if depth > 0 else None
    pool = ThreadPoolExecutor(depth) if depth > 0 else None
    ahead: Dict[int, object] = {}
    nxt = [0]                  # index in `mine` of the next job to submit

    def submit_upto(i_last: int) -> None:
        while nxt[0] <= min(i_last, len(mine) - 1):
            j = mine[nxt[0]]
            dec = dec_pool.submit(decode_job, readers, jobs[j], secondaries)
            ahead[j] = pool.submit(JobPrep, jobs[j], readers, fasta, windows, dec, secondaries)
            nxt[0] += 1

    # the writer thread: each exported job, in order, waits for its resolution, splices its bytes and
    # writes them at their offsets while the main thread masks and formats the next contigs (the
    # splice is numpy and native code, the writes are pwrite: both mostly outside the GIL).
    # GANON_WRITER=0 writes in line.
    writer = ThreadPoolExecutor(1) if os.environ.get("GANON_WRITER", "1") != "0" else None
    file_pool = ThreadPoolExecutor(4)
    pending: list = []          # futures of the writer (or jobs, in line)
    writer_failed = threading.Event()

    redo_readers: list = []

    def redo(job: "Job", force: List[bytes]) -> "Job":
        """Plan, mask and format ``job`` again with ``force`` planned as cross names (its own
        readers: the decode thread owns the others) and send its export in place of the first."""
        if not job.redo_needed(force):
            # every name it would force is absent from the job or already a cross name there: the
            # plan would not change — tell the coordinator to keep the export it has
            timing["redos_skipped"] = timing.get("redos_skipped", 0) + 1
            link.send_export({"redo_of": job.job, "unchanged": True, "forced": sorted(set(force) | set(job.forced)),
                              "err": None})
            job.forced = sorted(set(force) | set(job.forced))
            return job
        if not redo_readers:
            redo_readers.extend(BamReader(p, threads, window_bytes) for p in (tumor_bam, normal_bam))
        prep = JobPrep(job.spec, redo_readers, fasta, windows, secondaries=secondaries, force=force)
        done = Future()
        done.set_result(prep)
        j2 = Job(job.spec, redo_readers, fasta, windows, anonymizer, done)
        exp = j2.exports()
        exp["local_sizes"] = j2.local_sizes()
        exp["err"] = None
        exp["redo_of"] = job.job
        with totals_lock:
            totals[:] += np.asarray(j2.res.totals, np.int64)[:8] - np.asarray(job.res.totals, np.int64)[:8]
        link.send_export(exp)
        j2.release_device()
        return j2

    def finish(job: "Job") -> None:
        if writer_failed.is_set():   # an earlier job failed: its resolution may never come
            return
        try:
            t0 = time.time()
            res = link.recv_resolution()
            while res.get("redo") is not None and res.get("err") is None:
                if res["job"] != job.job:
                    raise RuntimeError(f"redo of job {res['job']} for job {job.job}")
                job = redo(job, res["redo"])
                res = link.recv_resolution()
            timing["wait_s"] += time.time() - t0
            if res.get("err") is not None:
                raise RuntimeError(f"another rank failed: {res['err']}")
            if res["job"] != job.job:
                raise RuntimeError(f"resolution of job {res['job']} for job {job.job}")
            t1 = time.time()
            data = job.output(res["out_n"], res["out_w"], res["ext"], block_size)
            for f in range(4):
                nb = sum(len(x) for x in data[f])
                if nb != res["sizes"][f]:
                    raise RuntimeError(f"job {job.job}: {nb} bytes for file {f}, {res['sizes'][f]} planned")
            # the four files written concurrently (pwrite drops the GIL; a file system serialises
            # buffered writes per file, not across files)
            futs = [file_pool.submit(_pwrite_all, fds[f], data[f], res["offsets"][f]) for f in range(4)
                    if any(len(x) for x in data[f])]
            for fu in futs:
                fu.result()
            stats_rows.append((job.job, job.stats()))
            timing["write_s"] += time.time() - t1
        except BaseException:
            writer_failed.set()
            raise

    def finish_oldest() -> None:
        p = pending.pop(0)
        if writer is None:
            finish(p)
        else:
            t0 = time.time()
            p.result()
            timing["writer_wait_s"] += time.time() - t0

    t_loop0 = time.time()
    timing["setup_s"] = t_loop0 - t_start   # (readers, job plan, exchange groups, inflater, coordinator)
    timing["groups_s"] = timing_groups
    fq0 = dict(native.FQ_TIMES)
    dec0 = DECODE_TIMES["decode_s"]
    try:
        try:
            for i, j in enumerate(mine):
                pre = None
                if pool is not None:
                    submit_upto(i + depth)
                    pre = ahead.pop(j)
                job = Job(jobs[j], readers, fasta, windows, anonymizer, pre, secondaries)
                t_exp0 = time.time()
                exp = job.exports()
                if getattr(job, "speculative", False):   # the permit of a speculative plan
                    t_p = time.time()
                    full = secondaries.forced_for(job.job)
                    timing["permit_check_s"] = timing.get("permit_check_s", 0.0) + time.time() - t_p
                    redo = job.redo_needed(full)
                    secondaries.note_spec(bool(redo))
                    if redo:   # planned again with them, on the redo readers
                        timing["spec_replans"] = timing.get("spec_replans", 0) + 1
                        job.release_device()
                        if not redo_readers:
                            redo_readers.extend(BamReader(p, threads, window_bytes) for p in (tumor_bam, normal_bam))
                        prep = JobPrep(job.spec, redo_readers, fasta, windows, secondaries=secondaries, force=full)
                        done = Future()
                        done.set_result(prep)
                        job = Job(job.spec, redo_readers, fasta, windows, anonymizer, done)
                        exp = job.exports()
                    else:   # (they plan the same here: declared forced, as an unchanged redo would)
                        job.forced = sorted(set(full) | set(job.forced))
                        exp["forced"] = job.forced
                exp["local_sizes"] = job.local_sizes()
                exp["err"] = None
                for k in ("decode_s", "plan_s", "mask_s", "format_s", "prefetch_s"):
                    timing[k] += job.timing[k]
                pp = timing.setdefault("prep_parts", {"decode_wait": 0.0, "plan": 0.0, "batch": 0.0})
                for k, v in zip(("decode_wait", "plan", "batch"), job.prep_parts):
                    pp[k] = round(pp[k] + v, 3)
                timing["jobs"] += 1
                # (job mode: the records starting in the job's range; the margin's belong to its neighbours)
                for t in job.tables:
                    own = slice(None) if job.spec.region is None else \
                        (np.asarray(t.pos) >= job.spec.region[0]) & (np.asarray(t.pos) < job.spec.region[1])
                    timing["reads"] += int(np.count_nonzero(np.ones(t.n, bool)[own]))
                    timing["bases"] += int(np.asarray(t.l_seq)[own].sum(dtype=np.int64))
                with totals_lock:
                    totals[:] += np.asarray(job.res.totals, np.int64)[:8]
                link.send_export(exp)
                job.release_device()
                timing["export_s"] = timing.get("export_s", 0.0) + time.time() - t_exp0
                pending.append(job if writer is None else writer.submit(finish, job))
                while len(pending) >= pend_max:
                    finish_oldest()
            t_drain0 = time.time()
            while pending:
                finish_oldest()
            timing["drain_s"] = time.time() - t_drain0
        except BaseException as e:   # every rank reaches the exchange below with its error
            failure = e
            if xchg is not None:     # plans waiting for this rank's decodes get the error
                xchg.fail(repr(e))
            # the coordinator may be waiting for this rank's next export: tell it
            link.send_export({"err": repr(e)})
            if writer is not None:   # jobs not started yet are dropped; the running one gets the error
                writer_failed.set()
                for p in pending:
                    p.cancel()
                writer.shutdown(wait=True)
                writer = None
        t_tail = time.time()   # (the tail's parts: tail_s below)
        if coord_thread is not None:
            coord_thread.join()
            timing["resolve_s"] = coord.resolve_s
            timing["prunes"] = coord.prunes
            timing["redos"] = coord.redos
            timing["redos_unchanged"] = coord.redos_unchanged
            timing["marked_written"] = coord.marked
            if coord_exc[0] is not None:   # rank 0 reports the coordinator's own error
                failure = coord_exc[0]
        tails = {"coordinator_join": time.time() - t_tail}
        err = repr(failure) if failure is not None else None
        t_tail = time.time()
        if xchg is not None:
            if failure is not None:
                xchg.fail(err)
            xchg.close(None if failure is None else 60.0)
            timing["permit_wait_s"] = round(xchg.wait_s, 3)
        tails["exchange_close"] = time.time() - t_tail
        t_tail = time.time()
        gathered = comm.allgather({"stats": stats_rows, "err": err})
        tails["gather"] = time.time() - t_tail
        t_tail = time.time()
        errs = [g["err"] for g in gathered if g["err"] is not None]
        if errs:
            if failure is not None:
                raise failure
            raise RuntimeError(f"another rank failed: {errs[0]}")
        # every rank ended cleanly: its sends all have their receives (a failed run never drains: a
        # failed rank stops receiving). The side groups serve this process's next run only when every
        # rank drained (one more small gather, so that all ranks cache alike and the next
        # run's new_group calls stay collective)
        drain_err = None
        try:
            link.drain()
        except Exception as e:   # noqa: BLE001
            drain_err = e
        if dist is not None and world > 1:
            drained = comm.allgather(drain_err is None)
            if all(drained):
                from .distributed import return_side_group
                return_side_group(dist, "link", link.group, True)
                if xchg is not None:
                    return_side_group(dist, "secondary", xchg.group, True)
        if drain_err is not None:
            raise drain_err
        all_stats = [g["stats"] for g in gathered]
        if rank == 0 and record_statistics:
            merged: Dict[str, List[int]] = {OUTSIDE_WINDOWS: [0] * 8}
            for _, rows in sorted((x for part in all_stats for x in part), key=lambda t: t[0]):
                for key, counts in rows.items():
                    if key == OUTSIDE_WINDOWS:
                        merged[key] = [a + b for a, b in zip(merged[key], counts)]
                    else:
                        merged[key] = list(counts)
            write_statistics(normal_stats_path or f"{normal_bam}.statistics.txt", merged)
        tails["drain_stats"] = time.time() - t_tail
        t_tail = time.time()
    finally:
        if writer is not None:
            writer.shutdown(wait=True)
        file_pool.shutdown(wait=True)
        if pool is not None:      # prefetches still running (a failed job) end before their reader closes
            for f in ahead.values():
                f.cancel()
            pool.shutdown(wait=True)
            dec_pool.shutdown(wait=True)
        for fd in fds:
            os.close(fd)
        # the readers' file mappings go on a thread of their own (unmapping a chromosome's BAM
        # took part of every rank's tail; nothing waits for it)
        threading.Thread(target=_close_all, args=(list(readers) + list(redo_readers),), daemon=True).start()
        if coord is not None:
            coord.close()
    if "tails" in locals():
        tails["close"] = time.time() - t_tail
        t_tail = time.time()
    timing["exchange_sent_bytes"] = link.sent_bytes
    timing["exchange_recv_bytes"] = link.recv_bytes
    totals = comm.allreduce_totals(totals)
    timing["totals"] = {k: int(v) for k, v in zip(("masked_snv_calls", "masked_bases", "reads_in", "reads_written",
                                                   "scopes", "rare_scopes", "large_tiles", "reserved"), totals)}
    comm.barrier()
    if "tails" in locals():
        tails["totals_barrier"] = time.time() - t_tail
        timing["tail_parts"] = {k: round(v, 3) for k, v in tails.items()}
    # this rank's main thread, stage by stage: what its wall is made of (the thread-time sums above
    # overlap; these do not): waiting for the job's prefetched decode + plan, its mask (batch build
    # included) and format on the device, the export, waiting for a writer slot, the last jobs'
    # writes, then the coordinator, the statistics and the final exchanges
    loop = time.time() - t_loop0
    cp = {"wait_decode_plan": timing["decode_s"] + timing["plan_s"], "mask": timing["mask_s"],
          "format": timing["format_s"], "export": timing.get("export_s", 0.0),
          "wait_writer": timing["writer_wait_s"] - timing.get("drain_s", 0.0), "drain_writes": timing.get("drain_s", 0.0)}
    cp["tail"] = max(0.0, loop - sum(cp.values()))
    timing["critical_path"] = {k: round(v, 3) for k, v in cp.items()}
    # the device formatter's share of "format": record upload, run, download of the bytes
    timing["decode_thread_s"] = round(DECODE_TIMES["decode_s"] - dec0, 3)
    timing["fastq_device"] = {k: round(native.FQ_TIMES[k] - fq0[k], 3) if k != "bytes" else native.FQ_TIMES[k] - fq0[k]
                              for k in native.FQ_TIMES}
    return timing
