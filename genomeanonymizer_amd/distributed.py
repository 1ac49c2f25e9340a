"""Multi-GPU execution of tumor/normal pairs: contig shards of one pair, or one pair per rank.

Scopes never cross contigs, so the masking shards with no data-path collective.
One process per GPU (torchrun). Two shard levels:

* several pairs and at least as many pairs as ranks: rank r runs pairs r, r + world, ... whole
  (the reference's own parallelism, one ProcessPoolExecutor task per pair,
  short_read_tumor_normal_anonymizer.py:944-961), each streamed on its own GPU with no exchange;
* otherwise the contigs of a pair are sharded (``assign_contigs``: round-robin in FASTA order, the
  north star's policy, or longest-processing-time-first by contig length, GANON_SHARD=lpt). Each
  rank decodes, plans, masks and formats its contigs in FASTA order on its own GPU with no
  lock-step: it sends what crosses contigs (the pairing operations of reads whose mate lies on
  another sequence and the FASTQ bytes of the records those may write) to rank 0 only, where a
  coordinator thread resolves the contigs in FASTA order as they arrive and answers the owner with
  its placeholder writes, the bytes of the records it writes from other contigs and the offsets of
  its bytes in the four output files; the owner writes there itself (stream.py). ``Link`` carries
  those messages (gloo point to point, queues inside rank 0).

The int64 totals (masked calls / bases / reads...) are all-reduced once at the end: RCCL over xGMI
on the default ``nccl`` group.
"""
from __future__ import annotations

import atexit
import os
import pickle
import queue
import threading
from typing import Dict, List, Optional, Sequence

import numpy as np

from .anonymizer_methods import CompleteGermlineAnonymizer
from .io.fasta import FastaRef
from .planner import Window


def assign_contigs(lengths: Sequence[int], world: int, policy: str = None) -> List[int]:
    """Owner rank of each contig. ``round_robin`` (default): contig i -> i % world. ``lpt``: longest
    contig first to the least loaded rank (load = summed contig length, ties to the lower rank) —
    within 4/3 of the best makespan for independent jobs; an hg38-like list (one chr1 per 3 Gb) caps
    round-robin at ~0.7 efficiency on 8 ranks."""
    policy = (policy or os.environ.get("GANON_SHARD", "round_robin")).lower()
    n = len(lengths)
    if world <= 1:
        return [0] * n
    if policy == "round_robin":
        return [i % world for i in range(n)]
    if policy != "lpt":
        raise ValueError(f"unknown contig shard policy {policy!r} (round_robin, lpt)")
    owner = [0] * n
    load = np.zeros(world, np.int64)
    for i in sorted(range(n), key=lambda k: (-int(lengths[k]), k)):
        r = int(np.argmin(load))
        owner[i] = r
        load[r] += int(lengths[i])
    return owner


def assign_samples(n_samples: int, world: int) -> List[int]:
    """Pairs to ranks when each rank runs whole pairs: round-robin."""
    return [i % max(1, world) for i in range(n_samples)]


# Side gloo groups of the streamed path (Link, SecondaryExchange), kept for the next run of this
# process once a run has ended cleanly on every rank: creating one took 0.13-0.33 s per rank and run
# on the 8-rank chromosome-scale line (`groups_s`), ~10 % of its wall. Keyed by purpose and the
# default process group (a group of a destroyed world is never reused); a run that failed anywhere
# returns nothing, so the next run makes fresh groups and no message of the failed one is left to
# meet it. Every rank takes and returns the same groups in the same order (the error state it
# returns on is the run's final all-gathered one), so new_group stays collective.
_SIDE_GROUPS: dict = {}


def _world_key(dist):
    try:
        pg = dist.distributed_c10d._get_default_group()
    except Exception:   # pragma: no cover
        pg = None
    return id(pg), pg


def release_side_groups(dist=None, stale_only_for=None) -> None:
    """Destroy the cached side groups (all of them, or those not of world key ``stale_only_for``). Called
    before the default group goes (genome_anonymizer.py, tools/e2e_bench.py) and at exit: a cached
    gloo group left to the interpreter's teardown destroyed its threads while joinable
    ("terminate called without an active exception" after a clean 8-rank run, round 6)."""
    if dist is None:
        try:
            import torch.distributed as dist
        except Exception:   # pragma: no cover
            return
    for key in list(_SIDE_GROUPS):
        if stale_only_for is not None and key[1] == stale_only_for:
            continue
        group, _ = _SIDE_GROUPS.pop(key)
        try:
            dist.destroy_process_group(group)
        except Exception:   # noqa: BLE001  (its world is gone already)
            pass


atexit.register(release_side_groups)


def take_side_group(dist, purpose: str):
    k, _ = _world_key(dist)
    # groups cached under another (destroyed) world are released: they are never reused
    release_side_groups(dist, stale_only_for=k)
    hit = _SIDE_GROUPS.pop((purpose, k), None)
    return hit[0] if hit is not None else dist.new_group(backend="gloo")


def return_side_group(dist, purpose: str, group, clean: bool) -> None:
    if group is None or not clean:
        return
    k, pg = _world_key(dist)
    _SIDE_GROUPS[(purpose, k)] = (group, pg)   # (pg kept: its id cannot be reused while cached)


class Link:
    """Messages between each rank's worker (its main thread) and the coordinator (a thread of rank
    0): exports go to rank 0, resolutions come back to the job's owner, in job order per rank (FIFO
    per pair of ranks). Rank 0's own worker talks to its coordinator through queues; the other ranks
    through a dedicated gloo group (pickled objects as uint8 tensors, a length message first).
    Sends never block (isend): a worker keeps masking while its exports travel."""

    EXPORT, RESOLUTION = 11, 12

    def __init__(self, dist=None):
        self.dist = dist
        self.rank = dist.get_rank() if dist is not None else 0
        self.world = dist.get_world_size() if dist is not None else 1
        self.group = take_side_group(dist, "link") if dist is not None and self.world > 1 else None
        self.q_exp: "queue.Queue" = queue.Queue()
        self.q_res: "queue.Queue" = queue.Queue()
        self._inflight: list = []
        self.sent_bytes = 0       # pickled payload bytes this rank sent / received over gloo
        self.recv_bytes = 0

    def _send(self, obj, dst: int, tag: int) -> None:
        import torch
        payload = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
        self.sent_bytes += len(payload)
        n = torch.tensor([len(payload)], dtype=torch.int64)
        t = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
        w1 = self.dist.isend(n, dst, group=self.group, tag=tag)
        w2 = self.dist.isend(t, dst, group=self.group, tag=tag)
        self._inflight.append((w1, w2, n, t))
        # completed sends release their buffers
        self._inflight = [x for x in self._inflight if not (x[0].is_completed() and x[1].is_completed())]

    def _recv(self, src: int, tag: int):
        import torch
        n = torch.zeros(1, dtype=torch.int64)
        self.dist.recv(n, src, group=self.group, tag=tag)
        t = torch.empty(int(n.item()), dtype=torch.uint8)
        self.dist.recv(t, src, group=self.group, tag=tag)
        self.recv_bytes += int(n.item())
        return pickle.loads(t.numpy().tobytes())

    # worker side
    def send_export(self, exp: dict) -> None:
        if self.rank == 0:
            self.q_exp.put(exp)
        else:
            self._send(exp, 0, self.EXPORT)

    def recv_resolution(self) -> dict:
        return self.q_res.get() if self.rank == 0 else self._recv(0, self.RESOLUTION)

    # coordinator side (rank 0)
    def recv_export(self, owner: int) -> dict:
        return self.q_exp.get() if owner == 0 else self._recv(owner, self.EXPORT)

    def send_resolution(self, owner: int, res: dict) -> None:
        if owner == 0:
            self.q_res.put(res)
        else:
            self._send(res, owner, self.RESOLUTION)

    def drain(self) -> None:
        """Wait for every send (a normal end: each has its matching receive)."""
        for w1, w2, _, _ in self._inflight:
            w1.wait()
            w2.wait()
        self._inflight = []


class SecondaryExchange:
    """Off-contig secondary alignments published across ranks before any job is planned (round 5;
    ADVICE r04: without it, a job whose mate-side names another rank's later decode forced was planned,
    masked and formatted again — serially, while the coordinator waited: on a 4-rank CPU probe with 1 %
    of the pairs carrying such a secondary, 2 of 3 jobs were planned twice and the run took 4x the
    one-process wall).

    Every rank reports each of its jobs once its decode thread has read it (DECODED: the job's
    (name, mate job) secondaries, or an error) to rank 0, whose registry keeps the decode frontier —
    the first job not decoded yet — and the secondaries by mate job. Job j may be planned once every
    job before it is decoded (only an earlier job's secondary can force a name on j: a later one's is
    marked written by the coordinator instead): rank 0 then sends j's owner a PERMIT with the names to
    plan as cross names. Each job is reported exactly once (a failing rank reports its remaining jobs
    as errors) and permitted exactly once (after an error, every job not permitted yet gets the error),
    so every receive has its send. Ranks couple only through their decode progress."""

    DECODED, PERMIT = 13, 14

    def __init__(self, dist, owner: Sequence[int]):
        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.group = take_side_group(dist, "secondary")
        self.owner = list(owner)
        self.n = len(owner)
        self.mine = [j for j in range(self.n) if owner[j] == self.rank]
        # locks: report_lock (the reported set), reg_lock (rank 0's registry; taken before io_lock),
        # io_lock (a leaf: isends and their in-flight list)
        self.report_lock = threading.Lock()
        self.io_lock = threading.Lock()
        self.reported: set = set()
        self._inflight: list = []
        self.cv = threading.Condition()
        self.permits: Dict[int, object] = {}
        self.threads: List[threading.Thread] = []
        self.wait_s = 0.0
        if self.rank == 0:
            self.reg_lock = threading.Lock()
            self.decoded = [False] * self.n
            self.frontier = 0
            self.next_permit = 0
            self.failed: Optional[str] = None
            self.by_mate: Dict[int, Dict[bytes, int]] = {}
            with self.reg_lock:
                self._advance()
            for r in range(1, self.world):
                cnt = sum(1 for o in owner if o == r)
                if cnt:
                    self.threads.append(threading.Thread(target=self._receive_reports, args=(r, cnt), daemon=True,
                                                         name=f"ganon-secx-{r}"))
        elif self.mine:
            self.threads.append(threading.Thread(target=self._receive_permits, daemon=True, name="ganon-secx-permits"))
        for t in self.threads:
            t.start()

    # transport (pickled objects as uint8 tensors, a length message first; as Link)
    def _send(self, obj, dst: int, tag: int) -> None:
        import torch
        payload = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
        n = torch.tensor([len(payload)], dtype=torch.int64)
        t = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
        with self.io_lock:
            w1 = self.dist.isend(n, dst, group=self.group, tag=tag)
            w2 = self.dist.isend(t, dst, group=self.group, tag=tag)
            self._inflight.append((w1, w2, n, t))
            self._inflight = [x for x in self._inflight if not (x[0].is_completed() and x[1].is_completed())]

    def _recv(self, src: int, tag: int):
        import torch
        n = torch.zeros(1, dtype=torch.int64)
        self.dist.recv(n, src, group=self.group, tag=tag)
        t = torch.empty(int(n.item()), dtype=torch.uint8)
        self.dist.recv(t, src, group=self.group, tag=tag)
        return pickle.loads(t.numpy().tobytes())

    # worker side
    def report(self, job: int, pairs) -> None:
        """Job ``job`` decoded (its decode thread): its secondaries whose mate another job reads."""
        self._report({"job": job, "pairs": list(pairs)})

    def fail(self, err: str) -> None:
        """This rank failed: every job of it not reported yet is reported as the error."""
        for j in self.mine:
            self._report({"job": j, "err": err})

    def _report(self, msg: dict) -> None:
        with self.report_lock:
            if msg["job"] in self.reported:
                return
            self.reported.add(msg["job"])
        if self.rank == 0:
            with self.reg_lock:
                self._on_report(msg)
        else:
            self._send(msg, 0, self.DECODED)

    def permit(self, job: int) -> List[bytes]:
        """Block until every job before ``job`` is decoded (on any rank); the names of the secondaries
        of earlier jobs whose mate ``job`` reads. Raises when a rank failed first, when this rank's
        receiver thread failed (it delivers its error), or after GANON_PERMIT_TIMEOUT seconds (1800)."""
        import time
        t0 = time.time()
        limit = float(os.environ.get("GANON_PERMIT_TIMEOUT", "1800"))
        with self.cv:
            while job not in self.permits:
                left = limit - (time.time() - t0)
                if left <= 0:
                    raise RuntimeError(f"secondary exchange: no permit for job {job} after {limit:.0f} s")
                self.cv.wait(left)
            v = self.permits.pop(job)
        self.wait_s += time.time() - t0
        if isinstance(v, str):
            raise RuntimeError(f"another rank failed: {v}")
        return v

    def _deliver(self, msg: dict) -> None:
        with self.cv:
            self.permits[msg["job"]] = msg["err"] if msg.get("err") is not None else msg["names"]
            self.cv.notify_all()

    def _receive_permits(self) -> None:
        got = set()
        try:
            for _ in self.mine:
                msg = self._recv(0, self.PERMIT)
                got.add(msg["job"])
                self._deliver(msg)
        except Exception as e:   # noqa: BLE001  (a daemon thread: its error must reach permit())
            err = f"secondary exchange: receiving permits failed: {e!r}"
            for j in self.mine:
                if j not in got:
                    self._deliver({"job": j, "err": err})

    # registry (rank 0)
    def _receive_reports(self, r: int, cnt: int) -> None:
        try:
            for _ in range(cnt):
                msg = self._recv(r, self.DECODED)
                with self.reg_lock:
                    self._on_report(msg)
        except Exception as e:   # noqa: BLE001  (every job not permitted yet gets the error)
            with self.reg_lock:
                self.failed = self.failed or f"secondary exchange: reports of rank {r} lost: {e!r}"
                self._advance()

    def _on_report(self, msg: dict) -> None:   # (reg_lock held)
        if msg.get("err") is not None:
            self.failed = self.failed or msg["err"]
        else:
            self.decoded[msg["job"]] = True
            for nm, mj in msg["pairs"]:
                d = self.by_mate.setdefault(int(mj), {})
                if d.get(nm, 1 << 62) > msg["job"]:
                    d[nm] = msg["job"]
        self._advance()

    def _advance(self) -> None:
        while self.frontier < self.n and self.decoded[self.frontier]:
            self.frontier += 1
        while self.next_permit < self.n and (self.failed is not None or self.next_permit <= self.frontier):
            j = self.next_permit
            self.next_permit += 1
            if self.failed is not None:
                msg = {"job": j, "err": self.failed}
            else:
                msg = {"job": j, "names": sorted(nm for nm, src in self.by_mate.get(j, {}).items() if src < j)}
            if self.owner[j] == 0:
                self._deliver(msg)
            elif self.failed is not None:
                try:    # (the transport may be what failed: the owner's receiver then fails on its own)
                    self._send(msg, self.owner[j], self.PERMIT)
                except Exception:   # noqa: BLE001
                    pass
            else:
                self._send(msg, self.owner[j], self.PERMIT)

    def close(self, timeout: Optional[float] = None) -> None:
        """Join the receiving threads and wait for every send (a normal end: each has its receive)."""
        for t in self.threads:
            t.join(timeout)
        if timeout is None:
            with self.io_lock:
                for w1, w2, _, _ in self._inflight:
                    w1.wait()
                    w2.wait()
                self._inflight = []


def anonymize_genome_sharded(windows: List[Window], tumor_bam: str, normal_bam: str, ref_file: str,
                             tumor_out: str, normal_out: str, record_statistics: bool,
                             anonymizer: CompleteGermlineAnonymizer = None, dist=None, threads: int = 8) -> dict:
    """Run one sample on the ranks of ``dist`` (torch.distributed, initialised; None = one rank).
    Returns the all-reduced totals."""
    from .stream import anonymize_genome_streaming
    anonymizer = anonymizer or CompleteGermlineAnonymizer(device=int(os.environ.get("LOCAL_RANK", 0)))
    timing = anonymize_genome_streaming(windows, tumor_bam, normal_bam, FastaRef(ref_file), anonymizer, tumor_out,
                                        normal_out, record_statistics, threads, dist=dist)
    global LAST_TIMING
    LAST_TIMING = timing
    return timing["totals"]


LAST_TIMING: dict = {}   # the stage timing of this process's last anonymize_genome_sharded (tests, tools)


def run_pairs_sharded(vcfs: Sequence[str], samples: Sequence[tuple], ref_file: str,
                      anonymizer: CompleteGermlineAnonymizer, outputs: Sequence[tuple], record_statistics: bool,
                      dist, threads: int = 8) -> List[dict]:
    """Every tumor/normal pair of a run over the ranks of ``dist``: with at least as many pairs as
    ranks, rank r runs pairs r, r + world, ... whole on its own GPU (the reference's one task per
    pair, SR:944-961; no exchange until the final error check); with fewer, each pair's contigs are
    sharded over all ranks (anonymize_genome_sharded). Returns this rank's per-pair totals."""
    from .io.vcf import read_vcf
    from .planner import get_windows
    from .stream import anonymize_genome_streaming
    rank, world = dist.get_rank(), dist.get_world_size()
    fa = FastaRef(ref_file)
    out: List[dict] = []
    if len(samples) >= world:
        owner = assign_samples(len(samples), world)
        err = None
        for i, (vcf, (t, n), (to, no)) in enumerate(zip(vcfs, samples, outputs)):
            if owner[i] != rank or err is not None:
                continue
            try:
                windows = get_windows(read_vcf(vcf), fa.index)
                timing = anonymize_genome_streaming(windows, t, n, fa, anonymizer, to, no, record_statistics, threads)
                out.append(timing["totals"])
            except BaseException as e:   # every rank reaches the check below
                err = e
        group = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else None
        flags = [None] * world
        dist.all_gather_object(flags, repr(err) if err is not None else None, group=group)
        if err is not None:
            raise err
        bad = [f for f in flags if f is not None]
        if bad:
            raise RuntimeError(f"another rank failed: {bad[0]}")
        return out
    for vcf, (t, n), (to, no) in zip(vcfs, samples, outputs):
        windows = get_windows(read_vcf(vcf), fa.index)
        out.append(anonymize_genome_sharded(windows, t, n, ref_file, to, no, record_statistics, anonymizer, dist,
                                            threads))
    return out
