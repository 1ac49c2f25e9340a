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

import os
import pickle
import queue
from typing import List, Sequence

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
        self.group = dist.new_group(backend="gloo") if dist is not None and self.world > 1 else None
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
