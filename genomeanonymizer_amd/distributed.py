"""Multi-GPU execution of one tumor/normal pair: contigs sharded over the ranks.

Scopes never cross contigs, so the masking shards with no data-path
collective: every rank (one process per GPU, torchrun) decodes the inputs and runs the same
deterministic host plan, masks the scopes of the contigs it owns on its own GPU, and hands
its masked reads to rank 0 through a shard file in ``workdir``. The only collective is the
all-reduce of the int64 totals (masked calls / masked bases / reads...) — RCCL over xGMI
with the ``nccl`` backend, gloo in the CPU tests. Rank 0 writes the FASTQ and statistics
files exactly as the single-GPU path does (contig order, cross-contig mates, single ends:
short_read_tumor_normal_anonymizer.py:625-760).

Contig -> rank assignment: ``round_robin`` over FASTA order (the north star's policy) or
``lpt`` (longest-processing-time first by the number of scope incidences; the default).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Sequence

import numpy as np

from .anonymizer_methods import CompleteGermlineAnonymizer, MaskResult
from .indels import IndelCall
from .io.bam import ReadTable
from .io.fasta import FastaRef
from .planner import Plan, Window, make_planner
from .variants import VariantType
from .writer import statistics_rows, write_fastqs, write_statistics


def contig_owner(plan: Plan, contigs: Sequence[str], world: int, policy: str = "lpt") -> Dict[str, int]:
    if policy == "round_robin":
        return {c: i % world for i, c in enumerate(contigs)}
    load = {c: 0 for c in contigs}
    for sc in plan.scopes:
        load[sc.contig] += len(sc.t_rows) + len(sc.n_rows)
    bins = [0] * world
    owner = {}
    for c in sorted(contigs, key=lambda c: (-load[c], contigs.index(c))):
        r = int(np.argmin(bins))
        owner[c] = r
        bins[r] += load[c]
    return owner


def _read_byte_index(tables, seq_base, ds: np.ndarray, row: np.ndarray) -> np.ndarray:
    """Indices into the batch's sequence blob of every packed byte of the reads (ds, row), read
    after read."""
    T, N = tables
    ds = np.asarray(ds, np.int64)
    row = np.asarray(row, np.int64)
    t0 = ds == 0
    r0, r1 = np.where(t0, row, 0), np.where(t0, 0, row)
    start = np.where(t0, seq_base[0] + T.seq_off[r0], seq_base[1] + N.seq_off[r1]).astype(np.int64)
    n = (np.where(t0, T.l_seq[r0], N.l_seq[r1]).astype(np.int64) + 1) // 2
    if len(n) == 0:
        return np.zeros(0, np.int64)
    first = np.concatenate([[0], np.cumsum(n)[:-1]])
    return np.repeat(start - first, n) + np.arange(int(n.sum()), dtype=np.int64)


def _edits_to_json(edits):
    return [[irp, c.pos, c.end, c.variant_type.value, c.length, c.allele, c.ref_allele] for irp, c in edits]


def _edits_from_json(items):
    return [(e[0], IndelCall(e[1], e[2], VariantType(e[3]), e[4], e[5], e[6])) for e in items]


def anonymize_genome_sharded(windows: List[Window], tumor_bam: str, normal_bam: str, ref_file: str,
                             tumor_out: str, normal_out: str, record_statistics: bool, rank: int, world: int,
                             workdir: str, anonymizer: CompleteGermlineAnonymizer = None, dist=None,
                             policy: str = "lpt", threads: int = 8) -> dict:
    """Run one sample on ``world`` ranks. ``dist`` is torch.distributed (already
    initialised) or None for a single rank. Returns the all-reduced totals."""
    anonymizer = anonymizer or CompleteGermlineAnonymizer(device=int(os.environ.get("LOCAL_RANK", 0)))
    fasta = FastaRef(ref_file)
    tables = plan = res = None
    failure = None
    try:
        tables = (ReadTable(tumor_bam, threads=threads), ReadTable(normal_bam, threads=threads))
        planner = make_planner(tables[0], tables[1], fasta, windows)
        plan = planner.run()
        owner = contig_owner(plan, list(fasta.references), world, policy)
        mine = [sc.id for sc in plan.scopes if owner[sc.contig] == rank]
        res = anonymizer.anonymize(planner, plan, scope_ids=mine)
        mine_set = set(mine)
        # this rank's written reads and their masked bytes (column arrays, no per-record Python)
        w_ds, w_row, w_sc = plan.written_arrays()
        sel = (w_sc >= 0) & np.isin(w_sc, np.fromiter(mine_set, np.int64, len(mine_set)))
        recs = np.stack([w_ds[sel], w_row[sel], w_sc[sel]], axis=1).astype(np.int64).reshape(-1, 3)
        idx = _read_byte_index(tables, res.seq_base, recs[:, 0], recs[:, 1])
        os.makedirs(workdir, exist_ok=True)
        shard = os.path.join(workdir, f"shard{rank}")
        np.savez(shard + ".npz", recs=recs, seq=res.seq_out[idx],
                 calls=res.scope_snv_calls, bases=res.scope_masked_bases, totals=res.totals)
        with open(shard + ".json", "w") as fh:
            json.dump({"indel_counts": {str(s): {vt.name: n for vt, n in c.items()}
                                        for s, c in res.scope_indel_counts.items()},
                       "leftovers": [[k[0], k[1], k[2], _edits_to_json(v)] for k, v in res.leftovers.items()]}, fh)
        totals = res.totals.astype(np.int64)
    except Exception as e:   # every rank must reach the collectives below, or the others hang
        failure = e
        totals = np.zeros(8, np.int64)
    if dist is not None:
        import torch
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
        flag = torch.tensor([1 if failure is not None else 0], dtype=torch.int64, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if int(flag.item()):
            if failure is not None:
                raise failure
            raise RuntimeError("anonymize_genome_sharded: another rank failed")
        tt = torch.from_numpy(totals.copy()).to(dev)
        dist.all_reduce(tt)
        totals = tt.cpu().numpy()
        dist.barrier()
    elif failure is not None:
        raise failure
    if rank == 0:
        merged = _merge_shards(plan, tables, res, workdir, world)
        write_fastqs(plan, merged, tables, (tumor_out, normal_out), backend=anonymizer.format_fastq)
        if record_statistics:
            write_statistics(f"{normal_bam}.statistics.txt", statistics_rows(plan, merged))
    if dist is not None:
        dist.barrier()
    return {k: int(v) for k, v in zip(("masked_snv_calls", "masked_bases", "reads_in", "reads_written", "scopes",
                                       "rare_scopes", "large_tiles", "reserved"), totals)}


def _merge_shards(plan: Plan, tables, res0: MaskResult, workdir: str, world: int) -> MaskResult:
    T, N = tables
    seq_out = np.concatenate([T.seq, N.seq]).astype(np.uint8)
    calls = np.zeros(len(plan.scopes), np.int32)
    bases = np.zeros(len(plan.scopes), np.int32)
    indel_counts, leftovers = {}, {}
    for r in range(world):
        z = np.load(os.path.join(workdir, f"shard{r}.npz"))
        calls += z["calls"]
        bases += z["bases"]
        zr = z["recs"]
        seq_out[_read_byte_index(tables, res0.seq_base, zr[:, 0], zr[:, 1])] = z["seq"]
        with open(os.path.join(workdir, f"shard{r}.json")) as fh:
            j = json.load(fh)
        for s, c in j["indel_counts"].items():
            indel_counts[int(s)] = {VariantType[k]: v for k, v in c.items()}
        for ds, row, s, e in j["leftovers"]:
            leftovers[(ds, row, s)] = _edits_from_json(e)
    return MaskResult(seq_out, res0.seq_base, {}, calls, bases, indel_counts, leftovers, res0.totals, {})
