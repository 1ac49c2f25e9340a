"""Multi-GPU execution of one tumor/normal pair: contigs sharded over the ranks.

Scopes never cross contigs, so the masking shards with no data-path collective.
One process per GPU (torchrun); rank r takes the FASTA contigs r, r + world, r + 2·world, ...
(round-robin in FASTA order, the north star's policy) and decodes (region reads through the BAM
index), plans, masks, formats and writes only those, on its own GPU — stream.py. Per round of
``world`` contigs the ranks exchange on the host (gloo) only what crosses contigs: the
pairing operations of reads whose mate lies on another sequence, the FASTQ bytes of the records
those may still write, and their byte counts, so every rank places its contig's bytes at the right
offset of the shared output files itself. The int64 totals (masked calls / bases / reads...) are
all-reduced once at the end — RCCL over xGMI on the default ``nccl`` group. The reference runs
pairs in parallel instead (short_read_tumor_normal_anonymizer.py:944-961).
"""
from __future__ import annotations

import os
from typing import List

from .anonymizer_methods import CompleteGermlineAnonymizer
from .io.fasta import FastaRef
from .planner import Window
from .stream import anonymize_genome_streaming


def contig_owner(contigs: List[str], world: int) -> dict:
    """Round-robin over FASTA order: the rank of each contig."""
    return {c: i % world for i, c in enumerate(contigs)}


def anonymize_genome_sharded(windows: List[Window], tumor_bam: str, normal_bam: str, ref_file: str,
                             tumor_out: str, normal_out: str, record_statistics: bool,
                             anonymizer: CompleteGermlineAnonymizer = None, dist=None, threads: int = 8) -> dict:
    """Run one sample on the ranks of ``dist`` (torch.distributed, initialised; None = one rank).
    Returns the all-reduced totals."""
    anonymizer = anonymizer or CompleteGermlineAnonymizer(device=int(os.environ.get("LOCAL_RANK", 0)))
    timing = anonymize_genome_streaming(windows, tumor_bam, normal_bam, FastaRef(ref_file), anonymizer, tumor_out,
                                        normal_out, record_statistics, threads, dist=dist)
    return timing["totals"]
