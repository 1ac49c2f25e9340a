"""Sample driver: tumor/normal pairs -> anonymized FASTQ (+ statistics).

Mirrors the reference module of the same name (short_read_tumor_normal_anonymizer.py):
``name_output`` (:55-58), ``get_windows`` (:71-131, in planner.py), ``anonymize_genome``
(:625-760) and ``run_short_read_tumor_normal_anonymizer`` (:889-967) with the same
arguments and output files:
  {tumor/normal prefix}.1.fastq / .2.fastq, .single_end.fastq when mates stay unpaired,
  {normal_bam}.statistics.txt with --record_statistics.
By default a sample streams contig by contig with bounded memory (stream.py: per-contig decode,
plan, one device batch, cross-contig pairing resolution, output at the contig's file offsets);
GANON_WHOLE_SAMPLE=1 selects the whole-sample path below (one plan and one device batch for the
sample), kept as the second implementation the tests compare against; a sample with secondary /
supplementary alignments or SA tags (the object model of DESIGN §1c, planned per contig only) goes
to the streamed path from there, which writes the same files.
"""
from __future__ import annotations

import logging
import os
import re
import time
from typing import Dict, List, Sequence, Tuple

from .anonymizer_methods import CompleteGermlineAnonymizer
from .io.bam import ReadTable
from .io.fasta import FastaRef
from .io.vcf import read_vcf
from .planner import UnsupportedInput, Window, get_windows, make_planner
from .writer import statistics_rows, write_fastqs, write_statistics

log = logging.getLogger("genomeanonymizer_amd")


def name_output(sample: str) -> str:
    """SR:55-58 (note: the pattern's '.' matches any character, as in the reference)."""
    return re.sub(".bam|.sam|.cram", ".anonymized", sample)


def has_split_alignments(table: ReadTable) -> bool:
    """Any secondary (0x100) or supplementary (0x800) record or SA tag (the reference's
    AnonymizedRead object model, AM:84-287)."""
    return bool(table.n) and (bool(((table.flag & 0x900) != 0).any()) or bool((table.sa_count() >= 0).any()))


def get_ref_idxs(fasta: FastaRef) -> Dict[str, int]:
    return dict(fasta.index)


def anonymize_genome(windows_in_sample: List[Window], tumor_bam_file: str, normal_bam_file: str,
                     ref_genome_file: str, anonymizer: CompleteGermlineAnonymizer, tumor_output_fastq: str,
                     normal_output_fastq: str, record_statistics: bool, available_threads: int = 8,
                     fasta: FastaRef = None, streaming: bool = None, dist=None) -> dict:
    fasta = fasta or FastaRef(ref_genome_file)
    if streaming is None:
        streaming = os.environ.get("GANON_WHOLE_SAMPLE", "0") != "1"
    if streaming or dist is not None:
        from .stream import anonymize_genome_streaming
        timing = anonymize_genome_streaming(windows_in_sample, tumor_bam_file, normal_bam_file, fasta, anonymizer,
                                            tumor_output_fastq, normal_output_fastq, record_statistics,
                                            available_threads, dist=dist)
        log.info("Anonymization complete for samples %s and %s: %s", tumor_output_fastq, normal_output_fastq,
                 timing)
        return timing
    t0 = time.time()
    tumor = ReadTable(tumor_bam_file, threads=available_threads)
    normal = ReadTable(normal_bam_file, threads=available_threads)
    if has_split_alignments(tumor) or has_split_alignments(normal):
        log.info("secondary / supplementary alignments or SA tags: the sample streams contig by contig")
        del tumor, normal   # (the streamed path decodes job by job: do not hold the whole sample too)
        from .stream import anonymize_genome_streaming
        return anonymize_genome_streaming(windows_in_sample, tumor_bam_file, normal_bam_file, fasta, anonymizer,
                                          tumor_output_fastq, normal_output_fastq, record_statistics,
                                          available_threads)
    t1 = time.time()
    planner = make_planner(tumor, normal, fasta, windows_in_sample)
    try:
        plan = planner.run()
    except UnsupportedInput as e:   # e.g. a duplicated record: the streamed path's object model has it
        log.info("%s: the sample streams contig by contig", e)
        del tumor, normal, planner   # (the whole-sample tables would double the RSS)
        from .stream import anonymize_genome_streaming
        return anonymize_genome_streaming(windows_in_sample, tumor_bam_file, normal_bam_file, fasta, anonymizer,
                                          tumor_output_fastq, normal_output_fastq, record_statistics,
                                          available_threads)
    t2 = time.time()
    res = anonymizer.anonymize(planner, plan)
    t3 = time.time()
    write_fastqs(plan, res, (tumor, normal), (tumor_output_fastq, normal_output_fastq),
                 backend=anonymizer.format_fastq)
    if record_statistics:
        write_statistics(f"{normal_bam_file}.statistics.txt", statistics_rows(plan, res))
    t4 = time.time()
    timing = {"decode_s": t1 - t0, "plan_s": t2 - t1, "mask_s": t3 - t2, "write_s": t4 - t3,
              "reads": int(tumor.n + normal.n), "bases": int(tumor.l_seq.sum() + normal.l_seq.sum()),
              "scopes": len(plan.scopes)}
    log.info("Anonymization complete for samples %s and %s: %s", tumor_output_fastq, normal_output_fastq, timing)
    return timing


def run_short_read_tumor_normal_anonymizer(vcf_variants_per_sample: Sequence[str],
                                           tumor_normal_samples: Sequence[Tuple[str, str]],
                                           ref_genome_file: str, anonymizer: CompleteGermlineAnonymizer,
                                           output_filenames: Sequence[Tuple[str, str]], record_statistics: bool,
                                           cpus: int = 1, enhance_parallelization: bool = False,
                                           dist=None) -> List[dict]:
    """SR:889-967. Several pairs run concurrently like the reference's process pool (SR:944-961):
    min(cpus, pairs) processes (GANON_PAIR_WORKERS overrides; 1 = in turn), each with its own HIP
    context on the anonymizer's device, the host threads split as the reference splits
    ``processes_by_sample``; a pair's own work (decode, plan, mask, format, files) is unchanged.
    One pair, a distributed run or an anonymizer with a custom engine (tests) run in this process.
    The reference's enhanced mode crashes whenever a sample is split; here it is
    accepted and has no effect."""
    if enhance_parallelization:
        log.warning("--enhanced_multiprocessing has no effect in this build (the reference's mode is broken, "
                    "SURVEY Q12)")
    fasta = FastaRef(ref_genome_file)
    ref_idx = get_ref_idxs(fasta)
    inputs = []
    for vcf, samples, outs in zip(vcf_variants_per_sample, tumor_normal_samples, output_filenames):
        inputs.append((get_windows(read_vcf(vcf), ref_idx), samples, outs))
    workers = int(os.environ.get("GANON_PAIR_WORKERS", str(min(max(1, int(cpus)), len(inputs)))))
    if workers > 1 and len(inputs) > 1 and dist is None and getattr(anonymizer, "_engine", None) is None:
        import multiprocessing as mp
        from concurrent.futures import ProcessPoolExecutor
        # (processes_by_sample, SR:945-946)
        threads = 1 if cpus <= len(inputs) else max(1, int(cpus) // len(inputs))
        # spawned: a forked child of a process that touched the GPU cannot use it
        with ProcessPoolExecutor(max_workers=min(workers, len(inputs)), mp_context=mp.get_context("spawn")) as ex:
            futs = [ex.submit(_anonymize_pair, windows, t_bam, n_bam, ref_genome_file, anonymizer.device, t_out, n_out,
                              record_statistics, threads)
                    for windows, (t_bam, n_bam), (t_out, n_out) in inputs]
            return [f.result() for f in futs]
    timings = []
    for windows, (t_bam, n_bam), (t_out, n_out) in inputs:
        timings.append(anonymize_genome(windows, t_bam, n_bam, ref_genome_file, anonymizer, t_out, n_out,
                                        record_statistics, max(1, int(cpus)), fasta=fasta, dist=dist))
    return timings


def _anonymize_pair(windows, t_bam, n_bam, ref_genome_file, device, t_out, n_out, record_statistics, threads) -> dict:
    """One pair in a pool process (its own HIP context on ``device``)."""
    anon = CompleteGermlineAnonymizer(device=device)
    try:
        return anonymize_genome(windows, t_bam, n_bam, ref_genome_file, anon, t_out, n_out, record_statistics, threads)
    finally:
        eng = getattr(anon, "_engine", None)
        if eng is not None and hasattr(eng, "close"):
            eng.close()
