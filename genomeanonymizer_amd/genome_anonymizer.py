"""Command line, same flags as the reference (genome_anonymizer.py:16-112):

  python -m genomeanonymizer_amd.genome_anonymizer -d DIR -s samples.tsv -r ref.fa \\
      [-m complete_germline] [-c CPUS] [--record_statistics] [--enhanced_multiprocessing] [-v N]

samples.tsv: tumor<TAB>normal<TAB>vcf per line, paths relative to DIR, '#' lines skipped.
Outputs next to the inputs: re.sub('.bam|.sam|.cram', '.anonymized', path) + .1/.2.fastq
(+ .single_end.fastq), and {normal_bam}.statistics.txt with --record_statistics.

Multi-GPU: launch under ``torchrun --nproc-per-node N`` (or set WORLD_SIZE/RANK/LOCAL_RANK):
contigs are sharded round-robin over the ranks; each rank decodes, masks and writes its own
contigs at their offsets of the shared output files (distributed.py, stream.py). More ranks than
GPUs (e.g. 4 per GPU) spread the host work (decode, planning, output) over more processes: rank r
uses GPU LOCAL_RANK % GPUs and the ranks talk over gloo instead of RCCL.
"""
from __future__ import annotations

import logging
import os
import sys
import time
from argparse import ArgumentParser, BooleanOptionalAction
from typing import List, Tuple

from .anonymizer_methods import ANONYMIZER_ALGORITHMS, CompleteGermlineAnonymizer
from .short_read_tumor_normal_anonymizer import name_output, run_short_read_tumor_normal_anonymizer

COMPLETE_GERMLINE_ANONYMIZER_ALGORITHM = "complete_germline"


def exec_parser(argv=None):
    parser = ArgumentParser(prog="GenomeAnonymizer",
                            description="Anonymization of sequencing data by removing germline variation "
                                        "(MI355X build)")
    parser.add_argument("-d", "--directory", type=str, required=True,
                        help="Directory in which the tumor-normal sample pairs and the samples text file are stored")
    parser.add_argument("-s", "--samples", type=str, required=True,
                        help="Text file with the tumor, normal and vcf file names of each sample, tab separated")
    parser.add_argument("-r", "--reference", type=str, required=True,
                        help="reference genome to which the reads are mapped")
    parser.add_argument("-m", "--method", type=str, required=False, default="complete_germline",
                        choices=["complete_germline"],
                        help="anonymization method: complete_germline masks all germline SNVs in the reads")
    parser.add_argument("-c", "--cpu", type=int, required=False, default=1,
                        help="Number of CPUs available (host BAM decode threads)")
    parser.add_argument("--record_statistics", action=BooleanOptionalAction,
                        help="Record statistics about the number of anonymized variants by region and type")
    parser.add_argument("--enhanced_multiprocessing", action=BooleanOptionalAction,
                        help="Accepted for compatibility; no effect (see SURVEY Q12)")
    parser.add_argument("-v", "--verbose", type=int, required=False, default=2, help="Verbosity of logging")
    parser.add_argument("--device", type=int, default=None, help="GPU index (default: LOCAL_RANK or 0)")
    return parser.parse_args(argv)


def join_dir_file(directory: str, param: str) -> str:
    return "".join((directory, "/", param)) if not directory.endswith("/") else "".join((directory, param))


def read_samples(path_to_samples: str, directory: str):
    samples: List[Tuple[str, str]] = []
    outputs: List[Tuple[str, str]] = []
    vcfs: List[str] = []
    with open(path_to_samples) as fh:
        for line in fh:
            if line.startswith("#"):
                continue
            f = line.strip().split("\t")
            t, n, v = (join_dir_file(directory, x) for x in f[:3])
            samples.append((t, n))
            vcfs.append(v)
            outputs.append((name_output(t), name_output(n)))
    return vcfs, samples, outputs


def run_anonymizer(argv=None) -> None:
    config = exec_parser(argv)
    logging.basicConfig(level=config.verbose * 10)
    t0 = time.time()
    logging.info("Beginning execution of GenomeAnonymizer (MI355X build)")
    if config.method not in ANONYMIZER_ALGORITHMS:
        logging.error("Anonymizer algorithm %s is not a valid option", config.method)
        sys.exit(1)
    vcfs, samples, outputs = read_samples(join_dir_file(config.directory, config.samples), config.directory)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    # launched by torchrun (any world size, one included): the process-group path
    launched = world > 1 or ("RANK" in os.environ and "MASTER_ADDR" in os.environ)
    n_dev = 1
    if launched:
        import torch
        n_dev = max(1, torch.cuda.device_count())   # (counting devices does not initialise the GPU)
    device = config.device if config.device is not None else local % n_dev
    anonymizer = CompleteGermlineAnonymizer(device=device)
    if launched:
        import torch.distributed as dist
        from .distributed import run_pairs_sharded
        if local_world > n_dev:   # ranks share a GPU: RCCL takes one rank per device
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(device)
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        logging.info("rank %d of %d: process group backend %s", dist.get_rank(), dist.get_world_size(),
                     dist.get_backend())
        # one pair per GPU when there are enough pairs, else each pair's contigs over all GPUs
        tots = run_pairs_sharded(vcfs, samples, config.reference, anonymizer, outputs, bool(config.record_statistics),
                                 dist, threads=max(1, config.cpu))
        logging.info("rank %d totals %s", dist.get_rank(), tots)
        from .distributed import release_side_groups
        release_side_groups(dist)
        dist.destroy_process_group()
    else:
        run_short_read_tumor_normal_anonymizer(vcfs, samples, config.reference, anonymizer, outputs,
                                               bool(config.record_statistics), config.cpu,
                                               bool(config.enhanced_multiprocessing))
    logging.info("Finished execution of GenomeAnonymizer successfully")
    logging.debug("Total execution time: %s s", time.time() - t0)


if __name__ == "__main__":
    run_anonymizer()
