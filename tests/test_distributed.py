"""The N>1 path (round-robin contig shards, one process per rank, each decoding, planning,
masking and writing its own contigs; per-round gloo exchange of the cross-contig pairing state;
totals all-reduce) on CPU with gloo: two ranks must write exactly the reference's files. The CPU
oracle stands in for the GPU (test infrastructure); tests/test_gpu_distributed.py runs the HIP
engine."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, workdir, q, engine="oracle", fail_rank=-1, fail_stage="job"):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "oracle"), os.path.join(repo, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pyoracle import OracleEngine
        from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
        from genomeanonymizer_amd.distributed import anonymize_genome_sharded
        from genomeanonymizer_amd.io.fasta import FastaRef
        from genomeanonymizer_amd.io.vcf import read_vcf
        from genomeanonymizer_amd.planner import get_windows
        from genomeanonymizer_amd.short_read_tumor_normal_anonymizer import name_output
        from genomeanonymizer_amd import writer
        writer.io_block_size = lambda d: 4096
        inp = os.path.join(workdir, "in")
        paths = {"T": os.path.join(inp, "tumor.bam"), "N": os.path.join(inp, "normal.bam"),
                 "ref": os.path.join(inp, "ref.fa"), "vcf": os.path.join(inp, "variants.vcf")}
        fa = FastaRef(paths["ref"])
        windows = get_windows(read_vcf(paths["vcf"]), fa.index)
        anon = CompleteGermlineAnonymizer(engine=OracleEngine()) if engine == "oracle" else CompleteGermlineAnonymizer(device=0)
        if rank == fail_rank:
            def boom(*a, **k):
                raise RuntimeError("injected failure")
            if fail_stage == "tail":      # the end-of-sample stage (pair_unmapped_mates, single ends)
                from genomeanonymizer_amd import native
                native.Resolver.finish = boom
            else:
                anon.anonymize = boom
        tot = anonymize_genome_sharded(windows, paths["T"], paths["N"], paths["ref"], name_output(paths["T"]),
                                       name_output(paths["N"]), True, anon, dist)
        from genomeanonymizer_amd import distributed
        q.put((rank, (tot, distributed.LAST_TIMING.get("redos", 0), distributed.LAST_TIMING.get("spec_replans", 0))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,index,world,xchg", [("edge", True, 2, "1"), ("tiny", False, 2, "1"),
                                                   ("fuzz2003", False, 2, "1"), ("fuzz3000", False, 2, "1"),
                                                   ("fuzz3008", True, 3, "1"), ("fuzz3000", False, 2, "0"),
                                                   ("fuzz3008", True, 3, "0")])
def test_two_rank_contig_shards_match_reference(name, index, world, xchg, tmp_path, monkeypatch):
    """fuzz3000 / fuzz3008 put secondaries off their mate's contig on another rank than the mate.
    With the secondary exchange (distributed.SecondaryExchange, default) every plan knows the earlier
    jobs' secondaries from every rank: no job is planned twice. Without it (GANON_SEC_EXCHANGE=0) the
    coordinator has the owner plan such a job again (the redo protocol, stream.py)."""
    monkeypatch.setenv("GANON_SEC_EXCHANGE", xchg)
    from helpers import GOLDEN, run_pipeline_vs_golden
    from genomeanonymizer_amd.synth.generate import generate, scenario
    import gzip
    import dataclasses
    workdir = str(tmp_path / name)
    paths = generate(dataclasses.replace(scenario(name), bam_index=index), os.path.join(workdir, "in"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, workdir, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs)
    results = dict(q.get() for _ in range(world))
    assert all(results[r][0] == results[0][0] for r in range(world))   # totals are all-reduced
    if name.startswith("fuzz3"):      # jobs planned again (rank 0's coordinator counts them)
        assert (results[0][1] > 0) == (xchg == "0")
        # with the exchange, a job planned at once with the names its rank knows is planned again by
        # its owner when the permit brings another rank's secondary names (the replan
        # after a speculative plan is taken, not only the redo protocol's absence)
        spec = sum(results[r][2] for r in range(world))
        assert (spec > 0) if xchg == "1" else (spec == 0), spec
    from genomeanonymizer_amd.short_read_tumor_normal_anonymizer import name_output
    for tag, pre in (("tumor", name_output(paths["T"])), ("normal", name_output(paths["N"]))):
        for suf in (".1.fastq", ".2.fastq", ".single_end.fastq"):
            gp = os.path.join(GOLDEN, name, f"{tag}{suf}.gz")
            if os.path.exists(gp):
                assert open(pre + suf, "rb").read() == gzip.open(gp).read(), tag + suf
    assert open(paths["N"] + ".statistics.txt").read() == open(os.path.join(GOLDEN, name, "normal.statistics.txt")).read()


@pytest.mark.parametrize("fail_rank,stage", [(1, "job"), (0, "tail")])
def test_a_failing_rank_stops_every_rank(tmp_path, fail_rank, stage):
    """A rank that raises — in a contig job, or rank 0 in the end-of-sample stage — still reaches
    the next exchange with its error flag: the other rank raises too instead of waiting in a
    collective forever (ADVICE r1 distributed.py, r2 stream.py)."""
    from genomeanonymizer_amd.synth.generate import generate, scenario
    workdir = str(tmp_path / "tiny")
    generate(scenario("tiny"), os.path.join(workdir, "in"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, "tiny", workdir, q, "oracle", fail_rank, stage))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    alive = [p.is_alive() for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert alive == [False, False]
    assert all(p.exitcode != 0 for p in procs)


def test_middle_rank_failure_with_ranks_still_exporting(tmp_path):
    """3 ranks over 6 contigs; rank 1 fails in its first job while ranks 0 and 2 are still exporting
    later contigs. The coordinator stops at rank 1's contig, sends the error only to the ranks with
    jobs left, and receives every export sent before their error answers (ADVICE r3 stream.py): all
    three processes end with an error, none hangs in a pending send."""
    from test_stream import _scenario
    from genomeanonymizer_amd.synth.generate import generate
    workdir = str(tmp_path / "six")
    generate(_scenario(23, n_contigs=6, split=False), os.path.join(workdir, "in"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 3, port, "six", workdir, q, "oracle", 1, "job")) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    alive = [p.is_alive() for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert alive == [False, False, False]
    assert all(p.exitcode != 0 for p in procs)


def test_three_rank_job_mode_matches_reference(tmp_path, monkeypatch):
    """Job mode over 3 ranks: ~2.5 kb runs of sections of each contig sharded over the ranks (region
    decode, secondaries whose mate another rank's job reads: planned again), files = the reference's."""
    import dataclasses
    import gzip
    from helpers import GOLDEN
    from genomeanonymizer_amd.synth.generate import generate, scenario
    from genomeanonymizer_amd.short_read_tumor_normal_anonymizer import name_output
    monkeypatch.setenv("GANON_JOB_BP", "2500")
    name = "fuzz3008"
    workdir = str(tmp_path / name)
    paths = generate(dataclasses.replace(scenario(name), bam_index=True), os.path.join(workdir, "in"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 3, port, name, workdir, q)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs)
    for tag, pre in (("tumor", name_output(paths["T"])), ("normal", name_output(paths["N"]))):
        for suf in (".1.fastq", ".2.fastq", ".single_end.fastq"):
            gp = os.path.join(GOLDEN, name, f"{tag}{suf}.gz")
            if os.path.exists(gp):
                assert open(pre + suf, "rb").read() == gzip.open(gp).read(), tag + suf
    assert open(paths["N"] + ".statistics.txt").read() == open(os.path.join(GOLDEN, name, "normal.statistics.txt")).read()
