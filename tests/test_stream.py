"""Bounded-memory streaming (stream.py): contig reader, contig-mode planning, cross-contig
resolution, multi-rank placement. The CPU oracle stands in for the device (test infrastructure);
tests/test_gpu.py and tests/test_gpu_distributed.py run the same paths on the HIP engine.

Parity: the streamed files must equal the whole-sample path's (planner.py/ganon_plan.cpp over the
whole BAM, one device batch), which tests/test_oracle.py pins to the reference's own outputs."""
import dataclasses
import os
import shutil

import numpy as np
import pytest
import torch.multiprocessing as mp


def _scenario(seed: int, n_contigs: int = 4, split: bool = False):
    from genomeanonymizer_amd.synth.generate import ContigSpec, ScenarioConfig
    rng = np.random.default_rng(seed)
    contigs = []
    for c in range(n_contigs):
        L = int(rng.integers(8_000, 30_000))
        wins, x = [], 1001 + int(rng.integers(0, 2000))
        while x < L - 1500 and len(wins) < 5:
            wins.append(x)
            x += 2003 + int(rng.integers(0, 6000))
        if c == 1:
            wins = []            # a contig without windows: one whole-contig section
        contigs.append(ContigSpec(f"chr{c}", L, int(rng.integers(80, 500)), windows=wins,
                                  keep_windows=int(rng.integers(0, 2)),
                                  holes=[("T" if rng.random() < 0.5 else "N", 3000, 3600)]))
    return ScenarioConfig(name=f"s{seed}", seed=seed, contigs=contigs, germline_snp_per_kb=5.0,
                          germline_indel_per_kb=1.0, hom_fraction=0.3, softclip_frac=0.05,
                          unmapped_mate_frac=0.04, n_base_frac=0.03, unplaced_frac=0.4, cross_contig_pairs=15,
                          bam_index=bool(seed % 2), chimeric_frac=0.1 if split else 0.0,
                          secondary_frac=0.05 if split else 0.0)


def _outputs(prefixes, stats_path):
    files = {}
    for pre in prefixes:
        for suf in (".1.fastq", ".2.fastq", ".single_end.fastq"):
            if os.path.exists(pre + suf):
                files[os.path.basename(pre) + suf] = open(pre + suf, "rb").read()
    files["stats"] = open(stats_path).read()
    return files


def _run(paths, outdir, whole: bool, anonymizer=None):
    from pyoracle import OracleEngine
    from genomeanonymizer_amd import short_read_tumor_normal_anonymizer as sr
    from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
    os.makedirs(outdir, exist_ok=True)
    t_out, n_out = os.path.join(outdir, "tumor"), os.path.join(outdir, "normal")
    old = os.environ.get("GANON_WHOLE_SAMPLE")
    os.environ["GANON_WHOLE_SAMPLE"] = "1" if whole else "0"
    try:
        sr.run_short_read_tumor_normal_anonymizer(
            [paths["vcf"]], [(paths["T"], paths["N"])], paths["ref"],
            anonymizer or CompleteGermlineAnonymizer(engine=OracleEngine()), [(t_out, n_out)], True, 4)
    finally:
        if old is None:
            os.environ.pop("GANON_WHOLE_SAMPLE")
        else:
            os.environ["GANON_WHOLE_SAMPLE"] = old
    return _outputs((t_out, n_out), paths["N"] + ".statistics.txt")


@pytest.mark.parametrize("index", [True, False])
def test_contig_reader_matches_whole_file_decode(index, tmp_path):
    from genomeanonymizer_amd.io.bam import BamReader, ReadTable
    from genomeanonymizer_amd.synth.generate import generate, scenario
    paths = generate(dataclasses.replace(scenario("config1"), bam_index=index), str(tmp_path / "in"))
    for key in ("T", "N"):
        full = ReadTable(paths[key])
        for window in (0, 1 << 17):   # default window, and the smallest (records straddle windows)
            R = BamReader(paths[key], threads=3, window=window)
            assert R.has_index == index
            assert R.ref_names == full.ref_names
            for tid in (0, 0):           # a repeated request rescans
                t = R.contig(tid)
                rows = np.nonzero(full.tid == tid)[0]
                assert t.n == len(rows)
                for f in ("pos", "end", "flag", "l_seq", "n_cigar", "mate_tid", "mate_pos", "name_len"):
                    assert np.array_equal(getattr(t, f), getattr(full, f)[rows]), f
                assert t.names == [full.names[r] for r in rows]
                lo, hi = int(full.seq_off[rows[0]]), int(full.seq_off[rows[-1]] + (full.l_seq[rows[-1]] + 1) // 2)
                assert np.array_equal(t.seq, full.seq[lo:hi])
                qlo = int(full.qual_off[rows[0]])
                assert np.array_equal(t.qual, full.qual[qlo:qlo + len(t.qual)])
            R.close()


def test_contig_reader_multi_contig_any_order(tmp_path):
    from genomeanonymizer_amd.io.bam import BamReader, ReadTable
    from genomeanonymizer_amd.synth.generate import generate, scenario
    for index in (True, False):
        paths = generate(dataclasses.replace(scenario("edge"), bam_index=index), str(tmp_path / f"in{index}"))
        full = ReadTable(paths["T"])
        R = BamReader(paths["T"], threads=2)
        for tid in (2, 0, 1, 1, 2):
            t = R.contig(tid)
            rows = np.nonzero(full.tid == tid)[0]
            assert t.n == len(rows) and np.array_equal(t.pos, full.pos[rows])
            assert t.names == [full.names[r] for r in rows]
        assert R.contig(-1).n == 0
        R.close()


@pytest.mark.parametrize("seed", [21, 22])
def test_streaming_matches_whole_sample(seed, tmp_path):
    """Cross-contig mates, unplaced / placed unmapped mates, single ends, a contig without windows:
    every file of the streamed run equals the whole-sample run's."""
    from genomeanonymizer_amd.synth.generate import generate
    paths = generate(_scenario(seed), str(tmp_path / "in"))
    whole = _run(paths, str(tmp_path / "whole"), True)
    streamed = _run(paths, str(tmp_path / "stream"), False)
    assert set(whole) == set(streamed)
    for k in whole:
        assert whole[k] == streamed[k], k
    assert any(k.endswith(".single_end.fastq") for k in whole)


@pytest.mark.parametrize("prune_min", [None, 0], ids=["default", "prune_on_growth"])
def test_streaming_many_contigs_matches_whole_sample(prune_min, tmp_path, monkeypatch):
    """12 contigs (a tiled sample): per-contig offsets and the carried state over many rounds; with
    GANON_CARRY_PRUNE_MIN=0 the carried records are pruned whenever they have doubled."""
    if prune_min is not None:
        monkeypatch.setenv("GANON_CARRY_PRUNE_MIN", str(prune_min))
    from genomeanonymizer_amd.synth.generate import generate, scenario
    from genomeanonymizer_amd.synth.tile import tile_sample
    base = generate(scenario("tiny"), str(tmp_path / "base"))
    paths = tile_sample(base, 6, str(tmp_path / "in"))
    whole = _run(paths, str(tmp_path / "whole"), True)
    streamed = _run(paths, str(tmp_path / "stream"), False)
    assert whole == streamed


def _rank_worker(rank, world, port, paths, outdir, q, shard=None):
    import sys
    if shard:
        os.environ["GANON_SHARD"] = shard
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
        windows = get_windows(read_vcf(paths["vcf"]), FastaRef(paths["ref"]).index)
        tot = anonymize_genome_sharded(windows, paths["T"], paths["N"], paths["ref"], os.path.join(outdir, "tumor"),
                                       os.path.join(outdir, "normal"), True,
                                       CompleteGermlineAnonymizer(engine=OracleEngine()), dist)
        q.put((rank, tot))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("split", [False, True], ids=["plain", "split_alignments"])
def test_three_ranks_match_one_rank(split, tmp_path):
    """3 ranks over 5 contigs (the last round leaves a rank idle): the files equal one rank's; with
    supplementary / secondary alignments the objects of complex names cross the ranks' contigs."""
    from test_distributed import _free_port
    from genomeanonymizer_amd.synth.generate import generate
    paths = generate(_scenario(23, n_contigs=5, split=split), str(tmp_path / "in"))
    one = _run(paths, str(tmp_path / "one"), False)
    stats_one = one.pop("stats")
    os.remove(paths["N"] + ".statistics.txt")
    out = str(tmp_path / "three")
    os.makedirs(out)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, 3, port, paths, out, q)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert [p.exitcode for p in procs] == [0, 0, 0]
    tots = dict(q.get() for _ in range(3))
    assert tots[0] == tots[1] == tots[2]
    three = _outputs((os.path.join(out, "tumor"), os.path.join(out, "normal")), paths["N"] + ".statistics.txt")
    assert three.pop("stats") == stats_one
    assert three == one


def _uneven_scenario(seed: int):
    """One contig with >= 5x the reads of any other plus 100 tiny contigs (alt/decoy-like), with
    cross-contig and unplaced mates."""
    from genomeanonymizer_amd.synth.generate import ContigSpec, ScenarioConfig
    rng = np.random.default_rng(seed)
    contigs = [ContigSpec("chrBig", 60_000, 1500, windows=[1500 + 4000 * k for k in range(12)], keep_windows=1)]
    for c in range(100):
        L = int(rng.integers(3_000, 5_000))
        contigs.append(ContigSpec(f"decoy{c}", L, int(rng.integers(3, 30)),
                                  windows=[1200 + int(rng.integers(0, 300))] if rng.random() < 0.6 else []))
    return ScenarioConfig(name=f"u{seed}", seed=seed, contigs=contigs, germline_snp_per_kb=4.0,
                          germline_indel_per_kb=0.5, hom_fraction=0.3, softclip_frac=0.03,
                          unmapped_mate_frac=0.03, unplaced_frac=0.4, cross_contig_pairs=40, bam_index=True)


@pytest.mark.parametrize("world,shard", [(3, "round_robin"), (4, "lpt")])
def test_uneven_contigs_many_ranks_match_one_rank(world, shard, tmp_path):
    """De-lock-stepped ranks (distributed.py): no rounds — each rank works through its own contigs
    and rank 0's coordinator resolves them in FASTA order as they arrive. An uneven contig list (one
    contig with >= 5x the reads of the others, 100 tiny decoys), round-robin and LPT shards: the
    files equal one rank's."""
    from test_distributed import _free_port
    from genomeanonymizer_amd.distributed import assign_contigs
    from genomeanonymizer_amd.synth.generate import generate
    paths = generate(_uneven_scenario(31), str(tmp_path / "in"))
    one = _run(paths, str(tmp_path / "one"), False)
    stats_one = one.pop("stats")
    os.remove(paths["N"] + ".statistics.txt")
    out = str(tmp_path / "many")
    os.makedirs(out)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, paths, out, q, shard)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert [p.exitcode for p in procs] == [0] * world
    tots = dict(q.get() for _ in range(world))
    assert all(tots[r] == tots[0] for r in range(world))
    many = _outputs((os.path.join(out, "tumor"), os.path.join(out, "normal")), paths["N"] + ".statistics.txt")
    assert many.pop("stats") == stats_one
    assert many == one
    if shard == "lpt":   # the loads end within one decoy of each other
        lens = [60_000] + [4_000] * 100
        owner = assign_contigs(lens, world, "lpt")
        load = [sum(l for l, o in zip(lens, owner) if o == r) for r in range(world)]
        assert max(load) - min(load) <= 4_000


def test_contig_shard_policies():
    from genomeanonymizer_amd.distributed import assign_contigs
    assert assign_contigs([5, 1, 1, 1], 2) == [0, 1, 0, 1]
    assert assign_contigs([5, 1, 1, 1], 2, "lpt") == [0, 1, 1, 1]
    assert assign_contigs([3, 3, 2, 2, 2], 2, "lpt") == [0, 1, 0, 1, 0]
    with pytest.raises(ValueError):
        assign_contigs([1], 2, "random")


def _pairs_worker(rank, world, port, pairs, ref, q):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "oracle"), os.path.join(repo, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pyoracle import OracleEngine
        from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
        from genomeanonymizer_amd.distributed import run_pairs_sharded
        vcfs = [p["vcf"] for p in pairs]
        samples = [(p["T"], p["N"]) for p in pairs]
        outs = [(p["out"] + "/tumor", p["out"] + "/normal") for p in pairs]
        tots = run_pairs_sharded(vcfs, samples, ref, CompleteGermlineAnonymizer(engine=OracleEngine()), outs, True,
                                 dist)
        q.put((rank, len(tots)))
    finally:
        dist.destroy_process_group()


def test_one_pair_per_rank(tmp_path):
    """Several tumor/normal pairs over as many ranks: each rank runs its pairs whole (the
    reference's one task per pair, SR:944-961); every pair's files equal a single-rank run's."""
    import shutil
    from test_distributed import _free_port
    from genomeanonymizer_amd.synth.generate import generate
    base = generate(_scenario(41, n_contigs=3), str(tmp_path / "in"))
    pairs = []
    for k in range(3):
        d = tmp_path / f"pair{k}"
        d.mkdir()
        p = {"vcf": base["vcf"], "out": str(d)}
        for tag in ("T", "N"):
            dst = str(d / os.path.basename(base[tag]))
            shutil.copy(base[tag], dst)
            if os.path.exists(base[tag] + ".bai"):
                shutil.copy(base[tag] + ".bai", dst + ".bai")
            p[tag] = dst
        pairs.append(p)
    one = _run(base, str(tmp_path / "one"), False)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pairs_worker, args=(r, 2, port, pairs, base["ref"], q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert [p.exitcode for p in procs] == [0, 0]
    counts = dict(q.get() for _ in range(2))
    assert counts == {0: 2, 1: 1}              # pairs 0, 2 on rank 0, pair 1 on rank 1
    for p in pairs:
        got = _outputs((p["out"] + "/tumor", p["out"] + "/normal"), p["N"] + ".statistics.txt")
        assert got == one


_DIGEST = r"""
import hashlib, sys
sys.path.insert(0, sys.argv[1])
from genomeanonymizer_amd import native
from genomeanonymizer_amd.io.bam import BamReader, ReadTable
h = hashlib.sha256()
for path in sys.argv[2:]:
    full = ReadTable(path, threads=3)
    R = BamReader(path, threads=2, window=1 << 17)
    for t in [full] + [R.contig(i) for i in range(len(full.ref_names))]:
        for f in ("pos", "end", "flag", "l_seq", "n_cigar", "name_len", "cigar", "seq", "qual", "aux", "names_blob"):
            h.update(getattr(t, f).tobytes())
    R.close()
print(native.host_lib().ganon_host_inflate_backend().decode(), h.hexdigest())
"""


def test_libdeflate_and_zlib_inflaters_decode_alike(tmp_path):
    """The host inflater (the system libdeflate when present, else zlib; GANON_INFLATE=zlib forces
    zlib) decodes every field alike, whole-file and contig by contig; the views of the decoder's
    buffers outlive the reader."""
    import subprocess
    import sys
    from genomeanonymizer_amd.synth.generate import generate, scenario
    paths = generate(dataclasses.replace(scenario("edge"), bam_index=True), str(tmp_path / "in"))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for mode in ("default", "zlib"):
        env = dict(os.environ)
        env.pop("GANON_INFLATE", None)
        if mode == "zlib":
            env["GANON_INFLATE"] = "zlib"
        r = subprocess.run([sys.executable, "-c", _DIGEST, repo, paths["T"], paths["N"]], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        out[mode] = r.stdout.split()
    assert out["zlib"][0] == "zlib"
    if os.path.exists("/usr/lib/x86_64-linux-gnu/libdeflate.so.0"):
        assert out["default"][0] == "libdeflate"
    assert out["default"][1] == out["zlib"][1]


def test_decoded_blobs_are_views_kept_alive(tmp_path):
    """ReadTable's byte blobs are views of the native decoder's buffers: they stay valid after the
    table and its reader are gone (the owner is freed with the last view)."""
    import gc
    from genomeanonymizer_amd.io.bam import BamReader
    from genomeanonymizer_amd.synth.generate import generate, scenario
    paths = generate(scenario("tiny"), str(tmp_path / "in"))
    R = BamReader(paths["T"], threads=2)
    t = R.contig(0)
    seq, qual, names = t.seq, t.qual, t.names_blob
    ref = (seq.copy(), qual.copy(), names.copy())
    assert not seq.flags.owndata
    del t
    R.close()
    del R
    gc.collect()
    junk = [np.full(1 << 16, 0xAB, np.uint8) for _ in range(64)]   # reuse of freed memory would show
    assert np.array_equal(seq, ref[0]) and np.array_equal(qual, ref[1]) and np.array_equal(names, ref[2])
    del junk


def test_names_present_equals_blob_search(tmp_path):
    """stream._names_present (one vectorized pass, Job.redo_needed) finds exactly the names a search
    of the NUL-separated names blob finds: present names, absent ones, prefixes and extensions of
    present names, names of every length around the 8-byte key words, empty input."""
    from genomeanonymizer_amd import stream
    from genomeanonymizer_amd.io.bam import BamReader
    from genomeanonymizer_amd.synth.generate import generate, scenario
    paths = generate(scenario("fuzz3000"), str(tmp_path / "in"))
    R = BamReader(paths["T"], threads=2)
    t = R.contig(0)
    present = stream._names(t, np.arange(t.n))
    rng = np.random.default_rng(7)
    pick = [present[i] for i in rng.choice(len(present), 200, replace=False)]
    probes = pick + [p[:-1] for p in pick[:40]] + [p + b"x" for p in pick[:40]] + \
        [b"q" * k for k in range(1, 20)] + [p[:8] for p in pick[:20]] + [b"no_such_read_%d" % i for i in range(50)]
    blob = b"\0" + t.names_blob.tobytes()
    want = {nm for nm in probes if blob.find(b"\0" + nm + b"\0") >= 0}
    assert stream._names_present(t, probes) == want
    assert set(pick) <= want
    assert stream._names_present(t, []) == set()
    R.close()


def _python_buffer_alloc():
    """A ganon_buf_alloc_fn / ganon_buf_free_fn pair over ctypes buffers (the page-locked allocator's
    stand-in on the CPU), with the live blocks and the number of allocations."""
    import ctypes as C
    live, calls = {}, [0]
    AF = C.CFUNCTYPE(C.c_int, C.c_int64, C.POINTER(C.c_void_p))
    FF = C.CFUNCTYPE(C.c_int, C.c_void_p)

    def alloc(n, out):
        b = C.create_string_buffer(int(n))
        live[C.addressof(b)] = b
        out[0] = C.addressof(b)
        calls[0] += 1
        return 0

    def free(p):
        live.pop(p, None)
        return 0
    return AF(alloc), FF(free), live, calls


@pytest.mark.parametrize("scan_buffer", ["fresh", "reader_owned"])
def test_region_reader_matches_fetch(scan_buffer, tmp_path):
    """ganon_bam_reader_region (BAI linear index, htslib overlap semantics, placed unmapped records
    at [pos, pos + 1)) against the whole-file table's fetch on random regions of a multi-window BAM;
    with the scans' bytes in fresh buffers, and in one buffer the reader keeps and reuses across its
    scans (ganon_bam_reader_set_buffer_alloc: page-locked with the GPU inflater)."""
    import ctypes as C
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.io.bam import BamReader, ReadTable
    from genomeanonymizer_amd.synth.fastpair import make_pair
    d = str(tmp_path / "in")
    make_pair(d, n_contigs=2, contig_len=400_000, pairs_per_contig=20_000, window_every=20_000)
    rng = np.random.default_rng(3)
    for key in ("tumor", "normal"):
        path = os.path.join(d, f"{key}.bam")
        full = ReadTable(path)
        rd = BamReader(path, 4)
        if scan_buffer == "reader_owned":
            af, ff, live, calls = _python_buffer_alloc()
            rd._keep_alloc = (af, ff)
            native.host_lib().ganon_bam_reader_set_buffer_alloc(rd._h, C.cast(af, C.c_void_p), C.cast(ff, C.c_void_p))
        assert rd.has_index
        for tid, (name, L) in enumerate(zip(full.ref_names, full.ref_lens)):
            for _ in range(20):
                a = int(rng.integers(0, L))
                b = int(min(L, a + rng.integers(0, 60_000)))
                exp = full.fetch(name, a, b)
                got = rd.region(tid, a, b)
                assert got.n == len(exp)
                assert np.array_equal(np.asarray(got.pos), np.asarray(full.pos)[exp])
                assert np.array_equal(np.asarray(got.flag), np.asarray(full.flag)[exp])
                assert np.array_equal(np.asarray(got.qual), np.concatenate([np.asarray(full.qual)[
                    int(full.qual_off[i]):int(full.qual_off[i]) + int(full.l_seq[i])] for i in exp]) if len(exp)
                    else np.zeros(0, np.uint8))
            # contig scans use the same buffer
            assert rd.contig(tid).n == int((np.asarray(full.tid) == tid).sum())
        rd.close()
        if scan_buffer == "reader_owned":
            assert calls[0] >= 1 and not live    # grown through the allocator, freed at close


def _rank_worker_timing(rank, world, port, paths, outdir, q):
    """_rank_worker, reporting the rank's exchange bytes and rank 0's coordinator seconds."""
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "oracle"), os.path.join(repo, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pyoracle import OracleEngine
        from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
        from genomeanonymizer_amd import distributed
        from genomeanonymizer_amd.io.fasta import FastaRef
        from genomeanonymizer_amd.io.vcf import read_vcf
        from genomeanonymizer_amd.planner import get_windows
        windows = get_windows(read_vcf(paths["vcf"]), FastaRef(paths["ref"]).index)
        distributed.anonymize_genome_sharded(windows, paths["T"], paths["N"], paths["ref"], os.path.join(outdir, "tumor"),
                                             os.path.join(outdir, "normal"), True,
                                             CompleteGermlineAnonymizer(engine=OracleEngine()), dist)
        t = distributed.LAST_TIMING
        q.put((rank, {k: t.get(k) for k in ("exchange_sent_bytes", "exchange_recv_bytes", "resolve_s", "jobs",
                                             "reads", "wait_s")}))
    finally:
        dist.destroy_process_group()


def test_four_ranks_24_contigs_exchange(tmp_path):
    """4 ranks over a 24-contig sample (cross-contig, unplaced and unmapped mates): the files equal one
    rank's; every rank's exchange with rank 0's coordinator (pickled exports and resolutions over
    gloo) and the coordinator's resolve time are reported."""
    from test_distributed import _free_port
    from genomeanonymizer_amd.synth.generate import generate
    paths = generate(_scenario(41, n_contigs=24), str(tmp_path / "in"))
    one = _run(paths, str(tmp_path / "one"), False)
    stats_one = one.pop("stats")
    os.remove(paths["N"] + ".statistics.txt")
    out = str(tmp_path / "four")
    os.makedirs(out)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker_timing, args=(r, 4, port, paths, out, q)) for r in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert [p.exitcode for p in procs] == [0] * 4
    rep = dict(q.get() for _ in range(4))
    print("4-rank exchange:", rep)
    assert sum(r["jobs"] for r in rep.values()) == 24
    assert rep[0]["resolve_s"] is not None and rep[0]["exchange_recv_bytes"] > 0
    assert all(rep[r]["exchange_sent_bytes"] > 0 for r in (1, 2, 3))
    four = _outputs((os.path.join(out, "tumor"), os.path.join(out, "normal")), paths["N"] + ".statistics.txt")
    assert four.pop("stats") == stats_one
    assert four == one


def test_one_corrupt_sample_fails_cleanly_and_the_next_run_is_right(tmp_path):
    """a job's tumor and normal BAMs are read at once on the sample pool. Only the tumor
    BAM is corrupt, past the header (a BGZF block of its second contig): the run raises the reader's
    inflate error once the normal sample's read of that job has finished (stream._map_samples waits for
    both before raising, so the failure path never closes a reader a read is still inside), and the
    next runs in the same process — the same sample pool — write equal files streamed and whole."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.fastpair import make_pair
    paths = make_pair(str(tmp_path / "in"), n_contigs=3, contig_len=400_000, pairs_per_contig=4_000, seed=3)
    bad = dict(paths)
    bad["T"] = str(tmp_path / "bad_tumor.bam")
    data = bytearray(open(paths["T"], "rb").read())
    assert len(data) > 2 << 20     # (the reader's header read takes the first MiB)
    mid = len(data) * 6 // 10
    data[mid:mid + 4096] = bytes(4096)
    open(bad["T"], "wb").write(bytes(data))
    shutil.copy(paths["T"] + ".bai", bad["T"] + ".bai")
    with pytest.raises(native.GanonError, match="inflate|BGZF|block"):
        _run(bad, str(tmp_path / "bad"), False)
    whole = _run(paths, str(tmp_path / "whole"), True)
    streamed = _run(paths, str(tmp_path / "stream"), False)
    assert whole == streamed


def test_reader_with_inflater_and_buffer_alloc_reads_windows_into_its_buffer(tmp_path):
    """The GPU-inflater configuration of the reader on the CPU: windows for the inflater are read by
    pread into the reader's allocator-provided buffer (page-locked with the GPU inflater) and handed to
    the inflater callback (here zlib in Python); region reads equal the whole-file table's fetch, and
    the buffers go back through the allocator at close."""
    import ctypes as C
    import zlib
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.io.bam import BamReader, ReadTable
    from genomeanonymizer_amd.synth.fastpair import make_pair
    d = str(tmp_path / "in")
    make_pair(d, n_contigs=2, contig_len=400_000, pairs_per_contig=20_000, window_every=20_000)
    INF = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint8), C.c_int64, C.POINTER(C.c_int64),
                      C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.c_int64,
                      C.POINTER(C.c_uint8), C.c_int64)
    calls = [0]

    def inflate(user, comp, comp_len, in_off, in_len, out_off, out_len, n, out, out_total):
        calls[0] += 1
        base_in, base_out = C.addressof(comp.contents), C.addressof(out.contents)
        for i in range(n):
            o = zlib.decompress(C.string_at(base_in + in_off[i], in_len[i]), -15)
            if len(o) != out_len[i]:
                return 1
            C.memmove(base_out + out_off[i], o, len(o))
        return 0
    cb = INF(inflate)
    path = os.path.join(d, "tumor.bam")
    full = ReadTable(path)
    rd = BamReader(path, 4)
    af, ff, live, allocs = _python_buffer_alloc()
    lib = native.host_lib()
    lib.ganon_bam_reader_set_buffer_alloc(rd._h, C.cast(af, C.c_void_p), C.cast(ff, C.c_void_p))
    lib.ganon_bam_reader_set_inflater(rd._h, C.cast(cb, C.c_void_p), None, 1)
    for tid, (name, L) in enumerate(zip(full.ref_names, full.ref_lens)):
        for a, b in ((0, int(L)), (1000, 200_000), (150_000, 390_000)):
            exp = full.fetch(name, a, b)
            got = rd.region(tid, a, b)
            assert got.n == len(exp)
            assert np.array_equal(np.asarray(got.pos), np.asarray(full.pos)[exp])
    assert calls[0] > 0 and allocs[0] >= 2     # (the scan buffer and the compressed-window buffer)
    rd.close()
    assert not live


def test_reader_region_decoder_protocol(tmp_path):
    """The device region decoder's protocol on the CPU (ganon_bam_reader_set_region_decoder, include/
    ganon_host.h; the GPU's ganon_region_decode is checked in tests/test_region_device.py): a Python
    decoder that either returns a region's columns in a block of its own (here: another reader's
    decode, laid out in one buffer) or declines after inflating the window into `out` (the reader's
    walk then goes on from there). Both ways the tables equal the plain reader's, the decoder sees the
    region and the window's first record offset, and every block goes back through release when its
    table closes."""
    import ctypes as C
    import gc
    import zlib
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.io.bam import BamReader
    from genomeanonymizer_amd.synth.fastpair import make_pair
    d = str(tmp_path / "in")
    make_pair(d, n_contigs=2, contig_len=400_000, pairs_per_contig=20_000, window_every=20_000)
    path = os.path.join(d, "tumor.bam")
    ref, helper = BamReader(path, 4), BamReader(path, 4)
    u8p, i64p, i32p = C.POINTER(C.c_uint8), C.POINTER(C.c_int64), C.POINTER(C.c_int32)
    REG = C.CFUNCTYPE(C.c_int, C.c_void_p, u8p, C.c_int64, i64p, i32p, i64p, i32p, C.c_int64, u8p, C.c_int64,
                      C.c_int64, C.c_int32, C.c_int64, C.c_int64, C.c_int, C.POINTER(native.BamView),
                      C.POINTER(C.c_void_p))
    FF = C.CFUNCTYPE(C.c_int, C.c_void_p)
    live, seen, mode = {}, [], ["done"]
    cols_i32 = ("tid", "pos", "end", "flag", "mapq", "l_seq", "n_cigar", "mate_tid", "mate_pos", "tlen", "name_len",
                "aux_len")
    cols_i64 = ("name_off", "cig_off", "seq_off", "qual_off", "aux_off")
    blobs = (("names", "names_blob", "names_bytes"), ("cigar", "cigar", "cigar_ops"), ("seq", "seq", "seq_bytes"),
             ("qual", "qual", "qual_bytes"), ("aux", "aux", "aux_bytes"))

    def decode(user, comp, comp_len, in_off, in_len, out_off, out_len, n, out, out_total, p0, tid, beg, end,
               at_eof, cols, block):
        seen.append((tid, beg, end, p0, mode[0]))
        if mode[0] == "decline":
            base_in, base_out = C.addressof(comp.contents), C.addressof(out.contents)
            for i in range(n):
                o = zlib.decompress(C.string_at(base_in + in_off[i], in_len[i]), -15)
                C.memmove(base_out + out_off[i], o, len(o))
            return 0
        t = helper.region(tid, beg, end)
        parts = [np.ascontiguousarray(getattr(t, f)) for f in cols_i32 + cols_i64] + \
            [np.ascontiguousarray(getattr(t, a)) for _, a, _ in blobs]
        offs, size = [], 0
        for a in parts:
            offs.append(size)
            size += (a.nbytes + 255) // 256 * 256
        buf = C.create_string_buffer(max(size, 1))
        base = C.addressof(buf)
        for a, o in zip(parts, offs):
            if a.nbytes:
                C.memmove(base + o, a.ctypes.data, a.nbytes)
        v = cols.contents
        v.n_records = t.n
        for k, f in enumerate(cols_i32 + cols_i64):
            setattr(v, f, C.cast(base + offs[k], type(getattr(v, f))))
        for j, (f, a, nb) in enumerate(blobs):
            k = len(cols_i32) + len(cols_i64) + j
            setattr(v, f, C.cast(base + offs[k], type(getattr(v, f))) if f != "names" else base + offs[k])
            setattr(v, nb, int(getattr(t, a).size))
        live[base] = buf
        block[0] = base
        return 1

    def release(p):
        live.pop(p, None)
        return 0
    dec, rel = REG(decode), FF(release)
    rd = BamReader(path, 4)
    lib = native.host_lib()
    lib.ganon_bam_reader_set_region_decoder(rd._h, C.cast(dec, C.c_void_p), None, 1, C.cast(rel, C.c_void_p))
    for m in ("done", "decline"):
        mode[0] = m
        for tid, L in enumerate(ref.ref_lens):
            for a, b in ((0, int(L)), (1000, 200_000), (150_000, 390_000), (399_000, int(L) + 5)):
                exp, got = ref.region(tid, a, b), rd.region(tid, a, b)
                assert got.n == exp.n and got.n > 0
                for f in cols_i32 + cols_i64 + ("names_blob", "cigar", "seq", "qual", "aux"):
                    assert np.array_equal(np.asarray(getattr(got, f)), np.asarray(getattr(exp, f))), (m, f)
                assert seen[-1][:3] == (tid, a, b)
        del got, exp
        gc.collect()
        assert not live                     # (each table's block released with its last view)
    assert {s[4] for s in seen} == {"done", "decline"}
    assert all(s[3] >= 0 for s in seen)
    rd.close()
    ref.close()
    helper.close()
