"""Parity of the HIP path (libganon_hip.so through the C ABI) — needs an MI355X.

Bit-exact for every written read's packed bases and for the per-scope counts, against
(1) the reference's own per-scope outputs (tests/golden/scopes, made by
oracle/make_scope_golden.py), (2) the CPU oracle on seeded edge-case and config-2 batches,
(3) the reference's end-to-end FASTQ/statistics files (tests/golden/<scenario>).
"""
import numpy as np
import pytest

from helpers import load_scope_golden, run_pipeline_vs_golden, written_reads_equal

pytestmark = pytest.mark.gpu



@pytest.fixture(scope="module")
def masker(hip_built):
    from genomeanonymizer_amd import native
    m = native.HipMasker(0)
    yield m
    m.close()


@pytest.fixture(scope="module")
def oracle():
    from pyoracle import OracleEngine
    return OracleEngine()


def _all_reads_equal(arr, a, b):
    """Written reads and pass-through reads (write_scope -1 in the batch: plain copies)."""
    L = (arr["read_len"].astype(np.int64) + 1) // 2
    bad = []
    for r in range(len(L)):
        o, n = int(arr["seq_off"][r]), int(L[r])
        if not np.array_equal(a[o:o + n], b[o:o + n]):
            bad.append(r)
    return bad


@pytest.mark.parametrize("seed", [101, 202, 303])
def test_hip_matches_reference_scopes(masker, seed):
    arr, exp_seq, exp_calls = load_scope_golden(seed)
    out, calls, bases, tot = masker.mask(arr)
    assert written_reads_equal(arr, out, exp_seq) == []
    assert np.array_equal(calls, exp_calls)


@pytest.mark.parametrize("seed", list(range(1, 13)))
def test_hip_matches_oracle_edge_batches(masker, oracle, seed):
    from genomeanonymizer_amd.synth.batch import random_batch
    kw = {}
    if seed % 3 == 0:
        kw["rare_frac"] = 0.3
    if seed % 4 == 0:
        kw["wide_scopes"] = 4
    arr = random_batch(seed, n_scopes=40, **kw)
    o_out, o_calls, o_bases, o_tot = oracle.mask(arr)
    in_batch = np.zeros(len(arr["read_len"]), bool)
    in_batch[arr["incid_read"]] = True
    out, calls, bases, tot = masker.mask(arr)
    bad = [r for r in _all_reads_equal(arr, out, o_out) if in_batch[r] or arr["write_scope"][r] >= 0]
    assert bad == []
    assert np.array_equal(calls, o_calls) and np.array_equal(bases, o_bases)
    assert tot[0] == o_tot[0] and tot[1] == o_tot[1]


def test_retired_variants_are_rejected(masker):
    """The round-1 A/B kernels are gone from the product library (ABI 3): asking for one is an
    error, not a silent fallback."""
    from genomeanonymizer_amd import native
    for v in (1, 2, 3, 4, 6):
        with pytest.raises(native.GanonError):
            masker.set_variant(v)
    masker.set_variant(5)
    masker.set_variant(0)


def test_reload_rebuilds_every_derived_array(masker, oracle):
    """ganon_batch_reload reuses the device buffers of another batch (grow-only): batch A, then
    a differently shaped batch B, then A again — every run rebuilds segments, groups and pieces
    from the raw arrays on the device, so each result equals a fresh one-shot mask."""
    from genomeanonymizer_amd.synth.batch import config2_batch, random_batch
    a, _ = config2_batch(n_reads=120_000, genome=40_000_000, n_windows=12_000, n_germline=30_000, seed=4)
    b = random_batch(31, n_scopes=50, rare_frac=0.2, wide_scopes=3)
    want_a, want_b = masker.mask(a), masker.mask(b)
    db = masker.upload(a)
    try:
        for arr, want in ((a, want_a), (b, want_b), (a, want_a)):
            if arr is not a or db.seq_bytes != len(a["seq_nt16"]):
                db.reload(arr)
            db.run()
            db.run()        # twice: no state of a run may leak into the next
            got = db.download()
            for k in range(4):
                assert np.array_equal(got[k], want[k]), k
    finally:
        db.free()
    o_out, o_calls, o_bases, _ = oracle.mask(b)
    assert np.array_equal(want_b[1], o_calls) and np.array_equal(want_b[2], o_bases)


def test_resident_reference_matches_private(masker):
    """ganon_ref_upload: one genome resident in HBM, batches uploaded against it (no reference in
    the batch) give the same bytes and counts as batches carrying their own reference."""
    from genomeanonymizer_amd.synth.batch import config2_batch
    arr, _ = config2_batch(n_reads=100_000, genome=30_000_000, n_windows=10_000, n_germline=20_000, seed=9)
    want = masker.mask(arr)
    ref = masker.upload_reference(arr["ref_nt16"])
    no_ref = {k: v for k, v in arr.items() if k != "ref_nt16"}
    db = masker.upload(no_ref, ref=ref)
    try:
        db.run()
        got = db.download()
    finally:
        db.free()
        ref.free()
    for k in range(4):
        assert np.array_equal(got[k], want[k]), k


@pytest.mark.parametrize("seed,keep,err", [(5, False, 0.02), (6, True, 0.05)])
def test_dense_scopes_match_oracle(masker, oracle, seed, keep, err):
    """Thousands of observations per scope and one site seen by ~600 reads: the group kernel's
    LDS list overflows into the group's global region; at 5 % errors (more mismatches than the
    region holds, ~2 % of the bases) the region is split by key range."""
    from genomeanonymizer_amd.synth.batch import dense_batch
    arr = dense_batch(seed, keep_hot_site=keep, error_rate=err)
    o_out, o_calls, o_bases, _ = oracle.mask(arr)
    assert o_calls[0] > 1000
    db = masker.upload(arr)
    try:
        db.run()
        out, calls, bases, _ = db.download()
        paths = db.path_counts()
    finally:
        db.free()
    assert np.array_equal(calls, o_calls)
    assert np.array_equal(bases, o_bases)
    assert np.array_equal(out, o_out)
    assert paths["overflowing_lists"] > 0, paths
    assert (paths["key_range_splits"] > 0) == (err > 0.04), paths


@pytest.mark.parametrize("seed", [5, 6])
def test_long_reads_match_oracle(masker, oracle, seed):
    """SURVEY §8(d) C5 shape: 10-100 kb reads with ~5 % 1-3 bp indels, soft clips, N runs and
    IUPAC codes in the reference; window scopes span up to ~200 kb (the LDS tile path)."""
    from genomeanonymizer_amd.synth.batch import longread_batch
    arr, info = longread_batch(seed, n_reads=120)
    assert info["max_span"] > 16384
    o_out, o_calls, o_bases, o_tot = oracle.mask(arr)
    assert o_calls.sum() > 100
    out, calls, bases, tot = masker.mask(arr)
    assert np.array_equal(calls, o_calls)
    assert np.array_equal(bases, o_bases)
    assert np.array_equal(out, o_out)


def test_deep_coverage_short_reads_match_oracle(masker, oracle):
    """SURVEY §8(d) C3 density (~60x tumor+normal) on a small genome: window scopes of ~800
    reads, observation lists near and over their LDS capacity."""
    from genomeanonymizer_amd.synth.batch import config2_batch
    arr, info = config2_batch(n_reads=800_000, genome=2_000_000, n_contigs=2, n_windows=600, n_germline=2_000)
    o_out, o_calls, o_bases, _ = oracle.mask(arr)
    out, calls, bases, tot = masker.mask(arr)
    assert np.array_equal(calls, o_calls)
    assert np.array_equal(bases, o_bases)
    assert np.array_equal(out, o_out)


def test_hip_huge_scopes_tile_path_matches_oracle(masker, oracle):
    """Scopes wider than 2^20 positions take the LDS tile path (k_tile_large + k_mask_large), and
    tiles meeting IUPAC/'=' bases re-run on the 16-code tally; both equal the oracle."""
    from genomeanonymizer_amd.synth.batch import random_batch
    arr = random_batch(8, n_scopes=12, rare_frac=0.3, wide_scopes=2, wide_span=(1_100_000, 1_200_000))
    o_out, o_calls, o_bases, o_tot = oracle.mask(arr)
    db = masker.upload(arr)
    try:
        db.run()
        out, calls, bases, tot = db.download()
        info = db.info()
    finally:
        db.free()
    assert info["huge_scopes"] == 2 and info["huge_tiles"] >= 2 * 67
    assert tot[5] >= 1, "no tile went through the 16-code re-run"
    assert np.array_equal(calls, o_calls) and np.array_equal(bases, o_bases)
    written = arr["write_scope"] >= 0
    L = (arr["read_len"].astype(np.int64) + 1) // 2
    for r in np.nonzero(written)[0]:
        o, n = int(arr["seq_off"][r]), int(L[r])
        assert np.array_equal(out[o:o + n], o_out[o:o + n]), r


def test_hip_configs2_density_matches_oracle(masker, oracle):
    """BASELINE configs[2] density on a slice the oracle covers: 30x tumor + 30x normal 150 bp
    reads, a germline het SNP every ~37 bp (an ~80 M-site set on 3 Gb), a window every 10 kb
    (2.4 M reads, 6 Mb). Window scopes hold ~860 reads and ~1,700 observations, gap union scopes
    several thousand: the group kernel's LDS lists overflow into the global region path."""
    from genomeanonymizer_amd.synth.batch import config2_batch
    arr, info = config2_batch(n_reads=2_400_000, genome=6_000_000, n_contigs=2, n_windows=600,
                              n_germline=162_000, seed=12, window_spacing=10_000)
    assert info["germline_snps"] > 150_000
    from genomeanonymizer_amd import native
    o_out, o_calls, o_bases, o_tot = oracle.mask(arr)
    db = masker.upload(arr)
    try:
        runs = {}
        for obs in (512, 0):          # the 512-entry lists (region path forced) and the auto choice
            masker.set_param(native.PARAM_GROUP_OBS, obs)
            db.run()
            runs[obs] = db.download() + (db.path_counts(),)
    finally:
        masker.set_param(native.PARAM_GROUP_OBS, 0)
        db.free()
    for obs, (out, calls, bases, tot, paths) in runs.items():
        assert np.array_equal(calls, o_calls), obs
        assert np.array_equal(bases, o_bases), obs
        assert np.array_equal(out, o_out), obs
    assert o_bases.sum() > 100_000
    assert runs[512][4]["overflowing_lists"] > 0, runs[512][4]


def test_hip_deep_coverage_filter_matches_oracle(masker, oracle):
    """SURVEY C3 density (60x tumor + normal, a germline het SNP per kb, 0.1 % sequencing errors,
    a window every 10 kb): gap union scopes of ~4,000 reads overflow the 512-entry LDS list; the
    pass's Bloom bitmaps drop the single-dataset keys (sequencing errors) and most such lists are
    classified in LDS instead of the global region (GrpShared patch area reused)."""
    from genomeanonymizer_amd.synth.batch import config2_batch
    arr, info = config2_batch(n_reads=2_000_000, genome=5_000_000, n_contigs=2, n_windows=500,
                              n_germline=5_000, seed=31, window_spacing=10_000)
    o_out, o_calls, o_bases, _ = oracle.mask(arr)
    db = masker.upload(arr)
    try:
        db.run()
        out, calls, bases, _ = db.download()
        paths = db.path_counts()
    finally:
        db.free()
    assert np.array_equal(calls, o_calls)
    assert np.array_equal(bases, o_bases)
    assert np.array_equal(out, o_out)
    assert paths["overflowing_lists"] > 0 and paths["filtered_into_lds"] > 0, paths


@pytest.mark.parametrize("whole", [False, True], ids=["streaming", "whole_sample"])
@pytest.mark.parametrize("name", ["tiny", "edge", "config1", "fuzz5", "fuzz9", "long1", "fuzz9001", "long2",
                                  "longpair"])
def test_hip_pipeline_matches_reference(name, whole, tmp_path, hip_built, monkeypatch):
    from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
    monkeypatch.setenv("GANON_WHOLE_SAMPLE", "1" if whole else "0")
    bad = run_pipeline_vs_golden(name, str(tmp_path / name), CompleteGermlineAnonymizer(device=0))
    assert bad == {}


@pytest.mark.parametrize("whole", [False, True], ids=["streaming", "whole_sample"])
@pytest.mark.parametrize("name", ["fuzz1001", "fuzz2000", "fuzz2003", "fuzz3000", "fuzz3008"])
def test_hip_pipeline_split_alignments_match_reference(name, whole, tmp_path, hip_built, monkeypatch):
    """Supplementary (SA) and secondary alignments through the streamed HIP product: one device copy
    per (alignment, scope), the object log replayed over them (objects.py); the reference's files.
    fuzz3000 / fuzz3008: secondaries off their mate's contig, second-scope copies of cross names,
    unmapped supplementary / secondary / SA-tagged mates in the end-of-sample tail. Whole-sample
    mode hands such samples to the streamed path."""
    from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
    monkeypatch.setenv("GANON_WHOLE_SAMPLE", "1" if whole else "0")
    bad = run_pipeline_vs_golden(name, str(tmp_path / name), CompleteGermlineAnonymizer(device=0))
    assert bad == {}


@pytest.mark.parametrize("name", ["config1", "fuzz3008", "long1"])
def test_hip_job_mode_matches_reference(name, tmp_path, hip_built, monkeypatch):
    """Job mode through the HIP product: contigs cut into ~2.5 kb runs of sections (region decode with
    a margin, one device batch per job, cross names resolved in job order); the reference's files."""
    from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
    monkeypatch.setenv("GANON_WHOLE_SAMPLE", "0")
    monkeypatch.setenv("GANON_JOB_BP", "2500")
    bad = run_pipeline_vs_golden(name, str(tmp_path / name), CompleteGermlineAnonymizer(device=0), bam_index=True)
    assert bad == {}


def test_hip_streaming_matches_whole_sample_many_contigs(tmp_path, hip_built, monkeypatch):
    """The streamed product (per-contig decode, contig-mode plans, one HIP batch per contig with the
    genome resident, cross-contig resolution) against the whole-sample product on a 12-contig
    tiled sample with cross-contig mates, unplaced mates and single ends: identical files."""
    import os
    from test_stream import _run
    from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
    from genomeanonymizer_amd.synth.generate import generate, scenario
    from genomeanonymizer_amd.synth.tile import tile_sample
    base = generate(scenario("edge"), str(tmp_path / "base"))
    paths = tile_sample(base, 4, str(tmp_path / "in"))
    anon = CompleteGermlineAnonymizer(device=0)
    whole = _run(paths, str(tmp_path / "whole"), True, anon)
    streamed = _run(paths, str(tmp_path / "stream"), False, anon)
    assert whole == streamed
    assert any(k.endswith(".single_end.fastq") for k in whole)


def test_cli_matches_reference(tmp_path, hip_built):
    """python -m genomeanonymizer_amd.genome_anonymizer with the reference's flags."""
    import gzip
    import os
    import subprocess
    import sys
    from helpers import GOLDEN, REPO
    from genomeanonymizer_amd.synth.generate import generate, scenario
    d = str(tmp_path / "cli")
    paths = generate(scenario("edge"), d)
    env = dict(os.environ, PYTHONPATH=REPO, GANON_IO_BLOCK="4096")   # the fixtures' st_blksize
    r = subprocess.run([sys.executable, "-m", "genomeanonymizer_amd.genome_anonymizer", "-d", d, "-s", "samples.tsv",
                        "-r", paths["ref"], "--record_statistics", "-c", "4"], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    for tag, stem in (("tumor", "tumor"), ("normal", "normal")):
        for suf in (".1.fastq", ".2.fastq", ".single_end.fastq"):
            gp = os.path.join(GOLDEN, "edge", f"{tag}{suf}.gz")
            assert open(os.path.join(d, f"{stem}.anonymized{suf}"), "rb").read() == gzip.open(gp).read()
    assert open(paths["N"] + ".statistics.txt").read() == open(os.path.join(GOLDEN, "edge", "normal.statistics.txt")).read()


def test_cli_concurrent_pairs(tmp_path, hip_built):
    """-s listing several pairs: they run concurrently, one process and HIP context each on the one
    GPU (the reference's process pool, SR:944-961); every pair's files are the reference's."""
    import gzip
    import os
    import shutil
    import subprocess
    import sys
    from helpers import GOLDEN, REPO
    from genomeanonymizer_amd.synth.generate import generate, scenario
    d = str(tmp_path / "pairs")
    paths = generate(scenario("edge"), os.path.join(d, "a"))
    for sub in ("b", "c"):
        os.makedirs(os.path.join(d, sub))
        for f in ("tumor.bam", "normal.bam", "variants.vcf"):
            shutil.copy(os.path.join(d, "a", f), os.path.join(d, sub, f))
    with open(os.path.join(d, "samples.tsv"), "w") as fh:
        fh.write("#tumor\tnormal\tvcf\n")
        for sub in ("a", "b", "c"):
            fh.write(f"{sub}/tumor.bam\t{sub}/normal.bam\t{sub}/variants.vcf\n")
    env = dict(os.environ, PYTHONPATH=REPO, GANON_IO_BLOCK="4096")
    r = subprocess.run([sys.executable, "-m", "genomeanonymizer_amd.genome_anonymizer", "-d", d, "-s", "samples.tsv",
                        "-r", paths["ref"], "--record_statistics", "-c", "6"], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    for sub in ("a", "b", "c"):
        for tag in ("tumor", "normal"):
            for suf in (".1.fastq", ".2.fastq", ".single_end.fastq"):
                gp = os.path.join(GOLDEN, "edge", f"{tag}{suf}.gz")
                assert open(os.path.join(d, sub, f"{tag}.anonymized{suf}"), "rb").read() == gzip.open(gp).read()
        assert open(os.path.join(d, sub, "normal.bam.statistics.txt")).read() == \
            open(os.path.join(GOLDEN, "edge", "normal.statistics.txt")).read()


def test_cli_concurrent_pairs_error_reaches_caller(tmp_path, hip_built):
    """A pair that fails inside the process pool (GANON_PAIR_WORKERS=2: spawned children, a HIP context
    each) fails the run: its error comes back through the pool to the CLI, which exits non-zero and
    names it."""
    import os
    import shutil
    import subprocess
    import sys
    from helpers import REPO
    from genomeanonymizer_amd.synth.generate import generate, scenario
    d = str(tmp_path / "pairs")
    generate(scenario("edge"), os.path.join(d, "a"))
    os.makedirs(os.path.join(d, "b"))
    for f in ("normal.bam", "variants.vcf"):
        shutil.copy(os.path.join(d, "a", f), os.path.join(d, "b", f))
    with open(os.path.join(d, "b", "tumor.bam"), "wb") as fh:   # not a BGZF file
        fh.write(b"this is not a BAM file" * 64)
    with open(os.path.join(d, "samples.tsv"), "w") as fh:
        fh.write("#tumor\tnormal\tvcf\n")
        for sub in ("a", "b"):
            fh.write(f"{sub}/tumor.bam\t{sub}/normal.bam\t{sub}/variants.vcf\n")
    env = dict(os.environ, PYTHONPATH=REPO, GANON_PAIR_WORKERS="2")
    r = subprocess.run([sys.executable, "-m", "genomeanonymizer_amd.genome_anonymizer", "-d", d, "-s", "samples.tsv",
                        "-r", os.path.join(d, "a", "ref.fa"), "-c", "2"], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode != 0
    assert "b/tumor.bam" in r.stderr or "BGZF" in r.stderr, r.stderr[-2000:]


def test_hip_config2_matches_oracle(masker, oracle):
    """BASELINE configs[1] layout at 2 M reads: every byte and count equal to the oracle."""
    from genomeanonymizer_amd.synth.batch import config2_batch
    arr, info = config2_batch(n_reads=2_000_000, genome=600_000_000, n_windows=200_000, n_germline=200_000)
    o_out, o_calls, o_bases, o_tot = oracle.mask(arr)
    L = (arr["read_len"].astype(np.int64) + 1) // 2
    assert np.all(L == 75)
    out, calls, bases, tot = masker.mask(arr)
    assert np.array_equal(calls, o_calls)
    assert np.array_equal(bases, o_bases)
    assert np.array_equal(out, o_out)
    assert tot[2] == info["reads"]



@pytest.mark.parametrize("layout", ["dataset_major", "shuffled"])
def test_hip_buffer_layouts_match_oracle(masker, oracle, layout):
    """The product path's sequence layout (every tumor read, then every normal read:
    build_batch) gives each scope group one partition piece per dataset; a shuffled buffer
    leaves most written bytes outside their group's pieces (far-list masks). Bytes and counts
    equal the oracle's, and every read's masked bases equal those of the interleaved layout."""
    from genomeanonymizer_amd.synth.batch import config2_batch, dataset_major, relayout
    arr, _ = config2_batch(n_reads=400_000, genome=120_000_000, n_windows=40_000, n_germline=40_000)
    if layout == "dataset_major":
        dm = dataset_major(arr)
    else:
        dm = relayout(arr, np.random.default_rng(7).permutation(len(arr["read_len"])))
    o_out, o_calls, o_bases, _ = oracle.mask(dm)
    out, calls, bases, tot = masker.mask(dm)
    assert np.array_equal(calls, o_calls) and np.array_equal(bases, o_bases)
    assert np.array_equal(out, o_out)
    assert bases.sum() > 0
    out_i, calls_i, _, _ = masker.mask(arr)
    assert np.array_equal(calls_i, calls)
    nb = (arr["read_len"].astype(np.int64) + 1) // 2
    first = np.concatenate([[0], np.cumsum(nb)[:-1]])
    rel = np.arange(int(nb.sum()), dtype=np.int64) - np.repeat(first, nb)
    ia = np.repeat(arr["seq_off"].astype(np.int64), nb) + rel
    idm = np.repeat(dm["seq_off"].astype(np.int64), nb) + rel
    assert np.array_equal(out_i[ia], out[idm])


def test_hip_device_path_is_idempotent_and_deterministic(masker):
    """Running the same uploaded batch twice gives identical bytes and totals; masking the
    masked output again changes nothing for TN-masked bases (they now equal the ref)."""
    from genomeanonymizer_amd.synth.batch import config2_batch
    arr, _ = config2_batch(n_reads=200_000, genome=60_000_000, n_windows=20_000, n_germline=40_000)
    db = masker.upload(arr)
    db.run()
    db.sync()
    a = db.download()
    db.run()
    db.sync()
    b = db.download()
    db.free()
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[3], b[3])
    arr2 = dict(arr)
    arr2["seq_nt16"] = a[0]
    out2, calls2, bases2, _ = masker.mask(arr2)
    assert bases2.sum() == 0


def test_hip_empty_and_degenerate_batches(masker):
    from genomeanonymizer_amd.synth.batch import random_batch
    from genomeanonymizer_amd import native
    z = lambda dt: np.zeros(0, dt)
    empty = {"ref_start": z(np.int32), "read_len": z(np.int32), "seq_off": z(np.int64), "seq_nt16": z(np.uint8),
             "cig_off": z(np.int64), "n_cig": z(np.int32), "cigar": z(np.uint32), "dataset": z(np.uint8),
             "write_scope": z(np.int32), "scope_incid_off": np.zeros(1, np.int64), "incid_read": z(np.int32),
             "scope_span_start": z(np.int32), "scope_span_len": z(np.int32), "scope_ref_off": z(np.int64),
             "ref_nt16": z(np.uint8), "keep_pos": z(np.int32), "keep_code": z(np.uint8)}
    out, calls, bases, tot = masker.mask(empty)
    assert len(out) == 0 and tot[2] == 0
    arr = random_batch(3, n_scopes=10)
    bad = dict(arr)
    bad["write_scope"] = arr["write_scope"].copy()
    bad["write_scope"][0] = len(arr["scope_span_len"]) + 5
    with pytest.raises(native.GanonError):
        masker.mask(bad)
    bad = dict(arr)
    bad["scope_span_len"] = np.maximum(arr["scope_span_len"] - 10, 0).astype(np.int32)
    with pytest.raises(native.GanonError):
        masker.mask(bad)


@pytest.fixture(scope="module")
def c2_full():
    """BASELINE configs[1] at full size: the bench workload (10 M reads, 3.0 Gb, 1 M windows)."""
    from genomeanonymizer_amd.synth.batch import config2_batch
    arr, info = config2_batch()
    return arr, info


def test_hip_config2_full_size_matches_oracle_and_is_idempotent(masker, oracle, c2_full):
    """Full BASELINE configs[1] batch: every byte and count equal to the C oracle, and masking
    the masked output again masks nothing (each masked base now equals the reference)."""
    arr, info = c2_full
    assert info["reads"] == 10_000_000
    out, calls, bases, tot = masker.mask(arr)
    o_out, o_calls, o_bases, _ = oracle.mask(arr)
    assert np.array_equal(calls, o_calls)
    assert np.array_equal(bases, o_bases)
    assert np.array_equal(out, o_out)
    assert tot[1] == bases.sum() > 0
    del o_out
    arr2 = dict(arr)
    arr2["seq_nt16"] = out
    out2, calls2, bases2, _ = masker.mask(arr2)
    assert bases2.sum() == 0 and calls2.sum() == 0
    assert np.array_equal(out2, out)


def test_hip_fastq_full_size_matches_host_formatter(masker, c2_full):
    """10 M FASTQ records formatted on the device equal libganon_host.so's byte for byte."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.fastq import fastq_records
    arr, _ = c2_full
    recs = fastq_records(arr, seed=11, reverse_frac=0.5, name_len=(30, 45), check_bad=False)
    got = masker.format_fastq(recs)
    want = native.host_format_fastq(recs)
    assert len(got) == native.fastq_bytes(recs) == len(want)
    assert got == want


def test_hip_config2_indel_cigars_full_size_matches_oracle(oracle, hip_built):
    """BASELINE configs[1] at full size with realistic CIGARs (the bench's c2id line: 10 M reads,
    germline het deletions 0.1/kb and sequencing indels 1.5e-4/base, ~3 % of the reads aM dD/I bM),
    through the multi-segment fused path plus the germline indel tally, exactly as the bench steps
    it (upload, then speculative replans on a context that planned another batch in between), against
    the C oracle (every byte, per-scope calls and bases) and the indel restatement (every record).
    A parity bug of round 5 showed only at this size (runs crossing emptied sort segments)."""
    import indel_oracle
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch
    arr, info = config2_batch(germline_del_per_kb=0.1, seq_indel_per_base=1.5e-4)
    assert info["reads"] == 10_000_000 and info["indel_reads"] > 200_000
    o_out, o_calls, o_bases, _ = oracle.mask(arr)
    want_ind = native.indel_records_array(indel_oracle.indel_records(arr))
    assert len(want_ind) > 1000 and o_calls.sum() > 0
    small, _ = config2_batch(n_reads=150_000, genome=40_000_000, n_windows=12_000, n_germline=30_000, seed=77)
    m = native.HipMasker(0)
    try:
        ref = m.upload_reference(arr["ref_nt16"])
        db = m.upload({k: v for k, v in arr.items() if k != "ref_nt16"}, ref=ref)
        other = m.upload(small)
        assert db.shape()["prep_mode"] == "multi_segment_fused"
        ind = db.indel_tally(arr)
        for step in range(3):   # upload plan, then two fresh speculative replans after another batch's
            if step:
                other.replan()
                other.run()
                db.replan()
            db.run()
            ind.run()
            out, calls, bases, tot = db.download()
            got_ind = ind.download()
            assert np.array_equal(calls, o_calls), step
            assert np.array_equal(bases, o_bases), step
            assert np.array_equal(out, o_out), step
            assert tot[1] == bases.sum() and tot[2] == info["reads"], step
            assert np.array_equal(got_ind, want_ind), step
        ind.free()
        other.free()
        db.free()
        ref.free()
    finally:
        m.close()


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_hip_pipeline_matches_oracle_pipeline_on_random_scenarios(seed, tmp_path, hip_built):
    """Differential end-to-end check beyond the three golden scenarios: randomized samples with
    germline SNPs and indels, soft clips, N bases, unmapped / unplaced mates, cross-contig pairs and
    coverage holes, through the product (native planner, HIP masking + indel tally + HIP FASTQ) and
    through the oracle-backed pipeline (C oracle, indel restatement, FASTQ restatement, pinned by the
    reference's files in tests/test_oracle.py): every output file byte-identical."""
    import os
    from pyoracle import OracleEngine
    from genomeanonymizer_amd import short_read_tumor_normal_anonymizer as sr
    from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
    from genomeanonymizer_amd.synth.generate import ContigSpec, ScenarioConfig, generate
    rng = np.random.default_rng(seed)
    contigs = []
    for c in range(3):
        L = int(rng.integers(10_000, 40_000))
        wins, x = [], 1001 + int(rng.integers(0, 2000))
        while x < L - 1500 and len(wins) < 6:
            wins.append(x)
            x += 2003 + int(rng.integers(0, 6000))
        contigs.append(ContigSpec(f"chr{c}", L, int(rng.integers(100, 800)), windows=wins,
                                  keep_windows=int(rng.integers(0, 2)),
                                  holes=[("T" if rng.random() < 0.5 else "N", 3000, 3600)]))
    cfg = ScenarioConfig(name=f"d{seed}", seed=seed, contigs=contigs, germline_snp_per_kb=5.0,
                         germline_indel_per_kb=1.0, hom_fraction=0.3, softclip_frac=0.05,
                         unmapped_mate_frac=0.03, n_base_frac=0.03, unplaced_frac=0.4, cross_contig_pairs=8)
    paths = generate(cfg, str(tmp_path / "in"))
    outs = {}
    for tag, anon in (("hip", CompleteGermlineAnonymizer(device=0)),
                      ("oracle", CompleteGermlineAnonymizer(engine=OracleEngine()))):
        d = tmp_path / tag
        d.mkdir()
        t_out, n_out = str(d / "tumor"), str(d / "normal")
        sr.run_short_read_tumor_normal_anonymizer([paths["vcf"]], [(paths["T"], paths["N"])], paths["ref"], anon,
                                                  [(t_out, n_out)], True, 4)
        files = {}
        for pre in (t_out, n_out):
            for suf in (".1.fastq", ".2.fastq", ".single_end.fastq"):
                if os.path.exists(pre + suf):
                    files[os.path.basename(pre) + suf] = open(pre + suf, "rb").read()
        files["stats"] = open(paths["N"] + ".statistics.txt").read()
        outs[tag] = files
    assert outs["hip"].keys() == outs["oracle"].keys()
    for k in outs["hip"]:
        assert outs["hip"][k] == outs["oracle"][k], k
    assert len(outs["hip"]["tumor.1.fastq"]) > 10_000


@pytest.fixture(scope="module")
def masker_long(hip_built):
    """A context whose uploads always take the long-read prep (GANON_PARAM_PREP_LONG 1)."""
    from genomeanonymizer_amd import native
    m = native.HipMasker(0)
    m.set_param(native.PARAM_PREP_LONG, 1)
    yield m
    m.close()


@pytest.mark.parametrize("seed", [1, 3, 4, 8, 12])
def test_long_prep_on_short_batches_matches_oracle(masker_long, oracle, seed):
    """The long-read device prep (segment-weighted groups, one wave per incidence) forced on the
    edge-case batches: every read and count equal to the oracle, as the default prep gives."""
    from genomeanonymizer_amd.synth.batch import random_batch
    kw = {"rare_frac": 0.3} if seed % 3 == 0 else {}
    if seed % 4 == 0:
        kw["wide_scopes"] = 4
    arr = random_batch(seed, n_scopes=40, **kw)
    o_out, o_calls, o_bases, o_tot = oracle.mask(arr)
    in_batch = np.zeros(len(arr["read_len"]), bool)
    in_batch[arr["incid_read"]] = True
    out, calls, bases, tot = masker_long.mask(arr)
    bad = [r for r in _all_reads_equal(arr, out, o_out) if in_batch[r] or arr["write_scope"][r] >= 0]
    assert bad == []
    assert np.array_equal(calls, o_calls) and np.array_equal(bases, o_bases)


def test_long_prep_config2_matches_oracle(masker_long, oracle):
    from genomeanonymizer_amd.synth.batch import config2_batch
    arr, info = config2_batch(n_reads=400_000, genome=100_000_000, n_windows=40_000, n_germline=40_000)
    o_out, o_calls, o_bases, _ = oracle.mask(arr)
    out, calls, bases, tot = masker_long.mask(arr)
    assert np.array_equal(calls, o_calls)
    assert np.array_equal(bases, o_bases)
    assert np.array_equal(out, o_out)


def test_long_reads_c5_shape_groups_are_balanced(masker, oracle):
    """C5-shaped batch (reads of thousands of CIGAR ops): the long-read prep cuts groups on
    segments, so no group holds more than a few times the target (2816 segments in long-read mode
    since round 6: groups average at most twice that), and results equal the oracle."""
    from genomeanonymizer_amd.synth.batch import longread_batch
    arr, info = longread_batch(7, n_reads=400)
    o_out, o_calls, o_bases, _ = oracle.mask(arr)
    db = masker.upload(arr)
    try:
        bi = db.info()
        assert bi["groups"] * 2 * 2816 >= bi["segments"], bi
        db.run()
        out, calls, bases, tot = db.download()
    finally:
        db.free()
    assert np.array_equal(calls, o_calls)
    assert np.array_equal(bases, o_bases)
    assert np.array_equal(out, o_out)


@pytest.fixture(scope="module")
def masker_twopass(hip_built):
    """A context whose uploads take the two-pass per-group emit (GANON_PARAM_PREP_LONG 0)."""
    from genomeanonymizer_amd import native
    m = native.HipMasker(0)
    m.set_param(native.PARAM_PREP_LONG, 0)
    yield m
    m.close()


@pytest.mark.parametrize("seed", [2, 3, 4, 9])
def test_two_pass_prep_matches_oracle(masker_twopass, oracle, seed):
    """The default short-read prep is the one-segment emit; the two-pass emit stays selectable and
    exact."""
    from genomeanonymizer_amd.synth.batch import random_batch
    kw = {"rare_frac": 0.3} if seed % 3 == 0 else {}
    if seed % 4 == 0:
        kw["wide_scopes"] = 4
    arr = random_batch(seed, n_scopes=40, **kw)
    o_out, o_calls, o_bases, _ = oracle.mask(arr)
    in_batch = np.zeros(len(arr["read_len"]), bool)
    in_batch[arr["incid_read"]] = True
    out, calls, bases, tot = masker_twopass.mask(arr)
    bad = [r for r in _all_reads_equal(arr, out, o_out) if in_batch[r] or arr["write_scope"][r] >= 0]
    assert bad == []
    assert np.array_equal(calls, o_calls) and np.array_equal(bases, o_bases)


def test_replan_is_a_fresh_upload(masker, oracle):
    """ganon_batch_replan plans the resident raw arrays again from scratch (the bench's fresh-batch
    step): after reloading another batch and replanning, every run equals a one-shot mask; repeated
    replans leave nothing behind."""
    from genomeanonymizer_amd.synth.batch import config2_batch, random_batch
    a, _ = config2_batch(n_reads=150_000, genome=40_000_000, n_windows=12_000, n_germline=30_000, seed=21)
    b = random_batch(41, n_scopes=60, rare_frac=0.2, wide_scopes=3)
    want_a, want_b = masker.mask(a), masker.mask(b)
    db = masker.upload(a)
    try:
        for arr, want in ((a, want_a), (b, want_b), (a, want_a)):
            if db.seq_bytes != len(arr["seq_nt16"]) or arr is b:
                db.reload(arr)
            for _ in range(3):
                db.replan()
                db.run()
            got = db.download()
            for k in range(4):
                assert np.array_equal(got[k], want[k]), k
            assert db.shape()["prep_mode"].startswith("one_segment") or arr is b
    finally:
        db.free()
    o_out, o_calls, o_bases, _ = oracle.mask(a)
    assert np.array_equal(want_a[0], o_out) and np.array_equal(want_a[1], o_calls)


def _two_segment_copy(arr: dict, r: int) -> dict:
    """arr with read r's CIGAR replaced by 70M 5I 75M (same query length, shorter on the reference:
    two aligned segments, the read stays inside its scopes)."""
    b = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in arr.items()}
    assert int(b["n_cig"][r]) == 1 and int(b["read_len"][r]) == 150
    b["cig_off"][r] = len(b["cigar"])
    b["n_cig"][r] = 3
    b["cigar"] = np.concatenate([b["cigar"], np.array([70 << 4, (5 << 4) | 1, 75 << 4], np.uint32)])
    return b


# 9 aligned segments (query 150, 142 on the reference): one more than the fused mode takes
NINE_SEG = [(16, 0), (1, 1)] * 8 + [(14, 0)]


def test_speculative_plan_of_new_counts(hip_built):
    """Batches of other read / scope / incidence counts than the context's last plan speculate too
    (buffers sized from their counts, the context's last shape assumed, the scan gating the run):
    two resident batches of one sample replanned in turn give exactly their full plans' results; a
    batch with a two-segment read fits the fused shape (round 5: no gate); a batch that does not fit
    (a read of nine aligned segments) runs nothing, counts one gated run, and its download plans and
    runs it in full."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch
    kw = dict(genome=30_000_000, n_windows=10_000, n_germline=25_000, seed=34)
    a, _ = config2_batch(n_reads=120_000, read_seed=1, **kw)
    b, _ = config2_batch(n_reads=124_000, read_seed=2, **kw)
    assert len(a["read_len"]) != len(b["read_len"]) and len(a["incid_read"]) != len(b["incid_read"])
    cand = np.nonzero((b["write_scope"] >= 0) & (b["n_cig"] == 1) & (b["read_len"] == 150))[0]
    c = _recigar(b, int(cand[len(cand) // 2]), NINE_SEG)
    c2 = _two_segment_copy(b, int(cand[len(cand) // 3]))
    m = native.HipMasker(0)
    try:
        want = [m.mask(x) for x in (a, b, c, c2)]
        ref = m.upload_reference(a["ref_nt16"])
        dbs = [m.upload({k: v for k, v in x.items() if k != "ref_nt16"}, ref=ref) for x in (a, b, c, c2)]
        assert dbs[3].shape()["prep_mode"] == "multi_segment_fused"
        try:
            for _ in range(3):            # a, b, a, b, ...: every replan is of other counts
                for k in (0, 1):
                    dbs[k].replan()
                    dbs[k].run()
                    got = dbs[k].download()
                    assert all(np.array_equal(got[j], want[k][j]) for j in range(4))
            assert dbs[0].gated_runs() == 0 and dbs[1].gated_runs() == 0
            dbs[1].replan()               # (the context's last full shape: one-segment)
            dbs[1].run()
            dbs[3].replan()               # speculative; a two-segment read fits the fused shape
            dbs[3].run()
            got = dbs[3].download()
            assert dbs[3].gated_runs() == 0
            assert all(np.array_equal(got[j], want[3][j]) for j in range(4))
            dbs[2].replan()               # speculative; its nine-segment read stops the run
            dbs[2].run()
            assert dbs[2].gated_runs() == 1
            got = dbs[2].download()
            assert all(np.array_equal(got[j], want[2][j]) for j in range(4))
            assert dbs[2].shape()["max_seg"] == 9 and dbs[2].shape()["prep_mode"] == "two_pass"
            got = dbs[1].download()
            assert all(np.array_equal(got[j], want[1][j]) for j in range(4))
        finally:
            for d in dbs:
                d.free()
            ref.free()
    finally:
        m.close()


def test_speculative_replan_and_fallback(hip_built):
    """A replan after a one-segment plan of the same sizes is speculative (no synchronization); the
    scan's reduction gates the run. A batch that does not fit (a read with two segments) or fails
    validation runs nothing; ganon_batch_download plans it in full and runs it again, or returns the
    validation error. A read with two segments fits the fused shape (round 5) and runs as speculated;
    one with nine does not. GANON_PARAM_SPEC_PLAN 2 makes reloads speculate too (the testing knob)."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch
    a, _ = config2_batch(n_reads=120_000, genome=30_000_000, n_windows=10_000, n_germline=25_000, seed=33)
    cand = np.nonzero((a["write_scope"] >= 0) & (a["n_cig"] == 1) & (a["read_len"] == 150))[0]
    r = int(cand[len(cand) // 3])
    b = _recigar(a, r, NINE_SEG)
    b2 = _two_segment_copy(a, r)
    bad = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in a.items()}
    bad["seq_off"][r] = len(bad["seq_nt16"]) + 10
    m = native.HipMasker(0)
    try:
        want_a, want_b, want_b2 = m.mask(a), m.mask(b), m.mask(b2)
        m.set_param(native.PARAM_SPEC_PLAN, 2)
        db = m.upload(a)
        try:
            db.run()
            got = db.download()
            assert all(np.array_equal(got[k], want_a[k]) for k in range(4))
            assert db.shape()["prep_mode"].startswith("one_segment")   # (fused after a flat plan)
            db.reload(b2)         # speculative, fits: two segments in the fused mode
            db.run()
            got = db.download()
            assert all(np.array_equal(got[k], want_b2[k]) for k in range(4))
            assert db.gated_runs() == 0
            db.reload(b)          # speculative: the gate stops the run, download plans b in full
            db.run()
            got = db.download()
            assert all(np.array_equal(got[k], want_b[k]) for k in range(4))
            assert db.shape()["prep_mode"] == "two_pass" and db.shape()["max_seg"] == 9
            db.reload(a)          # b's plan was not one-segment: a full plan
            db.run()
            got = db.download()
            assert all(np.array_equal(got[k], want_a[k]) for k in range(4))
            for _ in range(3):    # speculative replans of the same contents
                db.replan()
                db.run()
            got = db.download()
            assert all(np.array_equal(got[k], want_a[k]) for k in range(4))
            db.reload(bad)        # speculative, invalid: nothing runs, download names the read
            db.run()
            with pytest.raises(native.GanonError, match="read"):
                db.download()
            db.reload(a)
            db.run()
            got = db.download()
            assert all(np.array_equal(got[k], want_a[k]) for k in range(4))
        finally:
            db.free()
    finally:
        m.close()


def test_far_list_overflow_grows_and_reruns(hip_built, oracle):
    """A far-mask list too small for the run (GANON_PARAM_FAR_INIT 1): k_finish reports the count it
    needed, ganon_batch_download grows the list and runs again — the bytes equal the oracle's."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch, relayout
    arr, _ = config2_batch(n_reads=200_000, genome=60_000_000, n_windows=20_000, n_germline=40_000, seed=8)
    sh = relayout(arr, np.random.default_rng(3).permutation(len(arr["read_len"])))
    o_out, o_calls, o_bases, _ = oracle.mask(sh)
    m = native.HipMasker(0)
    try:
        m.set_param(native.PARAM_FAR_INIT, 1)
        db = m.upload(sh)
        try:
            assert db.info()["far_capacity"] == 1
            db.run()
            out, calls, bases, tot = db.download()
            assert db.info()["far_capacity"] > 1
        finally:
            db.free()
    finally:
        m.close()
    assert o_bases.sum() > 10
    assert np.array_equal(out, o_out) and np.array_equal(calls, o_calls) and np.array_equal(bases, o_bases)


def _recigar(arr: dict, r: int, ops) -> dict:
    """arr with read r's CIGAR replaced by ops ((length, op code) pairs)."""
    b = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in arr.items()}
    b["cig_off"][r] = len(b["cigar"])
    b["n_cig"][r] = len(ops)
    b["cigar"] = np.concatenate([b["cigar"], np.array([(n << 4) | op for n, op in ops], np.uint32)])
    return b


def test_fused_one_segment_matches_record_pass(hip_built, oracle):
    """GANON_PARAM_FUSED_FLAT 1 (default): a one-segment batch builds no records in HBM — the scan's
    read descriptors and candidates feed the group kernel, which makes each incidence's record in LDS.
    Byte-equal to the record pass (PARAM 0) and the oracle on: a configs[1]-shaped batch; reads whose
    segment starts or ends more than 15 positions inside their reference span (the descriptor's wide
    form: 16D134M16S, 16S134M16D); a reference with N bases inside written reads' scopes (tiles that
    read the nt16 copy); a permuted buffer layout (candidates from unordered offsets); and the
    incidence errors, reported by the download in both modes."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch, relayout
    a, _ = config2_batch(n_reads=160_000, genome=40_000_000, n_windows=14_000, n_germline=40_000, seed=52)
    wr = np.nonzero((a["write_scope"] >= 0) & (a["n_cig"] == 1) & (a["read_len"] == 150))[0]
    b = _recigar(a, int(wr[100]), [(16, 2), (134, 0), (16, 4)])
    b = _recigar(b, int(wr[5000]), [(16, 4), (134, 0), (16, 2)])
    b = _recigar(b, int(wr[9000]), [(3, 2), (147, 0), (3, 4)])
    c = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in a.items()}
    for r in wr[::997][:40]:   # N bases in the reference under written reads
        s = int(c["write_scope"][r])
        nib = int(c["scope_ref_off"][s]) + int(c["ref_start"][r]) - int(c["scope_span_start"][s]) + 20
        c["ref_nt16"][nib // 2: nib // 2 + 4] = 0xFF
    d = relayout(a, np.random.default_rng(5).permutation(len(a["read_len"])))
    fused, rec = native.HipMasker(0), native.HipMasker(0)
    rec.set_param(native.PARAM_FUSED_FLAT, 0)
    try:
        for name, x in (("plain", a), ("wide", b), ("nref", c), ("layout", d)):
            o = oracle.mask(x)
            got_f, got_r = fused.mask(x), rec.mask(x)
            for k in range(3):
                assert np.array_equal(got_f[k], got_r[k]), (name, k)
                assert np.array_equal(got_f[k], o[k]), (name, k)
            assert np.array_equal(got_f[3], got_r[3]), name
            db = fused.upload(x)
            try:
                assert db.shape()["prep_mode"] == "one_segment_fused", name
            finally:
                db.free()
        assert o[2].sum() > 0
        for m in (fused, rec):
            bad = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in a.items()}
            bad["incid_read"][7] = len(a["read_len"]) + 3
            with pytest.raises(native.GanonError, match="out of range"):
                m.mask(bad)
            bad = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in a.items()}
            far = int(wr[np.nonzero(a["ref_start"][wr] > 500_000)[0][0]])
            bad["ref_start"][far] -= 100_000   # outside every scope that lists it
            with pytest.raises(native.GanonError, match="outside its span"):
                m.mask(bad)
    finally:
        fused.close()
        rec.close()


def test_fused_multi_segment_matches_record_pass(hip_built, oracle):
    """Short reads with I/D/N ops in the fused mode (round 5): the scan writes every segment of a read
    of 2-8 aligned segments as an extras record, the group kernel lists each such incidence on its
    first pass and streams the further segments after the group's incidences. Byte-equal to the
    record pass (the two-pass emit) and to the oracle on: a c2id-shaped batch (germline het deletions
    and sequencing indels, ~3 % of the reads aM dD/I bM); hand-made CIGARs of 2-8 segments (N skips,
    =/X runs, several I/D ops, a leading soft clip) with N bases in the reference under some of them;
    a shuffled buffer layout; a batch with a nine-segment read (the two-pass emit in both contexts);
    and the extras list grown from a capacity of 1 (GANON_PARAM_XREC_INIT 1: the plan scans again)."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch, relayout
    a, info = config2_batch(n_reads=200_000, genome=60_000_000, n_windows=20_000, n_germline=60_000, seed=61,
                            germline_del_per_kb=0.1, seq_indel_per_base=1.5e-4)
    assert 0.02 < info["indel_reads"] / info["reads"] < 0.05
    wr = np.nonzero((a["write_scope"] >= 0) & (a["n_cig"] == 1) & (a["read_len"] == 150))[0]
    shapes = [[(30, 0), (2, 2), (30, 0), (2, 1), (30, 0), (2, 2), (30, 0), (2, 1), (26, 0)],   # 5 segments
              [(50, 0), (20, 3), (80, 0), (20, 1)],                                         # N skip
              [(70, 7), (80, 8)],                                                           # = then X
              [(17, 0), (1, 1)] * 7 + [(24, 0)],                                            # 8 segments
              [(5, 4), (60, 0), (3, 1), (40, 0), (2, 2), (42, 0)]]                          # soft clip first
    b = a
    hand = []
    for k, r in enumerate(wr[37::211][:200]):
        b = _recigar(b, int(r), shapes[k % len(shapes)])
        hand.append(int(r))
    c = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in b.items()}
    for r in hand[::7]:   # N bases in the reference under multi-segment written reads
        s = int(c["write_scope"][r])
        nib = int(c["scope_ref_off"][s]) + int(c["ref_start"][r]) - int(c["scope_span_start"][s]) + 90
        c["ref_nt16"][nib // 2: nib // 2 + 3] = 0xFF
    d = relayout(b, np.random.default_rng(7).permutation(len(b["read_len"])))
    e = _recigar(b, int(wr[12345]), NINE_SEG)
    fused, rec, tiny = native.HipMasker(0), native.HipMasker(0), native.HipMasker(0)
    rec.set_param(native.PARAM_FUSED_FLAT, 0)
    tiny.set_param(native.PARAM_XREC_INIT, 1)
    try:
        for name, x, mode in (("c2id", a, "multi_segment_fused"), ("hand", b, "multi_segment_fused"),
                              ("nref", c, "multi_segment_fused"), ("layout", d, "multi_segment_fused"),
                              ("nine", e, "two_pass")):
            o = oracle.mask(x)
            got_f, got_r = fused.mask(x), rec.mask(x)
            for k in range(3):
                assert np.array_equal(got_f[k], got_r[k]), (name, k)
                assert np.array_equal(got_f[k], o[k]), (name, k)
            assert np.array_equal(got_f[3], got_r[3]), name
            db = fused.upload(x)
            try:
                assert db.shape()["prep_mode"] == mode, name
            finally:
                db.free()
            if name in ("c2id", "nref"):
                got_t = tiny.mask(x)
                assert all(np.array_equal(got_t[k], got_f[k]) for k in range(4)), name
        assert o[2].sum() > 0
    finally:
        fused.close()
        rec.close()
        tiny.close()


def test_fused_multi_segment_speculative_batches(hip_built):
    """c2id-shaped batches of other counts replanned in turn on one context (the bench's step): every
    plan speculates (no gated run) and every result equals the batch's full plan."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch
    kw = dict(genome=40_000_000, n_windows=12_000, n_germline=40_000, seed=62, germline_del_per_kb=0.1,
              seq_indel_per_base=1.5e-4)
    xs = [config2_batch(n_reads=n, read_seed=k, **kw)[0] for k, n in enumerate((150_000, 153_000, 147_000))]
    m = native.HipMasker(0)
    try:
        want = [m.mask(x) for x in xs]
        ref = m.upload_reference(xs[0]["ref_nt16"])
        dbs = [m.upload({k: v for k, v in x.items() if k != "ref_nt16"}, ref=ref) for x in xs]
        try:
            for _ in range(3):
                for k, db in enumerate(dbs):
                    db.replan()
                    db.run()
                    got = db.download()
                    assert all(np.array_equal(got[j], want[k][j]) for j in range(4)), k
            assert all(db.gated_runs() == 0 for db in dbs)
        finally:
            for db in dbs:
                db.free()
            ref.free()
    finally:
        m.close()


def test_plan_mode_does_not_depend_on_history(hip_built):
    """One context stepping one-segment and multi-segment (c2id-shaped) batches in turn: every result
    equals the batch's one-shot mask, and no plan falls back to the two-pass record path because of
    the batch before it (round 4's context stayed on the record pass after a non-flat plan: verdict
    r04 weak item 11). A speculative replan made for the other shape is gated and planned in full,
    so the switch step loses its speculation, not its result."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch
    kw = dict(genome=40_000_000, n_windows=12_000, n_germline=40_000, seed=63)
    xs = [config2_batch(n_reads=150_000, read_seed=0, **kw)[0],
          config2_batch(n_reads=152_000, read_seed=1, germline_del_per_kb=0.1, seq_indel_per_base=1.5e-4, **kw)[0],
          config2_batch(n_reads=148_000, read_seed=2, **kw)[0]]
    m = native.HipMasker(0)
    try:
        want = [m.mask(x) for x in xs]
        ref = m.upload_reference(xs[0]["ref_nt16"])
        dbs = [m.upload({k: v for k, v in x.items() if k != "ref_nt16"}, ref=ref) for x in xs]
        try:
            for _ in range(2):
                for k, db in enumerate(dbs):
                    db.replan()
                    db.run()
                    got = db.download()
                    assert all(np.array_equal(got[j], want[k][j]) for j in range(4)), k
                    assert db.shape()["prep_mode"] in ("one_segment_fused", "multi_segment_fused"), (k, db.shape())
        finally:
            for db in dbs:
                db.free()
            ref.free()
    finally:
        m.close()


def test_incidence_errors_are_reported_by_download(masker):
    """The incidence checks run inside the device prep of every run: a read listed outside its
    scope's span, or a read index out of range, fails the download (GANON_E_ARG), never a fault."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import random_batch
    arr = random_batch(5, n_scopes=16)
    bad = dict(arr)
    bad["incid_read"] = arr["incid_read"].copy()
    bad["incid_read"][3] = len(arr["read_len"]) + 100
    db = masker.upload(bad)
    try:
        db.run()
        with pytest.raises(native.GanonError, match="out of range"):
            db.download()
    finally:
        db.free()
    bad = dict(arr)
    bad["write_scope"] = arr["write_scope"].copy()
    r = int(np.nonzero(arr["write_scope"] >= 0)[0][0])
    others = [s for s in range(len(arr["scope_span_len"])) if s != arr["write_scope"][r]]
    # a scope that does not list read r (the write-scope check after the masking kernels)
    lists = {s: set(arr["incid_read"][arr["scope_incid_off"][s]:arr["scope_incid_off"][s + 1]].tolist()) for s in others}
    s_bad = next(s for s in others if r not in lists[s])
    bad["write_scope"][r] = s_bad
    with pytest.raises(native.GanonError, match="does not list it exactly once"):
        masker.mask(bad)
