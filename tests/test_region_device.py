"""Region reads decoded on the device (ganon_region_decode, include/ganon.h; the reader's region
decoder, ganon_bam_reader_set_region_decoder, include/ganon_host.h): a region read's first window is
inflated, walked (cut mode: the window may end inside a record), cut at the region's end and filtered
by htslib's overlap test on the GPU, and the kept records' columns come back in one page-locked
block. Every table must equal the host reader's (ganon_bam_reader_region, the reference's
AlignmentFile.fetch(contig, beg, end), short_read_tumor_normal_anonymizer.py:570-573) column for
column and blob for blob — on multi-window pairs, on the edge / long-read / fuzz scenarios (unplaced
records at the end of the file, records longer than the walk's 2 KiB chunks), on regions past a
contig's end, empty and one-base regions, and through the host fallback (a window too small for the
region hands its inflated bytes back to the host walk)."""
import dataclasses
import os

import numpy as np
import pytest

COLS = ("tid", "pos", "end", "flag", "mapq", "l_seq", "n_cigar", "mate_tid", "mate_pos", "tlen", "name_len",
        "aux_len", "name_off", "cig_off", "seq_off", "qual_off", "aux_off", "names_blob", "cigar", "seq", "qual",
        "aux")


def _regions(L: int, rng, k: int):
    out = [(0, L), (0, L + 1000), (L - 1, L + 5), (0, 1), (L // 2, L // 2), (L // 3, L // 3 + 1)]
    for _ in range(k):
        a = int(rng.integers(0, L))
        out.append((a, int(min(L + 10, a + rng.integers(1, max(2, L // 3))))))
    return out


def _compare(paths, inflater, window, rng, k=12):
    from genomeanonymizer_amd.io.bam import BamReader
    n_tables = 0
    for path in paths:
        ref = BamReader(path, 4)
        dev = BamReader(path, 4, window, inflater=inflater)
        assert ref.has_index
        for tid, L in enumerate(ref.ref_lens):
            for a, b in _regions(int(L), rng, k):
                exp, got = ref.region(tid, a, b), dev.region(tid, a, b)
                assert got.n == exp.n, (path, tid, a, b)
                for f in COLS:
                    assert np.array_equal(np.asarray(getattr(got, f)), np.asarray(getattr(exp, f))), (path, tid, a, b, f)
                n_tables += 1
        dev.close()
        ref.close()
    return n_tables


@pytest.fixture(scope="module")
def inflater(hip_built):
    from genomeanonymizer_amd import native
    g = native.GpuInflater(0, min_blocks=1)
    yield g
    g.close()


@pytest.mark.gpu
def test_device_regions_equal_host_regions_on_pairs(inflater, tmp_path):
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.fastpair import make_pair
    d = str(tmp_path / "in")
    make_pair(d, n_contigs=3, contig_len=600_000, pairs_per_contig=30_000, window_every=20_000)
    paths = [os.path.join(d, f"{k}.bam") for k in ("tumor", "normal")]
    native.decode_phase_times(reset=True)
    n = _compare(paths, inflater, 0, np.random.default_rng(5))
    ph = native.decode_phase_times(reset=True)
    assert n > 0 and ph["device_regions"] > 0.8 * n, ph     # (empty regions read nothing)
    # a window of 128 KiB: the decoder's first window is at most 16 of them, so the larger regions go
    # on past it and the host walk takes over from the bytes it inflated
    n = _compare(paths, inflater, 1 << 17, np.random.default_rng(6))
    ph = native.decode_phase_times(reset=True)
    assert ph["device_fallbacks"] > 0 and ph["device_regions"] > 0, ph


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["edge", "long1", "fuzz3500", "config1"])
def test_device_regions_equal_host_regions_on_scenarios(inflater, name, tmp_path):
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.generate import generate, scenario
    cfg = dataclasses.replace(scenario(name), bam_index=True)
    p = generate(cfg, str(tmp_path / "in"))
    native.decode_phase_times(reset=True)
    n = _compare([p["T"], p["N"]], inflater, 0, np.random.default_rng(len(name)), k=20)
    ph = native.decode_phase_times(reset=True)
    assert n > 0 and ph["device_regions"] > 0, ph
