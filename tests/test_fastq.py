"""FASTQ record formatter: the HIP formatter (ganon_fastq_*,
include/ganon.h) against the restatement of the reference's record code
(oracle/fastq_oracle.py — pinned against the reference's own FASTQ files by the pipeline
tests in test_oracle.py, which format through it), and the host formatter against both.

Edge cases: N / IUPAC / '=' bases (forward: printed; reverse: the reference's KeyError,
SURVEY Q7, reported as the first bad record), zero-length reads and names, reversed and
stored-order qualities (Q1), records longer than an output tile (long reads), tiles holding
more records than the kernel stages in LDS (tiny records), empty record sets.
"""
import numpy as np
import pytest

import fastq_oracle
from genomeanonymizer_amd import native
from genomeanonymizer_amd.synth.fastq import bad_for_reverse, fastq_records


def _edge_records(seed, allow_bad=False, **kw):
    from genomeanonymizer_amd.synth.batch import random_batch
    arr = random_batch(seed, n_scopes=30, rare_frac=0.3)
    return arr, fastq_records(arr, seed=seed, allow_bad=allow_bad, qual_rev_frac=0.3, name_len=(0, 30), **kw)


def _tiny_records(n=6000, seed=3):
    """Records of 8-14 bytes: a 16 KiB output tile holds >1000 of them."""
    rng = np.random.default_rng(seed)
    seq_len = rng.integers(0, 4, n).astype(np.int32)
    nib = np.concatenate([[0], np.cumsum(seq_len.astype(np.int64))[:-1]]).astype(np.int64)
    codes = rng.choice(np.array([1, 2, 4, 8, 15], np.uint8), int(seq_len.sum()) + 2)
    seq = (codes[0::2][: (len(codes) + 1) // 2] << 4).astype(np.uint8)
    seq[: len(codes[1::2])] |= codes[1::2]
    name_len = rng.integers(0, 3, n).astype(np.int32)
    return {
        "seq_bufs": [seq], "seq_sel": np.zeros(n, np.uint8), "seq_nib_off": nib, "seq_len": seq_len,
        "reverse": (rng.random(n) < 0.5).astype(np.uint8),
        "qual_bufs": [rng.integers(2, 41, int(seq_len.sum()) + 1, dtype=np.uint8)],
        "qual_sel": np.zeros(n, np.uint8), "qual_off": nib.copy(), "qual_len": seq_len.copy(),
        "qual_rev": np.zeros(n, np.uint8), "names": rng.integers(65, 91, int(name_len.sum()) + 1, dtype=np.uint8),
        "name_off": np.concatenate([[0], np.cumsum(name_len.astype(np.int64))[:-1]]).astype(np.int64),
        "name_len": name_len, "mate": (1 + np.arange(n) % 2).astype(np.uint8),
    }


def _first_bad(recs):
    try:
        fastq_oracle.format_records(recs)
    except fastq_oracle.BadRecord as e:
        return e.index
    return None


# ---- CPU: oracle vs the host formatter ----------------------------------------------------

@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_host_formatter_matches_oracle(seed):
    arr, recs = _edge_records(seed)
    assert native.host_format_fastq(recs) == fastq_oracle.format_records(recs)


def test_host_formatter_tiny_records_match_oracle():
    recs = _tiny_records()
    assert native.host_format_fastq(recs) == fastq_oracle.format_records(recs)


def test_host_formatter_reports_first_bad_reverse_read():
    arr, recs = _edge_records(7, allow_bad=True, reverse_frac=0.9)
    bad = _first_bad(recs)
    assert bad is not None
    with pytest.raises(native.FastqBadRecord) as ei:
        native.host_format_fastq(recs)
    assert ei.value.index == bad


def test_bad_for_reverse_flags_non_acgtn_reads():
    arr, recs = _edge_records(8)
    flags = bad_for_reverse(arr["seq_nt16"], recs["seq_nib_off"], recs["seq_len"])
    for i in range(len(flags)):
        one = {k: (v[i:i + 1] if isinstance(v, np.ndarray) and len(v) == len(flags) else v) for k, v in recs.items()}
        one["reverse"] = np.ones(1, np.uint8)
        assert (_first_bad(one) is not None) == bool(flags[i])


# ---- GPU: the HIP formatter ----------------------------------------------------------------

@pytest.fixture(scope="module", params=[0, 15, 17, 13, 14, 16, 12, 9, 11, 3],
                ids=["span3", "span3_search", "span3_coarse", "span2", "span2_t2", "quad2", "rows", "quad1",
                     "quad2_select", "dword3"])
def masker(hip_built, request):
    """Every HIP formatter test runs on the span kernel (GANON_PARAM_FASTQ_KD 0, the default: 3 units
    per lane; 13 / 14: 2 per lane, one / two 8 KiB tiles per workgroup), the quad kernel (16, the
    default up to round 4; 9 = one quad per lane; 11 = the per-dword base select of round 1), the
    record-row kernel (12) and the dword kernel (3)."""
    m = native.HipMasker(0)
    m.set_param(native.PARAM_FASTQ_KD, request.param)
    yield m
    m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_hip_formatter_matches_oracle_edge_records(masker, seed):
    arr, recs = _edge_records(seed)
    assert masker.format_fastq(recs) == fastq_oracle.format_records(recs)


@pytest.mark.gpu
def test_hip_formatter_tiny_records(masker):
    recs = _tiny_records()
    assert masker.format_fastq(recs) == fastq_oracle.format_records(recs)


@pytest.mark.gpu
def test_hip_formatter_long_records(masker):
    from genomeanonymizer_amd.synth.batch import longread_batch
    arr, _ = longread_batch(5, n_reads=60)
    recs = fastq_records(arr, seed=5, qual_rev_frac=0.5)
    assert masker.format_fastq(recs) == native.host_format_fastq(recs)
    head = {k: (v[:6] if isinstance(v, np.ndarray) and len(v) == len(recs["seq_len"]) else v) for k, v in recs.items()}
    assert masker.format_fastq(head) == fastq_oracle.format_records(head)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [7, 9])
def test_hip_formatter_reports_first_bad_reverse_read(masker, seed):
    arr, recs = _edge_records(seed, allow_bad=True, reverse_frac=0.9)
    bad = _first_bad(recs)
    assert bad is not None
    with pytest.raises(native.FastqBadRecord) as ei:
        masker.format_fastq(recs)
    assert ei.value.index == bad


@pytest.mark.gpu
def test_hip_formatter_empty(masker):
    recs = _tiny_records(n=0)
    assert masker.format_fastq(recs) == b""


@pytest.mark.gpu
def test_hip_formatter_over_resident_batch(masker):
    """Records read straight from a device masking batch (masked output and input buffers),
    several runs: identical bytes each time, equal to formatting the downloaded output."""
    from genomeanonymizer_amd.synth.batch import config2_batch
    arr, _ = config2_batch(n_reads=200_000, genome=60_000_000, seed=4)
    db = masker.upload(arr)
    db.run()
    out, _, _, _ = db.download()
    recs = fastq_records(arr, seed=4)
    recs["seq_sel"] = (np.arange(len(recs["seq_len"])) % 3 == 0).astype(np.uint8)   # 1 = unmasked input
    host = dict(recs, seq_bufs=[out, arr["seq_nt16"]])
    expect = native.host_format_fastq(host)
    f = masker.fastq_upload(recs, seq_batch=db)
    try:
        for _ in range(3):
            f.run()
            assert f.download() == expect
    finally:
        f.free()
        db.free()
    n = 2000
    head = {k: (v[:n] if isinstance(v, np.ndarray) and len(v) == len(recs["seq_len"]) else v) for k, v in host.items()}
    assert native.host_format_fastq(head) == fastq_oracle.format_records(head)


@pytest.mark.gpu
def test_hip_formatter_config2_size_properties(masker):
    """A 2 M-read config-2 record set (every read, half of them reverse): the output is
    the size the record lengths give and byte-identical to the host formatter's."""
    from genomeanonymizer_amd.synth.batch import config2_batch
    arr, _ = config2_batch(n_reads=2_000_000, genome=600_000_000, seed=2)
    recs = fastq_records(arr, seed=2)
    got = masker.format_fastq(recs)
    exp = native.host_format_fastq(recs)
    assert len(got) == native.fastq_bytes(recs)
    assert got == exp


# ---- CPU: the output stage's per-job pre-formatting (writer.FastqFormatter.preformat) ----------

def _toy_tables():
    """Two small read tables (tumor 5 reads, normal 3) with one reverse tumor read holding an IUPAC
    base: formatting it is the reference's KeyError (Q7) — but only if it is written."""
    from types import SimpleNamespace
    rng = np.random.default_rng(7)
    tabs = []
    for ds, n in ((0, 5), (1, 3)):
        L = rng.integers(5, 40, n).astype(np.int32)
        seq_off = np.concatenate([[0], np.cumsum((L + 1) // 2)[:-1]]).astype(np.int64)
        seq = rng.choice(np.array([0x12, 0x48, 0x81, 0x24, 0xF1], np.uint8), int(((L + 1) // 2).sum()))
        qual_off = np.concatenate([[0], np.cumsum(L)[:-1]]).astype(np.int64)
        qual = rng.integers(2, 41, int(L.sum()), dtype=np.uint8)
        names = [f"r{ds}_{i}".encode() for i in range(n)]
        blob = np.frombuffer(b"".join(names), np.uint8)
        name_len = np.array([len(x) for x in names], np.int32)
        rev = (np.arange(n) % 2).astype(np.uint8)
        if ds == 0:
            seq[seq_off[1]] = 0x31            # read 1 (reverse): an 'M' first base
        t = SimpleNamespace(n=n, seq=seq, qual=qual, names_blob=blob, seq_off=seq_off, l_seq=L, qual_off=qual_off,
                            name_len=name_len, name_off=np.concatenate([[0], np.cumsum(name_len)[:-1]]).astype(np.int64),
                            flag=np.where(np.arange(n) % 2, 0x80, 0x40).astype(np.int64), is_reverse=rev)
        t.name = (lambda t_: (lambda r: bytes(t_.names_blob[t_.name_off[r]:t_.name_off[r] + t_.name_len[r]]).decode()))(t)
        tabs.append(t)
    res = SimpleNamespace(seq_out=np.zeros(1, np.uint8), seq_base=(0, 0), leftovers={})
    return tuple(tabs), res


def test_preformat_slices_match_direct_formatting_and_defer_q7():
    from genomeanonymizer_amd.writer import FastqFormatter
    tables, res = _toy_tables()
    ds = np.array([0] * 5 + [1] * 3, np.int64)
    row = np.array([0, 1, 2, 3, 4, 0, 1, 2], np.int64)
    sc = np.full(8, -1, np.int64)
    direct = FastqFormatter(tables, res)
    pre = FastqFormatter(tables, res)
    pre.preformat(ds, row, sc)
    assert pre._pre is not None and len(pre._pre.keys) == 7      # the Q7 read left out, not raised
    good = np.array([0, 2, 3, 4, 5, 6, 7])
    order = good[::-1]                                            # any order, any subset
    assert pre._native(ds[order], row[order], sc[order]) == direct._native(ds[order], row[order], sc[order])
    with pytest.raises(TypeError, match="r0_1"):                  # raised when it is written
        pre._native(ds[:3], row[:3], sc[:3])
    assert pre.unedited([(1, 2, -1), (0, 4, -1)]) == [direct._native(np.array([1]), np.array([2]), np.array([-1])),
                                                      direct._native(np.array([0]), np.array([4]), np.array([-1]))]


def test_preformat_by_row_matches_direct_formatting():
    """preformat's structured case (Job._format_instances: every read once in row order, then further
    copies): the reads' own records found by row, the others by key — duplicates of a read's own copy
    dropped — equal to formatting directly, in any order; a refused read falls back to the keyed case."""
    from genomeanonymizer_amd.writer import FastqFormatter
    tables, res = _toy_tables()
    tables[0].seq[tables[0].seq_off[1]] = 0x12        # (no Q7 read: the structured case holds)
    nb = tables[0].n + tables[1].n
    ds = np.array([0] * 5 + [1] * 3 + [0, 1, 0, 0], np.int64)
    row = np.array([0, 1, 2, 3, 4, 0, 1, 2, 2, 1, 3, 2], np.int64)
    sc = np.array([-1] * 8 + [-1, -1, -1, -1], np.int64)
    sc[nb:] = [-1, -1, -1, -1]
    direct = FastqFormatter(tables, res)
    pre = FastqFormatter(tables, res)
    assert pre.preformat(ds, row, sc, n_base=nb)
    assert pre._pre.base is not None and len(pre._pre.keys) == 0      # every extra is a read's own copy
    order = np.random.default_rng(1).permutation(nb)
    assert pre._native(ds[order], row[order], sc[order]) == direct._native(ds[order], row[order], sc[order])
    # the Q7 read: refused by the formatter -> the keyed case, the read left out
    tables2, res2 = _toy_tables()
    pre2 = FastqFormatter(tables2, res2)
    pre2.preformat(ds, row, sc, n_base=nb)
    assert pre2._pre.base is None and len(pre2._pre.keys) == 7
