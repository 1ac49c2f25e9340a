"""Germline indel tally.

CPU: the restatement (oracle/indel_oracle.py) on hand-built scopes with known answers from the
reference's arithmetic (variation_classifier.py:52-141, anonymizer_methods.py:537-556); it is
also pinned end-to-end by the reference's FASTQ/statistics files (tests/test_oracle.py runs the
pipeline with the oracle standing in for the device; tiny/edge/config1 hold germline indels).
GPU (marked): ganon_indel_* through the C ABI, record-for-record against the restatement.
"""
import numpy as np
import pytest

from genomeanonymizer_amd.synth.batch import _cigar_word, pack_nibbles

NT = {c: i for i, c in enumerate("=ACMGRSVTWYHKDBN")}


def _cig(s: str):
    out, num = [], ""
    for ch in s:
        if ch.isdigit():
            num += ch
        else:
            out.append(_cigar_word(ch, int(num)))
            num = ""
    return out


def scope_batch(ref: str, reads, n_scopes: int = 1):
    """reads: (scope list, pos, cigar, seq, dataset, write_scope). Incidences per scope: tumor
    then normal, file order (build_batch's layout)."""
    from genomeanonymizer_amd.synth.batch import _ref_end
    seq_parts, cig_parts, so, co = [], [], 0, 0
    seq_off, cig_off = [], []
    for _, pos, cg, sq, _, _ in reads:
        pk = pack_nibbles(np.array([NT[c] for c in sq], np.uint8))
        seq_parts.append(pk)
        seq_off.append(so)
        so += len(pk)
        words = _cig(cg)
        cig_parts.append(np.array(words, np.uint32))
        cig_off.append(co)
        co += len(words)
    ends = [_ref_end(r[1], _cig(r[2])) for r in reads]
    incid, offs, ss, sl = [], [0], [], []
    for s in range(n_scopes):
        ids = sorted([i for i, r in enumerate(reads) if s in r[0]], key=lambda i: (reads[i][4], i))
        incid.extend(ids)
        offs.append(len(incid))
        a = min(reads[i][1] for i in ids)
        ss.append(a)
        sl.append(max(ends[i] for i in ids) - a)
    return {
        "ref_start": np.array([r[1] for r in reads], np.int32),
        "read_len": np.array([len(r[3]) for r in reads], np.int32),
        "seq_off": np.array(seq_off, np.int64),
        "seq_nt16": np.concatenate(seq_parts),
        "cig_off": np.array(cig_off, np.int64),
        "n_cig": np.array([len(_cig(r[2])) for r in reads], np.int32),
        "cigar": np.concatenate(cig_parts),
        "dataset": np.array([r[4] for r in reads], np.uint8),
        "write_scope": np.array([r[5] for r in reads], np.int32),
        "scope_incid_off": np.array(offs, np.int64),
        "incid_read": np.array(incid, np.int32),
        "scope_span_start": np.array(ss, np.int32),
        "scope_span_len": np.array(sl, np.int32),
        "scope_ref_off": np.array(ss, np.int64),
        "ref_nt16": pack_nibbles(np.array([NT[c] for c in ref], np.uint8)),
        "keep_pos": np.full(n_scopes, -1, np.int32),
        "keep_code": np.zeros(n_scopes, np.uint8),
    }


REF = "ACGTACGTAC" * 10


def known_answer_batch():
    """Scope 0 over REF[0:100):
    r0 T 10M2I10M  at 5: INS pos 15, in_read_pos 10, allele GG
    r1 N 3H10M2I10M at 5: H counts toward in_read_pos (13): the allele is read at
                          seq[13:15], which this read makes GG -> the same call as r0 (TN)
    r2 N 10M2I10M  at 5: INS at 15 with another allele (TT): a second call at 15, rank 1
    r3 T 8M3D12M   at 30: DEL pos 38 len 3, allele = 2 read bases after the gap
    r4 N 8M3D12M   at 30: same DEL (TN) — written by scope 0
    r5 T 12M2D     at 60: trailing DEL at 72, allele clipped to '' ; N r6 covers 72 -> TN
    r6 N 12M2D     at 60
    r7 T 20M1I     at 75: trailing INS at pos 95 = reference_end; no normal read covers 95
    r8 N 20M1I     at 75:   -> TN but never masked (no normal column at 95)
    """
    gg = REF[5:15] + "GG" + REF[15:25]
    tt = REF[5:15] + "TT" + REF[15:25]
    d38 = REF[30:38] + REF[41:53]
    reads = [
        ([0], 5, "10M2I10M", gg, 0, 0),
        ([0], 5, "3H10M2I10M", REF[5:15] + "GGGGG" + REF[18:25], 1, 0),
        ([0], 5, "10M2I10M", tt, 1, -1),
        ([0], 30, "8M3D12M", d38, 0, -1),
        ([0], 30, "8M3D12M", d38, 1, 0),
        ([0], 60, "12M2D", REF[60:72], 0, 0),
        ([0], 60, "12M2D", REF[60:72], 1, 0),
        ([0], 75, "20M1I", REF[75:95] + "A", 0, 0),
        ([0], 75, "20M1I", REF[75:95] + "A", 1, 0),
    ]
    return scope_batch(REF, reads)


def test_indel_oracle_known_answers():
    import indel_oracle
    recs = sorted(indel_oracle.indel_records(known_answer_batch()))
    # (scope, pos, length, type, rank, kind, read, in_read_pos)
    assert recs == sorted([
        (0, 15, 2, 3, 0, 0, 0, 10), (0, 15, 2, 3, 0, 1, 0, 10), (0, 15, 2, 3, 0, 1, 1, 13),
        (0, 38, 3, 2, 0, 0, 3, 8), (0, 38, 3, 2, 0, 1, 4, 8),
        (0, 72, 2, 2, 0, 0, 5, 12), (0, 72, 2, 2, 0, 1, 5, 12), (0, 72, 2, 2, 0, 1, 6, 12),
    ])


def test_indel_oracle_rank_follows_registration_order():
    """Two calls at one position: the one whose first support the reference meets first (lower
    ref_start, then tumor before normal, then file order) is rank 0, whatever the slot order."""
    import indel_oracle
    a = REF[10:15] + "C" + REF[15:30]
    b = REF[12:15] + "GA" + REF[15:30]
    reads = [
        ([0], 12, "3M2I15M", b, 0, 0),     # allele GA, registered at column 12
        ([0], 10, "5M1I15M", a, 1, 0),     # allele C, registered at column 10 -> rank 0
        ([0], 10, "5M1I15M", a, 0, 0),
        ([0], 12, "3M2I15M", b, 1, 0),
    ]
    recs = indel_oracle.indel_records(scope_batch(REF, reads))
    ranks = {(r[2], r[5], r[6]): r[4] for r in recs}
    assert ranks[(1, 0, 2)] == 0 and ranks[(2, 0, 0)] == 1


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_hip_indel_tally_matches_oracle(seed, hip_built):
    import indel_oracle
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import indel_batch
    arr = indel_batch(seed)
    want = native.indel_records_array(indel_oracle.indel_records(arr))
    assert len(want) > 50
    m = native.HipMasker(0)
    try:
        *_, got = m.mask(arr, indels=True)
        m.set_param(native.PARAM_INDEL_SORT, 1)
        *_, got_global = m.mask(arr, indels=True)
    finally:
        m.close()
    assert np.array_equal(got, want)
    assert np.array_equal(got_global, want)


@pytest.mark.gpu
def test_hip_indel_known_answers_and_random_batches(hip_built):
    import indel_oracle
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import random_batch
    m = native.HipMasker(0)
    try:
        for arr in [known_answer_batch()] + [random_batch(s, n_scopes=24, wide_scopes=1) for s in (5, 6)]:
            want = native.indel_records_array(indel_oracle.indel_records(arr))
            *_, got = m.mask(arr, indels=True)
            assert np.array_equal(got, want)
    finally:
        m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"GANON_INDEL_WAVE_WALK": "1"}, {"GANON_INDEL_DENSE_MAP": "1"},
                                 {"GANON_INDEL_SORTMODE": "seg"}, {"GANON_INDEL_SORTMODE": "global"}],
                         ids=["thread_walk_hashed_tsort", "wave_walk", "dense_map", "segmented_sort", "global_sort"])
def test_hip_indel_short_read_paths_match_oracle(env, hip_built, monkeypatch):
    """Short-read batches (round 5): the candidate walks and the incidence expansion take a thread per
    read / incidence, the candidate map is hashed (2 bits per cell, 64 cells per op: a collision can
    only add a position), and the filtered observations, already scope-major, are sorted in place per
    scope (k_indel_tsort). Equal to the oracle, and to the wave-per-block walks, the dense genome map,
    rocPRIM's segmented sort and one global 64-bit sort (the A/B switches, read at indel upload), on
    dense indel batches and on a c2id-shaped batch (germline het deletions + sequencing indels, ~3 % of
    the reads)."""
    import indel_oracle
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import config2_batch, indel_batch
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    c2id, _ = config2_batch(n_reads=60_000, genome=6_000_000, n_windows=1_800, n_germline=6_000, seed=71,
                            germline_del_per_kb=0.3, seq_indel_per_base=3e-4)
    m = native.HipMasker(0)
    try:
        for arr in (indel_batch(5), indel_batch(6, indel_per_kb=30.0), c2id):
            want = native.indel_records_array(indel_oracle.indel_records(arr))
            assert len(want) > 20
            *_, got = m.mask(arr, indels=True)
            assert np.array_equal(got, want)
    finally:
        m.close()


def empty_segment_batch():
    """Three scopes of one contig, each call at the same position relative to its span: scopes 0 and 2
    hold a TN deletion (a tumor and a normal read), scope 1 a tumor-only one that the T∧N candidate
    filter removes — so scope 1's sort segment is empty and scopes 0 and 2 (one segment parity) meet in
    the sorted array with equal 32-bit keys (round 5's segmented-sort bug, tools/indel_ab.py)."""
    ref = "ACGTACGTAC" * 30
    reads = []
    for s, base in ((0, 5), (1, 105), (2, 205)):
        allele = ref[base:base + 8] + ref[base + 10:base + 22]
        reads.append(([s], base, "8M2D12M", allele, 0, s))
        if s != 1:
            reads.append(([s], base, "8M2D12M", allele, 1, s))
    return scope_batch(ref, reads, n_scopes=3)


def test_indel_oracle_empty_segment_batch():
    import indel_oracle
    recs = indel_oracle.indel_records(empty_segment_batch())
    calls = sorted((r[0], r[1]) for r in recs if r[5] == 0)
    assert calls == [(0, 13), (2, 213)]


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"GANON_INDEL_SORTMODE": "seg"}, {"GANON_INDEL_SORTMODE": "global"},
                                 {"GANON_INDEL_WAVE_WALK": "1"}],
                         ids=["segment_sort", "segmented_sort", "global_sort", "wave_walk"])
def test_hip_indel_runs_never_cross_scopes(env, hip_built, monkeypatch):
    """Equal sort keys of two scopes whose segments an emptied segment separates stay two runs: the
    segmented path marks every segment's first element (k_indel_segs) and a run stops there."""
    import indel_oracle
    from genomeanonymizer_amd import native
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    arr = empty_segment_batch()
    want = native.indel_records_array(indel_oracle.indel_records(arr))
    m = native.HipMasker(0)
    try:
        *_, got = m.mask(arr, indels=True)
    finally:
        m.close()
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_hip_indel_long_reads_match_oracle(hip_built):
    """C5 shape: 10-100 kb reads with ~5 % indel errors — ~10^5 observations, chance TN calls."""
    import indel_oracle
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import longread_batch
    arr, _ = longread_batch(7, n_reads=40)
    want = native.indel_records_array(indel_oracle.indel_records(arr))
    m = native.HipMasker(0)
    try:
        db = m.upload(arr)
        t = db.indel_tally(arr)
        for mode in (0, 1):     # segmented per-scope sort (default), one global sort
            m.set_param(native.PARAM_INDEL_SORT, mode)
            t.run()
            got = t.download()
            info = t.info()
            assert info["observations"] > 10_000
            assert np.array_equal(got, want), mode
        m.set_param(native.PARAM_INDEL_SORT, 0)
        t.free()
        db.free()
    finally:
        m.close()


def _py_edit(seq: bytes, qual: bytes, rev: bool, edits, times: int):
    """The per-record host loop the writer used before ganon_fastq_edit (indels.apply_leftovers,
    AM:178-203 / 254-270): stored sequence, forward-oriented qualities (Q1), then the record."""
    from genomeanonymizer_amd.indels import apply_leftovers
    s, q = bytearray(seq), list(qual[::-1] if rev else qual)
    for _ in range(times):
        s, q = apply_leftovers(s, q, edits)
    s, q = bytes(s), bytes(q)
    if rev:
        if s.translate(None, b"ACGTN"):
            raise TypeError("Q7")
        s, q = s[::-1].translate(bytes.maketrans(b"ACGTN", b"TGCAN")), q[::-1]
    return s, q


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_native_fastq_edit_matches_host_loop(seed):
    """ganon_fastq_edit (libganon_host.so) against the Python loop on random records and edits,
    including out-of-range positions, DEL alleles of the wrong length, non-ACGTN alleles on
    reverse reads (Q7), empty reads (int(nan)) and the doubled application (Q16)."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.indels import IndelCall
    from genomeanonymizer_amd.variants import VariantType
    rng = np.random.default_rng(seed)
    comp = bytes.maketrans(b"ACGTN", b"TGCAN")
    cases = []
    for i in range(400):
        rev = bool(rng.integers(2))
        L = int(rng.integers(0, 40)) if rng.random() < 0.9 else 0
        alpha = b"ACGTN" if rev else b"=ACMGRSVTWYHKDBN"
        seq = bytes(rng.choice(list(alpha), L).tolist()) if L else b""
        qual = bytes(rng.integers(0, 94, L).tolist())
        edits = []
        for _ in range(int(rng.integers(1, 4))):
            t = VariantType.DEL if rng.random() < 0.5 else VariantType.INS
            n = int(rng.integers(1, 6))
            irp = int(rng.integers(0, L + 5))
            if t is VariantType.DEL:
                k = n if rng.random() < 0.9 else n + 1
                ref = "".join(rng.choice(list("ACGT" if rng.random() < 0.95 else "ACGM"), k).tolist())
            else:
                ref = "A"
            edits.append((irp, IndelCall(irp, irp + 1, t, n, "A", ref)))
        times = int(rng.integers(1, 3))
        try:
            want = _py_edit(seq, qual, rev, edits, times)
        except TypeError:
            want = 1
        except ValueError as e:
            want = 3 if "NaN" in str(e) else 2
        printed = (seq[::-1].translate(comp) if rev else seq)
        name = f"r{i}".encode()
        rec = b"@" + name + b"/1\n" + printed + b"\n+\n" + bytes((b + 33) & 0xFF for b in qual) + b"\n"
        cases.append((rec, rev, edits, times, want))
    # one batch per case keeps the first-error semantics per record; plus one batch of all good ones
    good = [c for c in cases if not isinstance(c[4], int)]
    for batch in [[c] for c in cases] + [good]:
        recs = b"".join(c[0] for c in batch)
        rec_off = np.concatenate([[0], np.cumsum([len(c[0]) for c in batch])])
        ed, al, eo, ao, extra = [], [], [0], [0], 0
        for c in batch:
            for irp, x in c[2]:
                a = x.ref_allele.encode() if x.variant_type is VariantType.DEL else b""
                ed.append((irp, x.variant_type.value, x.length))
                al.append(a)
                ao.append(ao[-1] + len(a))
                extra += c[3] * (len(a) + x.length)
            eo.append(len(ed))
        try:
            data, lens = native.fastq_edit(recs, rec_off, np.array([c[1] for c in batch], np.uint8),
                                           np.array([c[3] for c in batch], np.int32), np.array(eo, np.int64),
                                           np.array(ed, np.int64), b"".join(al), np.array(ao, np.int64),
                                           len(recs) + extra)
        except native.FastqEditError as e:
            assert len(batch) == 1 and batch[0][4] == e.code, (batch[0], e.code)
            continue
        off = np.concatenate([[0], np.cumsum(lens)])
        for j, c in enumerate(batch):
            assert not isinstance(c[4], int), c
            s, q = c[4]
            name = c[0][:c[0].index(b"\n") + 1]
            assert data[off[j]:off[j + 1]] == name + s + b"\n+\n" + bytes((b + 33) & 0xFF for b in q) + b"\n"
