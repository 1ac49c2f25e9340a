"""Host-side logic that is not covered by the golden pipeline runs."""
import os
import random

import numpy as np
import pytest


def test_append_handle_model_matches_cpython(tmp_path):
    """writer.AppendHandle reproduces CPython's buffered text I/O with several append-mode
    handles open on one file (the reference's nested per-scope handles)."""
    from genomeanonymizer_amd.writer import AppendHandle
    rng = random.Random(5)
    for trial in range(20):
        path = str(tmp_path / f"f{trial}.txt")
        open(path, "w").close()
        block = os.stat(str(tmp_path)).st_blksize
        sink = []
        real, model = {}, {}
        recs = []
        for step in range(400):
            op = rng.random()
            if op < 0.08 or not real:
                hid = step
                real[hid] = open(path, "a")
                model[hid] = AppendHandle(sink, block)
            elif op < 0.16 and len(real) > 1:
                hid = rng.choice(list(real))
                real.pop(hid).close()
                model.pop(hid).close()
            else:
                hid = rng.choice(list(real))
                n = rng.choice([40, 300, 330, 333, 2000, 5000, 9000, 17000])
                rec = f"{len(recs):06d}" + "x" * (n - 7) + "\n"
                recs.append(rec)
                real[hid].write(rec)
                model[hid].write(len(recs) - 1, len(rec))
        for hid in list(real):
            real.pop(hid).close()
            model.pop(hid).close()
        got = open(path).read()
        assert got == "".join(recs[i] for i in sink), trial


def test_compare_and_windows():
    from genomeanonymizer_amd.variants import VariantRecord, VariantType, compare
    assert compare(0, 1, 5, 1, 1, 5) == -3 and compare(1, 1, 5, 0, 1, 5) == 3
    assert compare(0, 1, 5, 0, 5, 9) == -1 and compare(0, 1, 5, 0, 6, 9) == -2
    assert compare(0, 5, 9, 0, 1, 5) == 1 and compare(0, 6, 9, 0, 1, 5) == 2
    assert compare(0, 1, 5, 0, 2, 5) == -1 and compare(0, 2, 5, 0, 1, 5) == 1 and compare(0, 1, 5, 0, 1, 5) == 0
    from genomeanonymizer_amd.planner import get_windows
    recs = [VariantRecord("c2", 5000, 5000, 1, "A", "C", VariantType.SNV),
            VariantRecord("c1", 9000, 9003, 3, "ACGT", "A", VariantType.DEL),
            VariantRecord("c1", 3000, 3000, 1, "A", "G", VariantType.SNV)]
    ws = get_windows(recs, {"c1": 0, "c2": 1})
    assert [(w.sequence, w.first, w.last) for w in ws] == [("c1", 2000, 4001), ("c1", 8000, 10004),
                                                          ("c2", 4000, 6001)]
    assert str(ws[0]).startswith("c1,2000,4001,seq_name: c1 pos: 2999 end: 2999 var_type: VariantType.SNV")


def test_sections_and_region_errors(tmp_path):
    """Windows closer than 2003 bp give first > last gaps: the region query raises (Q4)."""
    from genomeanonymizer_amd.synth.bamwriter import write_fasta, write_bam
    from genomeanonymizer_amd.io.fasta import FastaRef
    from genomeanonymizer_amd.io.bam import ReadTable
    from genomeanonymizer_amd.planner import Window, get_genome_sections
    write_fasta(str(tmp_path / "r.fa"), [("a", "ACGT" * 3000), ("b", "ACGT" * 100)])
    fa = FastaRef(str(tmp_path / "r.fa"))
    ws = [Window("a", 2000, 4001, "v"), Window("a", 5000, 7001, "v")]
    secs = get_genome_sections(ws, fa)
    assert [(s.sequence, s.first, s.last) for s in secs] == [
        ("a", 1, 1999), ("a", 2000, 4001), ("a", 4002, 4999), ("a", 5000, 7001), ("a", 7002, 11999), ("b", 0, 0)]
    write_bam(str(tmp_path / "x.bam"), [("a", 12000), ("b", 400)], [])
    t = ReadTable(str(tmp_path / "x.bam"))
    with pytest.raises(ValueError):
        t.fetch("a", 4500, 4400)
    with pytest.raises(ValueError):
        t.fetch("a", -3, 100)
    assert len(t.fetch("a", 0, 100)) == 0


def test_name_output_quirk():
    from genomeanonymizer_amd.short_read_tumor_normal_anonymizer import name_output
    assert name_output("dir/tumor.bam") == "dir/tumor.anonymized"
    assert name_output("xbam/t.cram") == ".anonymized/t.anonymized"   # '.' matches any char


def test_batch_layout_and_validation(hip_built):
    """Batch arrays of the planner satisfy the ABI's validation rules (host-side check
    done through the oracle, which shares the layout)."""
    from genomeanonymizer_amd.synth.batch import random_batch, algorithmic_bytes
    arr = random_batch(4, n_scopes=8)
    L = arr["read_len"].astype(np.int64)
    assert np.all(arr["seq_off"] + (L + 1) // 2 <= len(arr["seq_nt16"]))
    assert arr["scope_incid_off"][-1] == len(arr["incid_read"])
    assert algorithmic_bytes(arr) > 0


def test_config2_batch_small():
    from genomeanonymizer_amd.synth.batch import config2_batch, algorithmic_bytes
    from pyoracle import OracleEngine
    arr, info = config2_batch(n_reads=20000, genome=6_000_000, n_windows=2000, n_germline=6000)
    assert info["reads"] == 20000 and info["window_scopes"] > 1000
    ws = arr["write_scope"]
    # every written read belongs to its write scope
    offs, inc = arr["scope_incid_off"], arr["incid_read"]
    member = set()
    for s in range(len(offs) - 1):
        for r in inc[offs[s]:offs[s + 1]].tolist():
            member.add((r, s))
    assert all((r, int(ws[r])) in member for r in np.nonzero(ws >= 0)[0])
    out, calls, bases, tot = OracleEngine().mask(arr)
    assert tot[2] == 20000
    assert algorithmic_bytes(arr) / info["reads"] > 170


def _plans(paths):
    from genomeanonymizer_amd.io.bam import ReadTable
    from genomeanonymizer_amd.io.fasta import FastaRef
    from genomeanonymizer_amd.io.vcf import read_vcf
    from genomeanonymizer_amd.planner import NativeSamplePlanner, SamplePlanner, get_windows
    fa = FastaRef(paths["ref"])
    ws = get_windows(read_vcf(paths["vcf"]), dict(fa.index))
    out = []
    for cls in (SamplePlanner, NativeSamplePlanner):
        t = (ReadTable(paths["T"]), ReadTable(paths["N"]))
        try:
            out.append(cls(t[0], t[1], fa, ws).run())
        except Exception as e:      # both must fail the same way
            out.append((type(e).__name__,))
    return out


def _same_plan(a, b):
    if isinstance(a, tuple) or isinstance(b, tuple):
        assert a == b
        return
    assert len(a.scopes) == len(b.scopes)
    for x, y in zip(a.scopes, b.scopes):
        assert (x.contig, x.first, x.last, x.span_start, x.span_end, x.is_variant_window, x.keep) == \
               (y.contig, y.first, y.last, y.span_start, y.span_end, y.is_variant_window, y.keep)
        assert np.array_equal(x.t_rows, y.t_rows) and np.array_equal(x.n_rows, y.n_rows)
    norm = lambda log: [tuple(int(v) if not isinstance(v, (str, tuple)) else
                              (tuple(int(u) for u in v) if isinstance(v, tuple) else v) for v in e) for e in log]
    assert norm(a.io_log) == norm(b.io_log)
    assert {d: [tuple(map(int, i)) for i in r] for d, r in a.single_end.items()} == \
           {d: [tuple(map(int, i)) for i in r] for d, r in b.single_end.items()}
    assert a.stats_events == b.stats_events
    assert a.write_single_end == b.write_single_end
    assert a.single_reapply == b.single_reapply


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_native_planner_matches_python_planner(seed, tmp_path):
    """ganon_plan_run (csrc/ganon_plan.cpp) against SamplePlanner on randomized scenarios with
    unmapped/unplaced mates, cross-contig pairs, coverage holes, windows near contig ends."""
    from genomeanonymizer_amd.synth.generate import ContigSpec, ScenarioConfig, generate
    rng = np.random.default_rng(seed)
    contigs = []
    for c in range(3):
        L = int(rng.integers(8_000, 30_000))
        nw = int(rng.integers(0, 5))
        wins = sorted(set(int(x) for x in rng.integers(1001, L - 1200, nw)))
        spaced = []
        for x in wins:                       # the reference needs >= 2003 bp between windows (Q4)
            if not spaced or x - spaced[-1] >= 2003:
                spaced.append(x)
        holes = [("T" if rng.random() < 0.5 else "N", int(h), int(h) + 500) for h in rng.integers(0, L - 600, 2)]
        contigs.append(ContigSpec(f"c{c}", L, int(rng.integers(50, 600)), windows=spaced,
                                  keep_windows=int(rng.integers(0, 2)), holes=holes))
    cfg = ScenarioConfig(name=f"r{seed}", seed=seed, contigs=contigs, germline_snp_per_kb=4.0,
                         germline_indel_per_kb=0.5, softclip_frac=0.05, unmapped_mate_frac=0.05,
                         unplaced_frac=0.4, cross_contig_pairs=10)
    paths = generate(cfg, str(tmp_path / "in"))
    a, b = _plans(paths)
    _same_plan(a, b)


@pytest.mark.parametrize("name", ["tiny", "edge"])
def test_native_planner_matches_python_planner_on_golden_inputs(name, tmp_path):
    from genomeanonymizer_amd.synth.generate import generate, scenario
    a, b = _plans(generate(scenario(name), str(tmp_path / "in")))
    _same_plan(a, b)


def test_native_planner_raises_like_python_planner(tmp_path):
    """Windows 1.5 kb apart: the gap between them has first > last and the region query raises
    ValueError in both planners, as pysam does in the reference."""
    from genomeanonymizer_amd.synth.generate import ContigSpec, ScenarioConfig, generate
    cfg = ScenarioConfig(name="q4", seed=9, contigs=[ContigSpec("c0", 20000, 300, windows=[3000, 4500, 9000]),
                                                     ContigSpec("c1", 5000, 100)])
    a, b = _plans(generate(cfg, str(tmp_path / "in")))
    assert a == b == ("ValueError",)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_native_io_replay_matches_python_model(seed):
    """ganon_io_replay against writer.replay_io (the CPython buffering model checked above) on
    random nested open/write/close logs with record sizes around the 8 KiB chunk and block."""
    from genomeanonymizer_amd import native, writer
    rng = random.Random(seed)
    log, open_h, nxt = [], [], 0
    for _ in range(3000):
        u = rng.random()
        if u < 0.08 or not open_h:
            log.append(("open", nxt))
            open_h.append(nxt)
            nxt += 1
        elif u < 0.14 and len(open_h) > 1:
            h = open_h.pop(rng.randrange(len(open_h)))
            log.append(("close", h))
        else:
            h = rng.choice(open_h)
            ds, sl = rng.randrange(2), rng.randrange(2)
            log.append(("write", h, ds, sl, (ds, len(log), -1)))
    for h in reversed(open_h):
        log.append(("close", h))
    sizes = {i: rng.choice([40, 300, 2000, 5000, 9000]) for i in range(len(log))}
    block = rng.choice([4096, 8192, 65536])
    want = writer.replay_io(log, lambda inst: sizes[inst[1]], block)
    from genomeanonymizer_amd.planner import Plan
    ev, rows = Plan([], log, {0: [], 1: []}, [], False).io_arrays()
    got = native.io_replay(ev, np.array([sizes[i] for i in range(len(log))], np.int64), block)
    for f in range(4):
        assert [i[1] for i in want[(f // 2, f % 2)]] == rows[got[f]].tolist()
