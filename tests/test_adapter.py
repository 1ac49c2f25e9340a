"""The reference-protocol adapter (genomeanonymizer_amd/reference_adapter.py):
``GpuCompleteGermlineAnonymizer.anonymize(variant_to_keep, tumor_normal_pileup, ref_genome,
stats_recorder)`` must yield, scope by scope, exactly the pairs the reference's
``CompleteGermlineAnonymizer.anonymize`` (anonymizer_methods.py:431-535) yields — same order, same
FASTQ records — and count the same calls. Expected values: tests/golden/adapter (made by
oracle/make_adapter_golden.py running the reference). The pileups come from the htslib-semantics
stub in oracle/stubs (test infrastructure), merged like pileup_io.iter_pileups (pileup_io.pyx:8-41).
CPU: the C oracle + indel restatement stand in for the device; GPU: libganon_hip.so."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden", "adapter")


def _pysam():
    stubs = os.path.join(REPO, "oracle", "stubs")
    if stubs not in sys.path:
        sys.path.insert(0, stubs)
    import pysam
    return pysam


def iter_pileups(t, n, fasta, contig, start, stop):
    """(tumor column | None, normal column | None) in position order (pileup_io.pyx:8-41)."""
    kw = dict(reference=contig, start=start, end=stop, fastafile=fasta, min_base_quality=0, min_mapping_quality=0,
              max_depth=1000000, stepper="nofilter", ignore_overlaps=False, ignore_orphans=False)
    it1, it2 = t.pileup(**kw), n.pileup(**kw)
    p1, p2 = next(it1, None), next(it2, None)
    while p1 is not None or p2 is not None:
        if p2 is None or (p1 is not None and p1.reference_pos < p2.reference_pos):
            yield p1, None
            p1 = next(it1, None)
        elif p1 is None or p1.reference_pos > p2.reference_pos:
            yield None, p2
            p2 = next(it2, None)
        else:
            yield p1, p2
            p1, p2 = next(it1, None), next(it2, None)


class Counter:
    def __init__(self):
        self.by_type = {}

    def count_variant(self, v):
        self.by_type[v.variant_type.name] = self.by_type.get(v.variant_type.name, 0) + 1


def run_adapter(name, engine):
    from genomeanonymizer_amd.reference_adapter import CalledVariant, GpuCompleteGermlineAnonymizer
    from genomeanonymizer_amd.variants import VariantType
    pysam = _pysam()
    d = os.path.join(GOLD, name)
    scopes = json.load(open(os.path.join(d, "scopes.json")))
    T = pysam.AlignmentFile(os.path.join(d, "t.bam"))
    N = pysam.AlignmentFile(os.path.join(d, "n.bam"))
    fasta = pysam.FastaFile(os.path.join(d, "ref.fa"))
    anon = GpuCompleteGermlineAnonymizer(engine=engine)
    out = []
    for contig, a, b, keep in scopes:
        kv = None if keep is None else CalledVariant(contig, keep[0], keep[0], VariantType.SNV, 1, keep[1], keep[2])
        rec = Counter()
        pairs = [[None if x is None else x.get_anonymized_fastq_record() for x in pair]
                 for pair in anon.anonymize(kv, iter_pileups(T, N, fasta, contig, a, b), fasta, stats_recorder=rec)]
        out.append({"pairs": pairs, "counts": rec.by_type})
    return out


def check(name, got):
    exp = json.load(open(os.path.join(GOLD, name, "expected.json")))
    assert len(got) == len(exp)
    for s, (g, e) in enumerate(zip(got, exp)):
        assert g["counts"] == e["counts"], s
        assert g["pairs"] == e["pairs"], s


@pytest.mark.parametrize("name", ["snv", "indel", "long"])
def test_adapter_matches_reference_with_oracle_engine(name):
    from pyoracle import OracleEngine
    check(name, run_adapter(name, OracleEngine()))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["snv", "indel", "long"])
def test_adapter_matches_reference_on_gpu(name, hip_built):
    from genomeanonymizer_amd import native
    m = native.HipMasker(0)
    try:
        check(name, run_adapter(name, m))
    finally:
        m.close()


def test_stub_pileup_columns_are_live_views():
    """pysam's PileupColumn is a view of the pileup engine's live buffer: the stub raises when a
    column is read after its iterator moved on, so a consumer that stores columns (the pattern the
    adapter snapshots against) fails here instead of reading another column's reads."""
    pysam = _pysam()
    d = os.path.join(GOLD, "snv")
    T = pysam.AlignmentFile(os.path.join(d, "t.bam"))
    contig = T.references[0]
    cols = list(T.pileup(reference=contig, start=0, end=T.lengths[0], stepper="nofilter"))
    assert len(cols) > 2
    with pytest.raises(ValueError):
        cols[0].pileups
