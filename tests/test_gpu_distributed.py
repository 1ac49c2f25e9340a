"""The N > 1 path on the GPU: two ranks (spawned processes, gloo for the totals all-reduce), both
masking their contig shards with the HIP engine on the one GPU of the box (HipMasker, not the
oracle), must write exactly the reference's files (tests/golden). Matches SURVEY §8(e):
per-contig shards, no data-path collective (short_read_tumor_normal_anonymizer.py:944-961 runs
pairs in parallel; the contigs of one pair shard here)."""
import os

import pytest
import torch.multiprocessing as mp

from test_distributed import _free_port, _worker

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["edge", "config1", "fuzz2003"])
def test_two_rank_hip_contig_shards_match_reference(name, tmp_path, hip_built):
    import gzip
    from helpers import GOLDEN
    from genomeanonymizer_amd.short_read_tumor_normal_anonymizer import name_output
    from genomeanonymizer_amd.synth.generate import generate, scenario
    workdir = str(tmp_path / name)
    paths = generate(scenario(name), os.path.join(workdir, "in"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, workdir, q, "hip")) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0, 0], codes
    results = dict(q.get() for _ in range(2))
    assert results[0] == results[1]            # totals are all-reduced
    assert results[0]["masked_snv_calls"] > 0
    for tag, pre in (("tumor", name_output(paths["T"])), ("normal", name_output(paths["N"]))):
        for suf in (".1.fastq", ".2.fastq", ".single_end.fastq"):
            gp = os.path.join(GOLDEN, name, f"{tag}{suf}.gz")
            if os.path.exists(gp):
                assert open(pre + suf, "rb").read() == gzip.open(gp).read(), tag + suf
    assert open(paths["N"] + ".statistics.txt").read() == open(os.path.join(GOLDEN, name, "normal.statistics.txt")).read()
