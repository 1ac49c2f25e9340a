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


@pytest.mark.parametrize("name", ["edge", "config1", "fuzz2003", "fuzz3008"])
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
    results = {r: v[0] for r, v in (q.get() for _ in range(2))}   # (totals, redos)
    assert results[0] == results[1]            # totals are all-reduced
    assert results[0]["masked_snv_calls"] > 0
    for tag, pre in (("tumor", name_output(paths["T"])), ("normal", name_output(paths["N"]))):
        for suf in (".1.fastq", ".2.fastq", ".single_end.fastq"):
            gp = os.path.join(GOLDEN, name, f"{tag}{suf}.gz")
            if os.path.exists(gp):
                assert open(pre + suf, "rb").read() == gzip.open(gp).read(), tag + suf
    assert open(paths["N"] + ".statistics.txt").read() == open(os.path.join(GOLDEN, name, "normal.statistics.txt")).read()


def test_cli_rccl_process_group_world_one(tmp_path, hip_built):
    """The CLI as torchrun starts it (RANK / WORLD_SIZE / MASTER_* set) with one rank: the nccl
    (RCCL) process group is created before any GPU call, the sample goes through the sharded
    streamed path (coordinator, Link over the gloo side group) and the int64 totals are all-reduced
    on a CUDA tensor by RCCL (stream._Comm.allreduce_totals). Files equal the reference's."""
    import gzip
    import subprocess
    import sys
    from helpers import GOLDEN, REPO
    from genomeanonymizer_amd.synth.generate import generate, scenario
    d = str(tmp_path / "rccl")
    paths = generate(scenario("fuzz3000"), d)
    env = dict(os.environ, PYTHONPATH=REPO, GANON_IO_BLOCK="4096", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               LOCAL_WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-m", "genomeanonymizer_amd.genome_anonymizer", "-d", d, "-s", "samples.tsv",
                        "-r", paths["ref"], "--record_statistics", "-c", "4", "-v", "2"], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "process group backend nccl" in r.stderr, r.stderr[-2000:]
    for tag in ("tumor", "normal"):
        for suf in (".1.fastq", ".2.fastq", ".single_end.fastq"):
            gp = os.path.join(GOLDEN, "fuzz3000", f"{tag}{suf}.gz")
            assert open(os.path.join(d, f"{tag}.anonymized{suf}"), "rb").read() == gzip.open(gp).read(), tag + suf
    assert open(paths["N"] + ".statistics.txt").read() == \
        open(os.path.join(GOLDEN, "fuzz3000", "normal.statistics.txt")).read()
