"""Shared test helpers: golden-fixture runs of the full pipeline."""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import shutil

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")


def input_digests(paths) -> dict:
    d = {}
    for key in ("ref", "vcf"):
        with open(paths[key], "rb") as fh:
            d[key] = hashlib.sha256(fh.read()).hexdigest()
    for key in ("T", "N"):
        with gzip.open(paths[key], "rb") as fh:
            d[key] = hashlib.sha256(fh.read()).hexdigest()
    return d


def run_pipeline_vs_golden(name: str, workdir: str, anonymizer, block_size: int = 4096, bam_index: bool = False):
    """Regenerate the scenario's inputs, run the product pipeline, compare every output
    file with the reference's. Returns a dict of mismatches (empty = byte-identical).
    ``bam_index``: write .bai files too (the streamed path's job mode reads regions through them)."""
    from genomeanonymizer_amd.synth.generate import make_inputs
    from genomeanonymizer_amd import short_read_tumor_normal_anonymizer as sr
    from genomeanonymizer_amd import writer
    meta = json.load(open(os.path.join(GOLDEN, name, "meta.json")))
    shutil.rmtree(workdir, ignore_errors=True)
    paths = make_inputs(name, os.path.join(workdir, "in"), bam_index)
    assert input_digests(paths) == meta["inputs_sha256"], "synthetic generator drifted from the fixtures"
    t_out, n_out = sr.name_output(paths["T"]), sr.name_output(paths["N"])
    orig = writer.io_block_size
    writer.io_block_size = lambda d: block_size   # the block size the fixtures were written with
    try:
        sr.run_short_read_tumor_normal_anonymizer([paths["vcf"]], [(paths["T"], paths["N"])], paths["ref"],
                                                  anonymizer, [(t_out, n_out)], True, 4)
    finally:
        writer.io_block_size = orig
    bad = {}
    for tag, pre in (("tumor", t_out), ("normal", n_out)):
        for suf in (".1.fastq", ".2.fastq", ".single_end.fastq"):
            gp = os.path.join(GOLDEN, name, f"{tag}{suf}.gz")
            mine = pre + suf
            if not os.path.exists(gp):
                if os.path.exists(mine):
                    bad[tag + suf] = "unexpected file"
                continue
            exp = gzip.open(gp).read()
            got = open(mine, "rb").read() if os.path.exists(mine) else b""
            if exp != got:
                el, gl = exp.split(b"\n"), got.split(b"\n")
                first = next((i for i, (a, b) in enumerate(zip(el, gl)) if a != b), min(len(el), len(gl)))
                bad[tag + suf] = f"line {first}: expected {el[first][:80] if first < len(el) else None!r} " \
                                 f"got {gl[first][:80] if first < len(gl) else None!r}"
    exp = open(os.path.join(GOLDEN, name, "normal.statistics.txt")).read()
    got = open(paths["N"] + ".statistics.txt").read()
    if exp != got:
        bad["statistics"] = "differs"
    return bad


def load_scope_golden(seed: int):
    z = np.load(os.path.join(GOLDEN, "scopes", f"random_{seed}.npz"))
    arr = {k: z[k] for k in z.files if not k.startswith("expected")}
    return arr, z["expected_seq"], z["expected_calls"]


def written_reads_equal(arr, out, expected):
    """Indices of written reads whose packed bytes differ."""
    ws = arr["write_scope"]
    L = (arr["read_len"].astype(np.int64) + 1) // 2
    bad = []
    for r in np.nonzero(ws >= 0)[0]:
        a, n = int(arr["seq_off"][r]), int(L[r])
        if not np.array_equal(out[a:a + n], expected[a:a + n]):
            bad.append(int(r))
    return bad
