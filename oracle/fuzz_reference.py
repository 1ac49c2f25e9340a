#!/usr/bin/env python3
"""Differential check of the product pipeline against the UNMODIFIED reference on random small
samples (TEST INFRASTRUCTURE ONLY, build container only: it imports the reference from
/root/reference at run time exactly as run_reference.py does; nothing derived from the reference
is written into the repository).

For each seed: a random multi-contig tumor/normal pair (germline SNPs and indels, soft clips,
unmapped / unplaced / cross-contig mates, coverage holes, windows), run through
run_short_read_tumor_normal_anonymizer of the reference and through this build's pipeline (the C
oracle standing in for the device, streamed and whole-sample), every output file compared.

usage: python oracle/fuzz_reference.py SEED [SEED ...]
       FUZZ_FASTPAIR=N_CONTIGS,CONTIG_LEN,PAIRS,SEC_FRAC python oracle/fuzz_reference.py SEED ...
       (the sample from synth/fastpair.py instead: the end-to-end bench's input shape, with SEC_FRAC
       of the pairs given an off-contig secondary alignment of read 1; BAMs indexed)
       FUZZ_LONGPAIR=N_CONTIGS,CONTIG_LEN,PAIRS python oracle/fuzz_reference.py SEED ...
       (synth/longpair.py: the long-read end-to-end line's shape — 10-100 kb paired reads with
       soft clips, sequencing and germline indels; BAMs indexed)
"""
from __future__ import annotations

import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, HERE]


def scenario(seed: int):
    """FUZZ_INDEX=1: the BAMs get a .bai (the product's job mode then cuts contigs into runs of
    sections of GANON_JOB_BP bases)."""
    import dataclasses
    from genomeanonymizer_amd.synth.generate import fuzz_scenario
    sc = fuzz_scenario(seed)
    return dataclasses.replace(sc, bam_index=True) if os.environ.get("FUZZ_INDEX") == "1" else sc


def run_ref(paths, work):
    import run_reference as rr
    mod_dir = os.path.join(work, "_mods")
    os.makedirs(mod_dir, exist_ok=True)
    with open(rr.PYX) as fh, open(os.path.join(mod_dir, "pileup_io.py"), "w") as out:
        out.write(rr._detype_pyx(fh.read()))
    for p in (rr.REFERENCE, mod_dir, os.path.join(REPO, "oracle", "stubs")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from src.GenomeAnonymizer.anonymizer_methods import CompleteGermlineAnonymizer
    from src.GenomeAnonymizer.short_read_tumor_normal_anonymizer import run_short_read_tumor_normal_anonymizer
    t_out, n_out = os.path.join(work, "ref_tumor"), os.path.join(work, "ref_normal")
    cwd = os.getcwd()
    os.chdir(work)
    try:
        run_short_read_tumor_normal_anonymizer([paths["vcf"]], [(paths["T"], paths["N"])], paths["ref"],
                                               CompleteGermlineAnonymizer(), [(t_out, n_out)], True, 1, False)
    finally:
        os.chdir(cwd)
    st = paths["N"] + ".statistics.txt"
    shutil.move(st, os.path.join(work, "ref_stats.txt"))
    return t_out, n_out


def files(t_out, n_out, stats):
    out = {}
    for tag, pre in (("tumor", t_out), ("normal", n_out)):
        for suf in (".1.fastq", ".2.fastq", ".single_end.fastq"):
            if os.path.exists(pre + suf):
                out[tag + suf] = open(pre + suf, "rb").read()
    out["stats"] = open(stats, "rb").read()
    return out


def main():
    from genomeanonymizer_amd.synth.generate import generate
    from genomeanonymizer_amd import writer
    writer.io_block_size = lambda d: 4096
    from pyoracle import OracleEngine
    from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
    from genomeanonymizer_amd import short_read_tumor_normal_anonymizer as sr
    bad = 0
    for seed in [int(x) for x in sys.argv[1:]]:
        work = tempfile.mkdtemp(prefix=f"ganon_fuzz_{seed}_")
        fp = os.environ.get("FUZZ_FASTPAIR")
        lp = os.environ.get("FUZZ_LONGPAIR")
        if lp:
            from genomeanonymizer_amd.synth.longpair import make_long_pair
            nc, cl, pp = lp.split(",")
            paths = make_long_pair(os.path.join(work, "in"), n_contigs=int(nc), contig_len=int(cl),
                                   pairs_per_contig=int(pp), seed=seed, window_every=max(5000, int(cl) // 20))
        elif fp:
            from genomeanonymizer_amd.synth.fastpair import make_pair
            nc, cl, pp, sf = fp.split(",")
            paths = make_pair(os.path.join(work, "in"), n_contigs=int(nc), contig_len=int(cl), pairs_per_contig=int(pp),
                              seed=seed, sec_frac=float(sf), window_every=max(5000, int(cl) // 20))
        else:
            paths = generate(scenario(seed), os.path.join(work, "in"))
        try:
            ref = files(*run_ref(paths, work), os.path.join(work, "ref_stats.txt"))
        except Exception as e:   # the reference raising is an outcome the product must match too
            ref = {"error": type(e).__name__}
        res = {}
        for mode in ("0", "1"):
            os.environ["GANON_WHOLE_SAMPLE"] = mode
            t_out, n_out = os.path.join(work, f"p{mode}_tumor"), os.path.join(work, f"p{mode}_normal")
            try:
                sr.run_short_read_tumor_normal_anonymizer([paths["vcf"]], [(paths["T"], paths["N"])], paths["ref"],
                                                          CompleteGermlineAnonymizer(engine=OracleEngine()),
                                                          [(t_out, n_out)], True, 2)
                res[mode] = files(t_out, n_out, paths["N"] + ".statistics.txt")
            except Exception as e:
                res[mode] = {"error": type(e).__name__, "message": str(e)[:200]}
        for mode, got in res.items():
            diff = sorted(k for k in set(ref) | set(got) if k != "message" and ref.get(k) != got.get(k))
            if diff:
                bad += 1
                print(f"seed {seed} mode {'whole' if mode == '1' else 'stream'}: differs in {diff}"
                      + (f" ({got.get('error')}: {got.get('message')} / reference {ref.get('error')})"
                         if 'error' in diff else ""), flush=True)
                for k in diff:
                    if k == "error":
                        continue
                    a, b = ref.get(k, b"").split(b"\n"), got.get(k, b"").split(b"\n")
                    i = next((i for i, (x, y) in enumerate(zip(a, b)) if x != y), min(len(a), len(b)))
                    print(f"   {k}: line {i}: ref {a[i][:90] if i < len(a) else None!r} got {b[i][:90] if i < len(b) else None!r}")
            else:
                print(f"seed {seed} mode {'whole' if mode == '1' else 'stream'}: identical", flush=True)
        shutil.rmtree(work, ignore_errors=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
