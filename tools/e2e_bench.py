#!/usr/bin/env python3
"""End-to-end timing of the product pipeline on one tumor/normal pair (BAM decode -> native
planner -> GPU masking + indel tally -> GPU FASTQ formatting -> files), the path a user of the
CLI runs. Prints one JSON line with per-stage seconds and reads/s.

    python tools/e2e_bench.py DIR   # DIR holds tumor.bam normal.bam ref.fa variants.vcf
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out", "e2e")
    os.makedirs(out, exist_ok=True)
    from genomeanonymizer_amd import short_read_tumor_normal_anonymizer as sr
    from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
    from genomeanonymizer_amd.io.fasta import FastaRef
    from genomeanonymizer_amd.io.vcf import read_vcf
    from genomeanonymizer_amd.planner import get_windows
    t0 = time.time()
    fasta = FastaRef(os.path.join(d, "ref.fa"))
    windows = get_windows(read_vcf(os.path.join(d, "variants.vcf")), dict(fasta.index))
    t_win = time.time() - t0
    anon = CompleteGermlineAnonymizer(device=0)
    anon.engine   # context creation outside the timed stages
    runs = []
    for _ in range(2):    # the first run pays one-time costs (module loads, device init)
        tim = sr.anonymize_genome(windows, os.path.join(d, "tumor.bam"), os.path.join(d, "normal.bam"),
                                  os.path.join(d, "ref.fa"), anon, os.path.join(out, "tumor"),
                                  os.path.join(out, "normal"), True, 16, fasta=fasta)
        runs.append(tim)
    tim = runs[-1]
    total = tim["decode_s"] + tim["plan_s"] + tim["mask_s"] + tim["write_s"]
    print(json.dumps({"reads": tim["reads"], "scopes": tim["scopes"], "windows_s": round(t_win, 3),
                      "stages_s": {k: round(v, 3) for k, v in tim.items() if k.endswith("_s")},
                      "total_s": round(total, 3), "reads_per_s": round(tim["reads"] / total, 1),
                      "first_run_total_s": round(sum(v for k, v in runs[0].items() if k.endswith("_s")), 3)}))


if __name__ == "__main__":
    main()
