#!/usr/bin/env python3
"""Synthetic tumor/normal pair for tools/e2e_bench.py: one 2 Mb contig with 20,000 pairs per
sample (germline SNPs + indels, soft clips, unmapped and cross-contig mates, a window every
20 kb), tiled into COPIES renamed contigs (synth/tile.py) with .bai indexes.

    python tools/e2e_data.py OUTDIR [COPIES] [SPLIT]   # default 24 copies: ~1.9 M reads in total;
                                                       # SPLIT: chimeric-read fraction (supplementary
                                                       # alignments with SA tags; secondaries at SPLIT/3)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    out = sys.argv[1]
    copies = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    split = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    from genomeanonymizer_amd.synth.generate import ContigSpec, ScenarioConfig, generate
    from genomeanonymizer_amd.synth.tile import tile_sample
    cfg = ScenarioConfig(name="e2e", seed=77,
                         contigs=[ContigSpec("chr", 2_000_000, 20_000, windows=[5000 + 20000 * k for k in range(99)]),
                                  ContigSpec("alt", 200_000, 2_000, windows=[5000, 60000])],
                         germline_snp_per_kb=1.0, germline_indel_per_kb=0.1, hom_fraction=0.2, softclip_frac=0.02,
                         unmapped_mate_frac=0.01, unplaced_frac=0.3, cross_contig_pairs=400,
                         chimeric_frac=split, secondary_frac=split / 3)
    base = generate(cfg, os.path.join(out, "base"))
    tile_sample(base, copies, out)
    print(out)


if __name__ == "__main__":
    main()
