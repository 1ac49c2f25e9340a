"""Deterministic synthetic tumor/normal paired-read scenarios.

Test and benchmark infrastructure. A scenario is a reference FASTA, a tumor BAM, a normal
BAM and a somatic "window" VCF, planted with:

* germline het/hom SNPs and short indels in both samples (the variants that must be masked),
* somatic SNVs in the tumor only at AF 0.4 (these define the windows; never masked),
* 0.1 % substitution errors, base qualities uniform in [2, 40],
* optional edge features: soft clips, placed-unmapped mates, N bases, IUPAC bases on
  forward reads, lower-case reference runs, per-sample coverage holes, and
  VCF records placed on germline sites (the kept-variant rule, anonymizer_methods.py:546-547).

FR pairs with flags 99/147 or 83/163, insert ~ N(300, 30). Read names are disjoint between
tumor and normal. Everything is driven by ``numpy.random.default_rng(seed)``
so the same bytes come out on every machine.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Dict, List, Sequence, Tuple

import numpy as np

from .bamwriter import BamRecord, write_bam, write_fasta, write_vcf

BASES = "ACGT"
COMP = {"A": "T", "C": "G", "G": "C", "T": "A"}


@dataclasses.dataclass
class ContigSpec:
    name: str
    length: int
    pairs: int                      # read pairs per sample
    windows: Sequence[int] = ()     # 1-based positions of somatic SNVs (the window VCF)
    keep_windows: int = 0           # extra VCF records placed on germline SNPs
    holes: Sequence[Tuple[str, int, int]] = ()  # (sample "T"/"N", start, end): no fragments


@dataclasses.dataclass
class ScenarioConfig:
    name: str
    seed: int
    contigs: Sequence[ContigSpec]
    read_len: int = 150
    insert_mean: float = 300.0
    insert_sd: float = 30.0
    germline_snp_per_kb: float = 1.0
    germline_indel_per_kb: float = 0.0
    hom_fraction: float = 0.2
    somatic_af: float = 0.4
    error_rate: float = 0.001
    softclip_frac: float = 0.0
    unmapped_mate_frac: float = 0.0
    n_base_frac: float = 0.0
    iupac_sites: int = 0            # sites where forward T and N reads carry the same IUPAC base
    lowercase_frac: float = 0.0     # fraction of the reference in lower-case runs
    n_ref_runs: int = 0             # runs of 'N' in the reference
    unplaced_frac: float = 0.0      # of the unmapped mates: unplaced (tid -1)
    cross_contig_pairs: int = 0     # per sample: pairs with mates on two different contigs
    bam_index: bool = False         # also write <bam>.bai
    chimeric_frac: float = 0.0      # per mapped 150M read: split into a primary + a hard-clipped supplementary (SA tags)
    secondary_frac: float = 0.0     # per mapped read: an extra secondary alignment (flag 0x100) elsewhere
    secondary_anywhere: bool = False  # secondaries on any contig (else near the mate's contig, BWA-style)
    unmapped_complex_frac: float = 0.0  # of the placed-unmapped mates: flagged secondary / supplementary or SA-tagged
    duplicate_frac: float = 0.0     # per record: written twice (a duplicated record, e.g. a BAM merged twice)


@dataclasses.dataclass
class HapVar:
    kind: str          # "SNP", "INS", "DEL"
    alt: str = ""      # SNP alt base / inserted bases
    dlen: int = 0      # deleted reference bases (after the anchor)


class _ContigModel:
    def __init__(self, cfg: ScenarioConfig, spec: ContigSpec, rng: np.random.Generator):
        self.spec = spec
        L = spec.length
        seq = np.array(list(BASES))[rng.integers(0, 4, L)]
        n_low = int(cfg.lowercase_frac * L / 200)
        self.ref_upper = "".join(seq.tolist())
        chars = list(self.ref_upper)
        for _ in range(n_low):
            s = int(rng.integers(0, max(1, L - 200)))
            e = min(L, s + int(rng.integers(20, 200)))
            for i in range(s, e):
                chars[i] = chars[i].lower()
        for _ in range(cfg.n_ref_runs):
            s = int(rng.integers(0, max(1, L - 50)))
            e = min(L, s + int(rng.integers(5, 50)))
            for i in range(s, e):
                chars[i] = "N"
        self.ref_text = "".join(chars)                 # what goes into the FASTA
        self.ref_up = self.ref_text.upper()            # what reads are drawn from
        # germline variants: haplotype 1 carries every het; hom on both haplotypes
        n_snp = int(round(cfg.germline_snp_per_kb * L / 1000))
        n_ind = int(round(cfg.germline_indel_per_kb * L / 1000))
        taken = set(int(w) - 1 for w in spec.windows)
        self.hap: List[Dict[int, HapVar]] = [dict(), dict()]
        self.germline: List[Tuple[int, HapVar, bool]] = []
        cand = rng.permutation(np.arange(10, L - 20))
        ci = 0

        def next_pos(ok=lambda p: True):
            nonlocal ci
            while ci < len(cand):
                p = int(cand[ci]); ci += 1
                if any(q in taken for q in range(p - 3, p + 8)):
                    continue
                if self.ref_up[p] not in BASES or not ok(p):
                    continue
                for q in range(p - 3, p + 8):
                    taken.add(q)
                return p
            raise RuntimeError("contig too small for the requested variants")

        for _ in range(n_snp):
            p = next_pos()
            alt = BASES[(BASES.index(self.ref_up[p]) + int(rng.integers(1, 4))) % 4]
            hom = bool(rng.random() < cfg.hom_fraction)
            v = HapVar("SNP", alt=alt)
            self.germline.append((p, v, hom))
        for _ in range(n_ind):
            p = next_pos(lambda p: all(c in BASES for c in self.ref_up[p:p + 8]))
            if rng.random() < 0.5:
                v = HapVar("INS", alt="".join(BASES[i] for i in rng.integers(0, 4, int(rng.integers(1, 5)))))
            else:
                v = HapVar("DEL", dlen=int(rng.integers(1, 5)))
            hom = bool(rng.random() < cfg.hom_fraction)
            self.germline.append((p, v, hom))
        self.germline.sort(key=lambda t: t[0])
        for p, v, hom in self.germline:
            self.hap[1][p] = v
            if hom:
                self.hap[0][p] = v
        # somatic SNVs (tumor only) at the window positions
        self.somatic: Dict[int, str] = {}
        for w in spec.windows:
            p = int(w) - 1
            r = self.ref_up[p]
            if r not in BASES:
                continue
            self.somatic[p] = BASES[(BASES.index(r) + int(rng.integers(1, 4))) % 4]
        # VCF records on germline SNPs (kept-variant rule)
        # (window positions must keep the reference's spacing rules, SURVEY Q4:
        #  1-based pos >= 1002, pos <= len - 1003, neighbours >= 2003 apart)
        self.keep_records: List[Tuple[int, str]] = []
        used = [int(w) for w in spec.windows]
        snps = [(p, v) for p, v, _ in self.germline if v.kind == "SNP"]
        for i in rng.permutation(len(snps)):
            if len(self.keep_records) >= spec.keep_windows:
                break
            p, v = snps[int(i)]
            q = p + 1
            if q < 1002 or q > L - 1003 or any(abs(q - u) < 2003 for u in used):
                continue
            used.append(q)
            self.keep_records.append((p, v.alt))
        self.keep_records.sort()

    def fragment(self, start: int, hap: int, flen: int):
        """Walk the haplotype from ref ``start``: returns list of events.

        Event = (kind, refpos, base) with kind 'M' (aligned base), 'I' (inserted base) or
        ('D', refpos, dlen).
        """
        ev = []
        nb = 0
        p = start
        hv = self.hap[hap]
        L = self.spec.length
        while nb < flen and p < L:
            v = hv.get(p)
            b = self.ref_up[p]
            if v is None:
                ev.append(("M", p, b)); nb += 1; p += 1
            elif v.kind == "SNP":
                ev.append(("M", p, v.alt)); nb += 1; p += 1
            elif v.kind == "INS":
                ev.append(("M", p, b)); nb += 1; p += 1
                for c in v.alt:
                    ev.append(("I", -1, c)); nb += 1
            else:
                ev.append(("M", p, b)); nb += 1
                ev.append(("D", p + 1, v.dlen))
                p += 1 + v.dlen
        return ev


def _events_to_read(ev):
    """Trim leading/trailing D events, turn a leading I run into a soft clip."""
    while ev and ev[0][0] == "D":
        ev = ev[1:]
    while ev and ev[-1][0] == "D":
        ev = ev[:-1]
    k = 0
    while k < len(ev) and ev[k][0] == "I":
        k += 1
    ops: List[Tuple[str, int]] = []
    if k:
        ops.append(("S", k))
    seq = [e[2] for e in ev[:k]]
    pos = None
    for e in ev[k:]:
        if e[0] == "D":
            op, n = "D", e[2]
        else:
            op, n = e[0], 1
            seq.append(e[2])
            if op == "M" and pos is None:
                pos = e[1]
        if ops and ops[-1][0] == op:
            ops[-1] = (op, ops[-1][1] + n)
        else:
            ops.append((op, n))
    return pos, ops, seq


def _base_events(ev):
    return [i for i, e in enumerate(ev) if e[0] != "D"]


def _add_split_alignments(recs, cfg, models, rng):
    """BWA-style extra alignments: a mapped all-M read becomes a primary (aligned head, soft-clipped
    tail) plus a supplementary record of its tail elsewhere (hard-clipped head, flag 0x800), each with
    an SA tag naming the other; or it gains a secondary alignment (flag 0x100, full sequence)
    elsewhere. The tail's bases are the read's own (they mismatch their new reference site)."""
    out = []
    names = [m.spec.name for m in models]
    for r in recs:
        if r.flag & 4 or r.tid < 0 or len(r.cigar) != 1 or r.cigar[0][0] != "M":
            out.append(r)
            continue
        L = len(r.seq)
        x = rng.random()
        if x < cfg.chimeric_frac and L > 60:
            k = int(rng.integers(30, L - 30))
            if rng.random() < 0.5:            # near the primary (same scope / section) or anywhere
                ti = r.tid
                lo = max(0, r.pos - 3000)
                spos = int(rng.integers(lo, max(lo + 1, min(models[ti].spec.length - (L - k) - 2, r.pos + 3000))))
            else:
                ti = int(rng.integers(0, len(models)))
                spos = int(rng.integers(0, models[ti].spec.length - (L - k) - 2))
            strand = "-" if r.flag & 16 else "+"
            s_rev = bool(rng.random() < 0.5)      # the tail may align on either strand
            sstrand = "-" if s_rev else "+"
            prim = BamRecord(r.name, r.flag, r.tid, r.pos, r.mapq, [("M", k), ("S", L - k)], r.mate_tid, r.mate_pos,
                             r.tlen, r.seq, r.qual,
                             [("SA", "Z", f"{names[ti]},{spos + 1},{sstrand},{k}H{L - k}M,60,0;")])
            supp = BamRecord(r.name, (r.flag & ~0x12) | 0x800 | (0x10 if s_rev else 0), ti, spos, 60,
                             [("H", k), ("M", L - k)], r.mate_tid, r.mate_pos, 0, r.seq[k:], list(r.qual)[k:],
                             [("SA", "Z", f"{names[r.tid]},{r.pos + 1},{strand},{k}M{L - k}S,{r.mapq},0;")])
            out += [prim, supp]
        elif x < cfg.chimeric_frac + cfg.secondary_frac:
            ti = r.mate_tid if r.mate_tid >= 0 else r.tid    # BWA-style: near the mate's contig
            if cfg.secondary_anywhere:      # e.g. a repeat copy on another chromosome
                ti = int(rng.integers(0, len(models)))
            spos = int(rng.integers(0, models[ti].spec.length - L - 2))
            sec = BamRecord(r.name, r.flag | 0x100, ti, spos, 0, [("M", L)], r.mate_tid, r.mate_pos, 0, r.seq,
                            list(r.qual))
            out += [r, sec]
        else:
            out.append(r)
    return out


def generate(cfg: ScenarioConfig, outdir: str) -> Dict[str, str]:
    """Write ``ref.fa``(+fai), ``tumor.bam``, ``normal.bam``, ``variants.vcf``,
    ``samples.tsv`` and ``truth.json`` into ``outdir``. Returns the paths."""
    os.makedirs(outdir, exist_ok=True)
    rng = np.random.default_rng(cfg.seed)
    models = [_ContigModel(cfg, spec, rng) for spec in cfg.contigs]
    contig_lens = [(s.name, s.length) for s in cfg.contigs]
    write_fasta(os.path.join(outdir, "ref.fa"), [(m.spec.name, m.ref_text) for m in models])
    # IUPAC sites shared by T and N forward reads
    iupac = {}
    for ti, m in enumerate(models):
        for _ in range(cfg.iupac_sites):
            p = int(rng.integers(200, m.spec.length - 200))
            if m.ref_up[p] in BASES:
                iupac[(ti, p)] = "R" if m.ref_up[p] not in "AG" else "Y"
    paths = {}
    for sample, prefix in (("T", "SIM-T"), ("N", "SIM-N")):
        recs: List[BamRecord] = []
        for ti, m in enumerate(models):
            spec = m.spec
            holes = [(a, b) for s, a, b in spec.holes if s == sample]
            made = 0
            attempt = 0
            while made < spec.pairs:
                attempt += 1
                if attempt > spec.pairs * 20:
                    break
                flen = int(round(rng.normal(cfg.insert_mean, cfg.insert_sd)))
                flen = max(flen, cfg.read_len + 10)
                if spec.length - flen - 2 <= 0:
                    break
                start = int(rng.integers(0, spec.length - flen - 2))
                if any(start < b and start + flen + 10 > a for a, b in holes):
                    continue
                hap = int(rng.integers(0, 2))
                ev = m.fragment(start, hap, flen)
                bidx = _base_events(ev)
                if len(bidx) < cfg.read_len + 5:
                    continue
                ev = [list(e) for e in ev]
                # somatic SNVs (tumor, per fragment with AF) and sequencing errors
                carries = sample == "T" and rng.random() < cfg.somatic_af
                for e in ev:
                    if e[0] == "M" and carries and e[1] in m.somatic:
                        e[2] = m.somatic[e[1]]
                for e in ev:
                    if e[0] != "D" and e[2] in BASES and rng.random() < cfg.error_rate:
                        e[2] = BASES[(BASES.index(e[2]) + int(rng.integers(1, 4))) % 4]
                ev = [tuple(e) for e in ev]
                bidx = _base_events(ev)
                left = ev[:bidx[cfg.read_len - 1] + 1]
                right = ev[bidx[-cfg.read_len]:]
                lpos, lops, lseq = _events_to_read(left)
                rpos, rops, rseq = _events_to_read(right)
                if lpos is None or rpos is None:
                    continue
                made += 1
                name = f"{prefix}:{ti}:{made}"
                # soft clips at the outer ends
                if cfg.softclip_frac and rng.random() < cfg.softclip_frac:
                    k = int(rng.integers(1, 21))
                    if lops[0][0] == "M" and lops[0][1] > k + 1:
                        lops = [("S", k), ("M", lops[0][1] - k)] + lops[1:]
                        lseq = [BASES[i] for i in rng.integers(0, 4, k)] + lseq[k:]
                        lpos += k
                if cfg.softclip_frac and rng.random() < cfg.softclip_frac:
                    k = int(rng.integers(1, 21))
                    if rops[-1][0] == "M" and rops[-1][1] > k + 1:
                        rops = rops[:-1] + [("M", rops[-1][1] - k), ("S", k)]
                        rseq = rseq[:-k] + [BASES[i] for i in rng.integers(0, 4, k)]
                lfwd_is_r1 = bool(rng.random() < 0.5)
                unmapped = cfg.unmapped_mate_frac and rng.random() < cfg.unmapped_mate_frac
                for seqlist in (lseq, rseq):
                    if cfg.n_base_frac and rng.random() < cfg.n_base_frac:
                        for _ in range(int(rng.integers(1, 4))):
                            seqlist[int(rng.integers(0, len(seqlist)))] = "N"
                # IUPAC on the forward (left) read only: reverse reads would crash the reference (Q7)
                for (tj, p), code in iupac.items():
                    if tj != ti:
                        continue
                    rp = lpos
                    qi = 0
                    for op, n in lops:
                        if op in "M=X":
                            if rp <= p < rp + n:
                                if rng.random() < 0.5:
                                    lseq[qi + (p - rp)] = code
                                break
                            rp += n; qi += n
                        elif op in "IS":
                            qi += n
                        elif op in "DN":
                            rp += n
                lend = lpos + sum(n for op, n in lops if op in "MDN=X")
                rend = rpos + sum(n for op, n in rops if op in "MDN=X")
                tlen = rend - lpos
                lq = rng.integers(2, 41, len(lseq)).tolist()
                rq = rng.integers(2, 41, len(rseq)).tolist()
                lflag = 1 | 2 | 32 | (64 if lfwd_is_r1 else 128)
                rflag = 1 | 2 | 16 | (128 if lfwd_is_r1 else 64)
                if unmapped:
                    lflag = (lflag & ~2 & ~32) | 8
                    rflag = (rflag & ~2 & ~16) | 4
                    useq = [BASES[i] for i in rng.integers(0, 4, cfg.read_len)]
                    uq = rng.integers(2, 41, cfg.read_len).tolist()
                    if cfg.unplaced_frac and rng.random() < cfg.unplaced_frac:
                        # unplaced unmapped mate (tid -1): never fetched, mate ends single-end (Q9)
                        recs.append(BamRecord(name, lflag, ti, lpos, 60, lops, -1, -1, 0, "".join(lseq), lq))
                        recs.append(BamRecord(name, rflag, -1, -1, 0, [], -1, -1, 0, "".join(useq), uq))
                        continue
                    tags = []
                    if cfg.unmapped_complex_frac and rng.random() < cfg.unmapped_complex_frac:
                        # an unmapped record the reference still turns into an object with
                        # supplementary state (AM:98-108): flagged secondary / supplementary, or an SA tag
                        kind = int(rng.integers(0, 3))
                        if kind == 0:
                            rflag |= 0x100
                        elif kind == 1:
                            rflag |= 0x800
                        else:
                            tags = [("SA", "Z", f"{models[ti].spec.name},{lpos + 1},+,{cfg.read_len}M,0,0;")]
                    recs.append(BamRecord(name, lflag, ti, lpos, 60, lops, ti, lpos, 0, "".join(lseq), lq))
                    recs.append(BamRecord(name, rflag, ti, lpos, 0, [], ti, lpos, 0, "".join(useq), uq, tags))
                else:
                    recs.append(BamRecord(name, lflag, ti, lpos, 60, lops, ti, rpos, tlen, "".join(lseq), lq))
                    recs.append(BamRecord(name, rflag, ti, rpos, 60, rops, ti, lpos, -tlen, "".join(rseq), rq))
        # pairs whose mates map to different contigs (cross-section mate pairing, SR:304-361)
        for k in range(cfg.cross_contig_pairs if len(models) > 1 else 0):
            ti, tj = (int(x) for x in rng.choice(len(models), size=2, replace=False))
            pair = []
            for tk in (ti, tj):
                m = models[tk]
                start = int(rng.integers(0, m.spec.length - cfg.read_len - 20))
                ev = m.fragment(start, int(rng.integers(0, 2)), cfg.read_len)
                pos, ops, seq = _events_to_read(ev)
                pair.append((tk, pos, ops, seq))
            name = f"{prefix}:x:{k}"
            (ta, pa, oa, sa), (tb, pb, ob, sb) = pair
            fa = 1 | 32 | 64
            fb = 1 | 16 | 128
            recs.append(BamRecord(name, fa, ta, pa, 60, oa, tb, pb, 0, "".join(sa),
                                  rng.integers(2, 41, len(sa)).tolist()))
            recs.append(BamRecord(name, fb, tb, pb, 60, ob, ta, pa, 0, "".join(sb),
                                  rng.integers(2, 41, len(sb)).tolist()))
        if cfg.chimeric_frac or cfg.secondary_frac:
            recs = _add_split_alignments(recs, cfg, models, rng)
        if cfg.duplicate_frac:
            recs = [x for r in recs for x in ((r, r) if rng.random() < cfg.duplicate_frac else (r,))]
        recs.sort(key=lambda r: (r.tid if r.tid >= 0 else 1 << 30, r.pos, bool(r.flag & 4), r.name,
                                 r.flag & 0xC0, r.flag & 0x900))
        path = os.path.join(outdir, "tumor.bam" if sample == "T" else "normal.bam")
        write_bam(path, contig_lens, recs, index=cfg.bam_index)
        paths[sample] = path
    # window VCF: somatic SNVs + records on germline SNPs (kept-variant rule)
    vrecs = []
    for m in models:
        for p, alt in m.somatic.items():
            vrecs.append((m.spec.name, p + 1, f"som{len(vrecs)}", m.ref_up[p], alt))
        for p, alt in m.keep_records:
            vrecs.append((m.spec.name, p + 1, f"keep{len(vrecs)}", m.ref_up[p], alt))
    order = {s.name: i for i, s in enumerate(cfg.contigs)}
    vrecs.sort(key=lambda r: (order[r[0]], r[1]))
    write_vcf(os.path.join(outdir, "variants.vcf"), contig_lens, vrecs)
    with open(os.path.join(outdir, "samples.tsv"), "w") as fh:
        fh.write("#tumor\tnormal\tvcf\ntumor.bam\tnormal.bam\tvariants.vcf\n")
    truth = {
        "germline": [[m.spec.name, p, v.kind, v.alt, v.dlen, hom] for m in models for p, v, hom in m.germline],
        "somatic": [[m.spec.name, p, a] for m in models for p, a in m.somatic.items()],
        "iupac": [[models[t].spec.name, p, c] for (t, p), c in iupac.items()],
    }
    with open(os.path.join(outdir, "truth.json"), "w") as fh:
        json.dump(truth, fh)
    paths.update(ref=os.path.join(outdir, "ref.fa"), vcf=os.path.join(outdir, "variants.vcf"),
                 samples=os.path.join(outdir, "samples.tsv"))
    return paths


# ---------------------------------------------------------------------------------------
# Named scenarios used by the golden fixtures and the tests
# ---------------------------------------------------------------------------------------

def fuzz_scenario(seed: int) -> ScenarioConfig:
    """Random small multi-contig pair (oracle/fuzz_reference.py; goldens tests/golden/fuzz<seed>)."""
    rng = np.random.default_rng(seed)
    contigs = []
    if seed >= 9000:
        # long paired reads: 2-8 kb, dense germline indels (long CIGARs), 0.5-2 % substitution errors
        rl = int(rng.integers(2000, 8001))
        for c in range(int(rng.integers(1, 3))):
            L = int(rng.integers(30_000, 60_000))
            wins, x = [], 1500 + int(rng.integers(0, 3000))
            while x < L - 1500 and len(wins) < 4:
                wins.append(x)
                x += 2003 + int(rng.integers(0, 12000))
            contigs.append(ContigSpec(f"c{c}", L, int(rng.integers(8, 24)), windows=wins,
                                      keep_windows=int(rng.integers(0, 2))))
        return ScenarioConfig(name=f"fuzz{seed}", seed=seed, contigs=contigs, read_len=rl,
                              insert_mean=float(2 * rl + rng.integers(500, 4000)), insert_sd=float(rl / 8),
                              germline_snp_per_kb=float(rng.uniform(1, 6)),
                              germline_indel_per_kb=float(rng.uniform(2, 8)), hom_fraction=0.4,
                              error_rate=float(rng.uniform(0.005, 0.02)), softclip_frac=0.2,
                              unmapped_mate_frac=0.05, n_base_frac=0.2, unplaced_frac=0.4,
                              cross_contig_pairs=int(rng.integers(0, 4)))
    for c in range(int(rng.integers(2, 4))):
        L = int(rng.integers(6_000, 14_000))
        wins, x = [], 1001 + int(rng.integers(0, 1500))
        while x < L - 1200 and len(wins) < 4:
            wins.append(x)
            x += 2003 + int(rng.integers(0, 3000))
        contigs.append(ContigSpec(f"c{c}", L, int(rng.integers(60, 260)), windows=wins,
                                  keep_windows=int(rng.integers(0, 2))))
    return ScenarioConfig(name=f"fuzz{seed}", seed=seed, contigs=contigs,
                          germline_snp_per_kb=float(rng.uniform(3, 10)),
                          germline_indel_per_kb=float(rng.uniform(1, 4)), hom_fraction=0.3,
                          softclip_frac=0.05, unmapped_mate_frac=0.05, n_base_frac=0.03,
                          unplaced_frac=0.4, cross_contig_pairs=int(rng.integers(5, 30)),
                          # seeds >= 1000: BWA-style supplementary (SA) and secondary alignments too;
                          # seeds >= 3000: secondaries on any contig (off their mate's contig) and
                          # placed-unmapped mates that are secondary / supplementary / SA-tagged
                          chimeric_frac=0.15 if seed >= 2000 else 0.03 if seed >= 1000 else 0.0,
                          secondary_frac=0.08 if seed >= 2000 else 0.02 if seed >= 1000 else 0.0,
                          secondary_anywhere=seed >= 3000,
                          unmapped_complex_frac=0.4 if seed >= 3000 else 0.0,
                          # seeds >= 3500: duplicated records too
                          duplicate_frac=0.02 if seed >= 3500 else 0.0)


# Golden inputs made by synth/longpair.py instead of a ScenarioConfig (the long-read end-to-end
# line's shape at golden size; always BAI-indexed)
LONGPAIR_GOLDEN = {"longpair": dict(n_contigs=2, contig_len=600_000, pairs_per_contig=12, seed=1,
                                    window_every=30_000)}


def make_inputs(name: str, outdir: str, bam_index: bool = False) -> Dict[str, str]:
    """The inputs of golden scenario ``name``: generate(scenario(name)) (``bam_index``: with .bai
    files), or synth/longpair.py for the names of LONGPAIR_GOLDEN."""
    if name in LONGPAIR_GOLDEN:
        from .longpair import make_long_pair
        return make_long_pair(outdir, **LONGPAIR_GOLDEN[name])
    sc = scenario(name)
    if bam_index:
        import dataclasses
        sc = dataclasses.replace(sc, bam_index=True)
    return generate(sc, outdir)


def scenario(name: str) -> ScenarioConfig:
    if name.startswith("fuzz"):
        return fuzz_scenario(int(name[4:]))
    if name == "config1":
        # BASELINE.json configs[0] / SURVEY §8(d) C1: chr20 1 Mb, 5,000 pairs per sample,
        # 1,000 germline het SNPs, 100 windows at 5,000 + 10,000*i (1-based).
        return ScenarioConfig(
            name="config1", seed=20,
            contigs=[ContigSpec("chr20", 1_000_000, 5000, windows=[5000 + 10000 * i for i in range(100)])],
            germline_snp_per_kb=1.0, hom_fraction=0.0)
    if name == "edge":
        # Small, dense scenario that exercises every quirk the planner must reproduce.
        return ScenarioConfig(
            name="edge", seed=7,
            contigs=[
                ContigSpec("ctgA", 24_000, 1400, windows=[3000, 9000, 15500, 21000], keep_windows=2,
                           holes=[("T", 11_000, 11_600), ("N", 18_000, 18_400)]),
                ContigSpec("ctgB", 12_000, 400, windows=[]),
                ContigSpec("ctgC", 16_000, 120, windows=[4000, 11000]),
            ],
            germline_snp_per_kb=6.0, germline_indel_per_kb=1.0, hom_fraction=0.3,
            softclip_frac=0.05, unmapped_mate_frac=0.02, n_base_frac=0.05, iupac_sites=2,
            lowercase_frac=0.05, n_ref_runs=2, unplaced_frac=0.3, cross_contig_pairs=25)
    if name == "long1":
        # Long paired reads (SURVEY §8(d) C5 in miniature, pinned file to file by the reference run):
        # 4-6 kb reads, 12 kb fragments, dense germline indels (hap-1 reads carry 20-40 I/D ops, many
        # over the 48-op threshold of the device's long-CIGAR walk), 1 % substitution errors, soft clips.
        return ScenarioConfig(
            name="long1", seed=41,
            contigs=[ContigSpec("lr1", 60_000, 24, windows=[6000, 20000, 41000], keep_windows=1),
                     ContigSpec("lr2", 40_000, 14, windows=[15000])],
            read_len=5000, insert_mean=12_000.0, insert_sd=1500.0,
            germline_snp_per_kb=3.0, germline_indel_per_kb=6.0, hom_fraction=0.5,
            error_rate=0.01, softclip_frac=0.2, n_base_frac=0.2, unmapped_mate_frac=0.05,
            unplaced_frac=0.3, cross_contig_pairs=3)
    if name == "long2":
        # configs[4]-length reads file to file: 15 kb paired reads (ONT-like 2 % substitutions, dense
        # germline indels: ~100-200 CIGAR ops per read), 34 kb fragments
        return ScenarioConfig(
            name="long2", seed=43,
            contigs=[ContigSpec("ont1", 150_000, 10, windows=[20000, 70000, 120000], keep_windows=1),
                     ContigSpec("ont2", 90_000, 5, windows=[45000])],
            read_len=15_000, insert_mean=34_000.0, insert_sd=3000.0,
            germline_snp_per_kb=2.0, germline_indel_per_kb=5.0, hom_fraction=0.5,
            error_rate=0.02, softclip_frac=0.3, n_base_frac=0.3, unmapped_mate_frac=0.05,
            unplaced_frac=0.5, cross_contig_pairs=2)
    if name == "tiny":
        return ScenarioConfig(
            name="tiny", seed=3,
            contigs=[ContigSpec("t1", 6_000, 150, windows=[2500], keep_windows=1),
                     ContigSpec("t2", 3_000, 40, windows=[])],
            germline_snp_per_kb=8.0, germline_indel_per_kb=1.5, hom_fraction=0.3,
            softclip_frac=0.1, unmapped_mate_frac=0.05, n_base_frac=0.05, iupac_sites=1,
            unplaced_frac=0.5, cross_contig_pairs=6)
    raise KeyError(name)
