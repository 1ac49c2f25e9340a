#!/usr/bin/env python3
"""Benchmark of the germline-masking hot path on BASELINE.json configs[1].

One step = everything a freshly arrived raw batch needs to be anonymized, starting from its raw
SoA arrays in HBM: ``ganon_batch_replan`` = the device plan of a fresh batch (one scan that
validates every read and scope, writes read ends and segments per read, the scope-group table and
the output-partition candidates; one synchronization for the prep mode and buffer sizes), then
``ganon_batch_run`` = the device prep (CIGAR walk of every (scope, read) incidence into aligned
segments with the incidence checks, output partition pieces, csrc/ganon_prep.hip) + SNV tally ->
TN classification -> overwrite for every scope and the copy of every other read (k_group,
k_finish) + the write-scope check, then the germline indel tally when the scan found I/D ops (none
in the config-2 synthetic reads: no launch). Nothing derived survives from one step to the next
(the 3 GB batch is also far larger than the 256 MB MALL). The batch is the config-2 layout (10 M
synthetic 150 bp tumor+normal reads on a 3.0 Gb genome with 1 M germline SNPs and a 1 M-window
VCF; genomeanonymizer_amd/synth/batch.py) copied to HBM once as raw SoA arrays.
Multi-GPU (torchrun): every rank owns its own config-2 shard (per-contig sharding makes shards
independent; weak scaling) and the only collective is the int64 totals all-reduce over RCCL of
each step, overlapped with the next step's kernels (double-buffered).

Prints one JSON line (rank 0). ``roofline`` is for the whole step (the prep kernels and the
masking kernels, all of which a step needs): the algorithmic bytes of the batch (SURVEY §8(d):
per read ceil(L/2) in + ceil(L/2) out + 4 n_cigar + 16, per extra incidence ceil(L/2) + 4 n_cigar +
8, per scope ceil(span/2) of reference) over the summed average durations of the step's kernels,
each measured with HIP events on the launch stream; ``roofline.dominant`` gives the masking kernel
alone. ``pcie_inclusive``: the same batch re-copied from pinned host memory every step (reload =
H2D + device validation + plan), run, and its masked bases copied back.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
GROUP_MAX_SPAN = 1 << 20                # kGrpMaxSpan: widest scope of the group kernels
PREP_KERNELS = ("prep_scan", "prep_scan_long", "prep_groups", "prep_emit", "prep_pieces")


def kernel_class(name: str) -> str:
    if name == "copy_seq":
        return "copy"
    if name.startswith("k_tile_large") or name.startswith("k_mask_large"):
        return "large"
    if name.startswith("k_group"):
        return "group"
    if name in ("indel_candidates", "k_indel_emit", "indel_sort", "k_indel_classify"):
        return name
    return ""


def indel_bytes(arr, n_obs: int, n_emit: int = None) -> dict:
    """Algorithmic bytes per launch of the indel tally (ganon_indel.hip): the emission reads the
    CIGARs of the incidences whose read has an I/D op and writes a 16-byte observation + 8-byte key
    + 4-byte index per op; the sort reads and writes each (key, index) pair once; the
    classification reads key, index and observation and writes flags, rank and the 8-byte
    registration key of every element; the scan reads the flags and writes 8-byte offsets."""
    ops = arr["cigar"] & 0xF
    has = np.zeros(len(arr["read_len"]), bool)
    rid = np.repeat(np.arange(len(arr["read_len"])), arr["n_cig"].astype(np.int64))
    has[np.unique(rid[(ops == 1) | (ops == 2)])] = True
    r = arr["incid_read"].astype(np.int64)
    cig = int((4 * arr["n_cig"].astype(np.int64)[r])[has[r]].sum())
    n_emit = n_obs if n_emit is None or n_emit < 0 else n_emit
    return {"indel_candidates": 2 * cig, "k_indel_emit": cig + 32 * n_emit, "indel_sort": 24 * n_emit,
            "k_indel_classify": 45 * n_emit}


def kernel_bytes(arr) -> dict:
    """Algorithmic bytes per launch of the masking kernels (SURVEY §8(d) per-unit figures).

    Per read: ceil(L/2) in + ceil(L/2) out + 4*n_cigar + 16; each further scope incidence
    ceil(L/2) + 4*n_cigar + 8; each scope ceil(span/2) of reference. The fused group kernel copies
    every byte of the output it does not leave to the huge-scope kernels (class "large": scopes
    over 2^20 positions, their written reads, incidences and reference). The per-class figures sum
    to the formula."""
    L = arr["read_len"].astype(np.int64)
    h = (L + 1) // 2
    nc = arr["n_cig"].astype(np.int64)
    span = arr["scope_span_len"].astype(np.int64)
    cls = np.where(span <= GROUP_MAX_SPAN, 0, 1)
    out = {"group": 0, "large": 0, "copy": 0}
    ws = arr["write_scope"].astype(np.int64)
    wcls = np.where(ws >= 0, cls[np.maximum(ws, 0)], 0)
    base = 2 * h + 4 * nc + 16
    out["group"] += int(base[wcls == 0].sum())
    out["large"] += int(base[wcls == 1].sum())
    offs = arr["scope_incid_off"]
    scope_of_inc = np.repeat(np.arange(len(span)), np.diff(offs))
    r = arr["incid_read"].astype(np.int64)
    # the first incidence of every read is covered by its base cost
    first = np.zeros(len(r), bool)
    is_ws = scope_of_inc == ws[r]
    order = np.lexsort((~is_ws, r))
    rs = r[order]
    firsts = np.ones(len(rs), bool)
    firsts[1:] = rs[1:] != rs[:-1]
    first[order[firsts]] = True
    extra = ~first
    cost = (h + 4 * nc + 8)[r]
    for k, n in enumerate(("group", "large")):
        out[n] += int(cost[extra & (cls[scope_of_inc] == k)].sum())
        out[n] += int(((span + 1) // 2)[cls == k].sum())
    return out


def cpu_baseline(arr, n_reads: int, budget_s: float = 10.0, threads: int = 0) -> dict:
    """SURVEY §8(d) ref-cpu-N and ref-cpu-1: the C oracle (the reference's per-scope classify +
    mask restated in C) over the same resident batch, on `threads` host threads (scope shards;
    16 = one GPU's CPU share on the box) and on one thread, each for about budget_s / 2."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from pyoracle import OracleEngine
    eng = OracleEngine()
    threads = threads or int(os.environ.get("OMP_NUM_THREADS", "16") or 16)

    def rate(th: int):
        eng.threads = th
        runs, t0 = 0, time.perf_counter()
        while True:
            eng.mask(arr)
            runs += 1
            el = time.perf_counter() - t0
            if el >= budget_s / 2 or runs >= 20:
                return n_reads * runs / el, runs, el

    mt, mt_runs, mt_s = rate(threads)
    st, st_runs, st_s = rate(1)
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": round(mt, 1), "unit": "reads/s", "cores": threads, "kind": "port",
            "host": {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "cpu_model": model,
                     "threads_used": threads, "why": "the GPU box's CPU share per GPU (OMP_NUM_THREADS)"},
            "sample": f"oracle/ganon_oracle.c (C restatement of the reference's per-scope classify+mask) over "
                      f"the whole {n_reads}-read batch: {threads} threads x{mt_runs} ({mt_s:.1f} s); one thread "
                      f"{st:.0f} reads/s x{st_runs} ({st_s:.1f} s); reference Python calibration: 1,196 reads/s "
                      f"(BASELINE.md §2)",
            "single_core_value": round(st, 1)}


CONFIGS = {
    "c2": {"defaults": {"reads": 10_000_000, "genome": 3_000_000_000, "windows": 1_000_000, "germline": 1_000_000},
           "generator": "genomeanonymizer_amd.synth.batch.config2_batch", "seed": 2,
           "workload": "BASELINE configs[1]: {reads}-read 150 bp tumor+normal batch, {germline} germline SNPs, "
                       "{windows}-window VCF, {genome} bp / 24 contigs, resident in HBM"},
    # configs[1] with realistic CIGARs (verdict r04 item 1): germline het deletions 0.1/kb and
    # sequencing indels 1.5e-4/base, so that ~3 % of the reads carry an I/D op and the germline indel
    # tally runs in every step
    "c2id": {"defaults": {"reads": 10_000_000, "genome": 3_000_000_000, "windows": 1_000_000, "germline": 1_000_000},
             "generator": "genomeanonymizer_amd.synth.batch.config2_batch(germline_del_per_kb=0.1, "
                          "seq_indel_per_base=1.5e-4)", "seed": 2,
             "workload": "BASELINE configs[1] with indel CIGARs: {reads}-read 150 bp tumor+normal batch, {germline} "
                         "germline SNPs + germline het deletions 0.1/kb + sequencing indels 1.5e-4/base (~3 % of "
                         "the reads aM dD/I bM), {windows}-window VCF, {genome} bp / 24 contigs, resident in HBM"},
    "c3": {"defaults": {"reads": 40_000_000, "genome": 100_000_000, "windows": 10_000, "germline": 100_000},
           "generator": "genomeanonymizer_amd.synth.batch.config2_batch", "seed": 3,
           "workload": "SURVEY C3 density: {reads} 150 bp reads (~60x tumor+normal) on {genome} bp, "
                       "1 germline het SNP per kb, a window every 10 kb, resident in HBM"},
    # (longread_batch places its own sites: a germline het SNP per kb and a window every 10 kb of
    # `genome`; --windows / --germline do not apply)
    "c5": {"defaults": {"reads": 20_000, "genome": 200_000_000, "windows": 0, "germline": 0},
           "generator": "genomeanonymizer_amd.synth.batch.longread_batch", "seed": 7,
           "workload": "SURVEY C5 shape: {reads} ONT-like reads 10-100 kb (5 % indels, soft clips) on {genome} bp "
                       "with {c5_germline} germline het SNPs (1 per kb; configs[4] names 1 M on 3 Gb) and "
                       "{c5_windows} windows (1 per 10 kb, scopes to ~200 kb), resident in HBM"},
}


def batch_reads(args, k: int) -> int:
    """Reads of pipeline batch k: the configured count -2 % / +-0 / +2 % in turn (mean = the
    configured count over every three batches), so consecutive batches differ in reads, scopes and
    incidences."""
    if args.batches * args.pipeline <= 1:
        return args.reads
    return args.reads + ((k % 3) - 1) * (args.reads // 50)


def make_batch(args, rank: int, k: int = 0):
    """Batch k of this rank: the same sample (genome, germline sites, windows: the config's seed +
    rank) with its own reads (read seed) and read count (batch_reads); c5: its own long-read batch."""
    from genomeanonymizer_amd.synth.batch import config2_batch, longread_batch
    if args.config == "c5":
        return longread_batch(seed=7 + rank + 100 * k, n_reads=args.reads, genome=args.genome)
    seed = CONFIGS[args.config]["seed"] + rank
    rs = 1000 * seed + k
    if args.config == "c3":
        return config2_batch(n_reads=batch_reads(args, k), genome=args.genome, n_contigs=4, n_windows=args.windows,
                             n_germline=args.germline, seed=seed, window_spacing=10_000, read_seed=rs)
    idp = {"germline_del_per_kb": 0.1, "seq_indel_per_base": 1.5e-4} if args.config == "c2id" else {}
    return config2_batch(n_reads=batch_reads(args, k), genome=args.genome, n_windows=args.windows,
                         n_germline=args.germline, seed=seed, read_seed=rs, **idp)


def fastq_bench(masker, db, arr, args, torch, rank: int) -> dict:
    """the FASTQ records of every read of the batch, formatted on the
    device straight from the masked output (ganon_fastq_*, no copy of the bases). Reported
    beside the masking line: formatter ms per run, its roofline, mask + format per step, and
    the host formatter (libganon_host.so, one thread) on a bounded sample."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.fastq import algorithmic_bytes as fq_bytes, fastq_records
    # c2/c3 reads are ACGT only: every read may be reverse (a bad one would fail the download);
    # c5 reads carry IUPAC codes, whose reverse complement is the reference's KeyError (Q7):
    # those reads stay forward
    recs = fastq_records(arr, seed=11 + rank, reverse_frac=0.5, name_len=(30, 45), check_bad=args.config == "c5")
    f = masker.fastq_upload(recs, seq_batch=db)
    for _ in range(args.warmup):
        f.run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        f.run()
    torch.cuda.synchronize()
    fmt_ms = (time.perf_counter() - t) / args.steps * 1e3
    t = time.perf_counter()
    for _ in range(args.steps):
        db.run()
        f.run()
    torch.cuda.synchronize()
    both_ms = (time.perf_counter() - t) / args.steps * 1e3
    masker.set_profiling(True)
    kt: dict = {}
    for _ in range(args.steps):
        f.run()
        f.sync()
        for name, launches, ms in f.kernel_times():
            k = kt.setdefault(name, [0, 0.0])
            k[0] += launches
            k[1] += ms
    masker.set_profiling(False)
    head = f.download()[:64]   # also checks the error slot (no bad record)
    f.free()
    n = len(recs["seq_len"])
    # HBM bytes of the format kernel from the newest PMC summary of this record count taken on these
    # formatter sources (tools/gpu_pmc_fastq.sh -> tools/pmc_step.py ... fastq)
    pmc, pmc_src, pmc_note = pmc_summary("fastq", n, kind="fastq")
    fq_traffic = None
    if pmc is not None:
        fq_traffic = max((v.get("hbm_bytes_per_launch", 0) for k, v in pmc.get("kernels", {}).items()
                          if k.startswith("k_fq_span") or k.startswith("k_fq_quad") or k.startswith("k_fq_format")),
                         default=None)
    alg = fq_bytes(recs)
    fmt_k = kt.get("k_fq_format", [1, float("nan")])
    k_ms = fmt_k[1] / fmt_k[0]
    # bytes the format kernel alone moves per launch: all but the length scan's inputs/outputs
    k_alg = alg - 4 * n
    # host formatter, one thread, bounded sample
    m = min(n, 400_000)
    sample = {k: (v[:m] if isinstance(v, np.ndarray) and len(v) == n else v) for k, v in recs.items()}
    sample["seq_bufs"] = [arr["seq_nt16"]]
    t = time.perf_counter()
    reps = 0
    while True:
        native.host_format_fastq(sample)
        reps += 1
        if time.perf_counter() - t > 3.0:
            break
    host_rps = m * reps / (time.perf_counter() - t)
    return {
        "records": n, "bytes_out": native.fastq_bytes(recs), "ms_per_run": round(fmt_ms, 4),
        "records_per_s": round(n / (fmt_ms * 1e-3), 1), "mask_plus_format_ms_per_step": round(both_ms, 4),
        "mask_plus_format_reads_per_s": round(n / (both_ms * 1e-3), 1),
        "kernels": {k: {"avg_ms": round(v[1] / v[0], 5), "launches": v[0] // args.steps} for k, v in kt.items()},
        "algorithmic_bytes_per_run": alg,
        "roofline": {"bound": "hbm", "kernel": "k_fq_format", "achieved": round(k_alg / (k_ms * 1e-3) / 1e9, 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(k_alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "algorithmic_bytes_per_launch": k_alg, "avg_launch_ms": round(k_ms, 5),
                     "traffic": fq_traffic, "traffic_source": pmc_src, "traffic_note": pmc_note},
        "cpu_host_formatter": {"value": round(host_rps, 1), "unit": "records/s", "cores": 1,
                               "kind": "host C++ (libganon_host.so ganon_fastq_format)",
                               "sample": f"first {m} records, {reps} passes"},
        "head": head.decode(errors="replace"),
    }


def pcie_bench(masker, db, arr, args, torch) -> dict:
    """The batch re-copied from pinned host memory every step: ganon_batch_reload (H2D of the raw
    arrays + device validation and plan, three synchronizations), ganon_batch_run, and the masked
    bases copied back (D2H). The same raw bytes the resident steps start from."""
    from genomeanonymizer_amd import native
    pinned = {}
    for k, v in arr.items():
        if k == "ref_nt16":   # resident on the device (ganon_ref_upload): not re-sent per batch
            continue
        t = torch.empty(v.nbytes, dtype=torch.uint8, pin_memory=True)
        a = t.numpy().view(v.dtype).reshape(v.shape)
        a[...] = v
        pinned[k] = (t, a)
    parr = {k: a for k, (_, a) in pinned.items()}
    out_t = torch.empty(len(arr["seq_nt16"]), dtype=torch.uint8, pin_memory=True)
    out = out_t.numpy()
    n = max(2, min(args.steps, 10))
    for _ in range(2):
        db.reload(parr)
        db.run()
        db.download_seq(out)
    t = time.perf_counter()
    for _ in range(n):
        db.reload(parr)
        db.run()
        db.download_seq(out)
    ms = (time.perf_counter() - t) / n * 1e3
    h2d = int(sum(v.nbytes for k, v in arr.items() if k != "ref_nt16"))
    return {"value": round(len(arr["read_len"]) / (ms * 1e-3), 1), "unit": "reads/s", "ms_per_batch": round(ms, 3),
            "batches": n, "h2d_bytes": h2d, "d2h_bytes": int(len(out)),
            "note": "pinned H2D of every raw read/scope array (the reference stays resident) + device "
                    "validation/plan + run + D2H of the masked bases, per batch"}


def _child_json(cmd, env_extra: dict, timeout: int, drop=()) -> dict:
    """Run a measurement in a child process (its own peak RSS and device context) and parse the
    last JSON line it prints (``drop``: variables of this environment the child must not see)."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra)
    t = time.perf_counter()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        return {"error": f"exit {r.returncode}: {r.stderr[-600:]}"}
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["child_wall_s"] = round(time.perf_counter() - t, 2)
    return out


def e2e_lines(args) -> dict:
    """the product pipeline file to file (BAM decode -> native planner -> HIP
    masking + indel tally -> HIP FASTQ formatting -> FASTQ files; tools/e2e_bench.py, streamed path)
    on a synthetic paired-BAM pair (synth/fastpair.py: 150 bp reads, germline SNPs + deletions,
    window VCF, .bai), and the same pipeline on the CPU (the C oracle masks on the host's cores, the
    host C++ formatter formats) on a bounded sample. Run in child processes before this process
    touches the GPU. The whole-sample path runs once on the same input: its files must equal the
    streamed ones."""
    import shutil
    import tempfile
    from genomeanonymizer_amd.synth.fastpair import make_pair
    d = tempfile.mkdtemp(prefix="ganon_e2e_")
    res = {}
    try:
        t = time.perf_counter()
        inp = os.path.join(d, "in")
        stage("e2e: generating the 24-contig pair")
        make_pair(inp, n_contigs=args.e2e_contigs, pairs_per_contig=args.e2e_pairs)
        gen_s = time.perf_counter() - t
        tool = os.path.join(REPO, "tools", "e2e_bench.py")
        # one process: the streamed and the whole-sample paths (their files must be equal)
        one = _child_json([sys.executable, tool, inp, os.path.join(d, "out"), "stream,whole"],
                          {"E2E_RUNS": str(args.e2e_runs)}, 900)
        # the product's host work over P processes sharing the GPU (the multi-rank path, gloo)
        hip = one
        if args.e2e_workers > 1:
            hip = _child_json([sys.executable, tool, inp, os.path.join(d, "out_w"), "stream"],
                              {"E2E_RUNS": str(args.e2e_runs), "E2E_WORKERS": str(args.e2e_workers)}, 900)
        st = hip.get("stream", {})
        same = None
        if args.e2e_workers > 1 and "error" not in hip and "error" not in one:
            same = all(open(os.path.join(d, "out_w", f"{x}_stream{sfx}"), "rb").read() ==
                       open(os.path.join(d, "out", f"{x}_whole{sfx}"), "rb").read()
                       for x in ("tumor", "normal") for sfx in (".1.fastq", ".2.fastq"))
        elif args.e2e_workers <= 1:
            same = one.get("stream_equals_whole")
        o1 = one.get("stream", {})
        res["e2e"] = {
            "value": st.get("reads_per_s"), "unit": "reads/s", "bases_per_sec": st.get("bases_per_s"),
            "reads": st.get("reads"), "workers": args.e2e_workers, "wall_s": st.get("stages_s", {}).get("wall_s"),
            "wall_s_runs": st.get("wall_s_runs"), "stages_s_rank0": st.get("stages_s"),
            "peak_rss_mb_rank0": st.get("peak_rss_mb"), "output_bytes": st.get("output_bytes"),
            "one_process": {"reads_per_s": o1.get("reads_per_s"), "stages_s": o1.get("stages_s"),
                            "peak_rss_mb": o1.get("peak_rss_mb")},
            "whole_sample": {k: one.get("whole", {}).get(k) for k in ("reads_per_s", "stages_s", "peak_rss_mb")},
            "files_equal_whole_sample": same,
            "workload": f"synth/fastpair.py: {args.e2e_contigs} contigs x 2 Mb, {args.e2e_pairs} pairs per contig "
                        f"and sample (150 bp, FR), 1 germline het SNP/kb + 0.1 het deletion/kb in tumor and normal, "
                        f"a somatic window SNV every 20 kb; streamed product in {args.e2e_workers} processes sharing "
                        f"the GPU (contigs sharded as over ranks, 16 / {args.e2e_workers} decode threads each), "
                        f"files written to local disk",
            "generate_s": round(gen_s, 1), "error": hip.get("error") or one.get("error")}
        # chromosome-scale contigs at configs[2] density (verdict r04 items 2-3): 2 x 20 Mb at 30x per
        # sample (2 M pairs per contig and sample: 16 M reads, scopes ~860 reads deep), the contigs cut
        # into runs of sections (job mode) over the same processes; then the same input in ONE process
        # in contig mode (GANON_JOB_BP=0: one job per contig, an independent plan) — its files must
        # equal the sharded run's
        if args.e2e_chrom_pairs > 0:
            t = time.perf_counter()
            cin = os.path.join(d, "chrom_in")
            stage("e2e: generating the chromosome-scale pair")
            make_pair(cin, n_contigs=2, contig_len=args.e2e_chrom_len, pairs_per_contig=args.e2e_chrom_pairs,
                      window_every=20_000, seed=9)
            cgen = time.perf_counter() - t
            cov = 2 * args.e2e_chrom_pairs * 150 / args.e2e_chrom_len
            stage("e2e: chromosome-scale runs")
            # (a warm run, then two timed runs: the best is the value, both are in wall_s_runs; single runs
            # spread ~2-4 % on one box)
            ch = _child_json([sys.executable, tool, cin, os.path.join(d, "chrom_out"), "stream"],
                             {"E2E_RUNS": "2", "E2E_WORKERS": str(args.e2e_workers), "E2E_DISK_PROBE": "1"}, 900)
            cs = ch.get("stream", {})
            env1 = {"E2E_RUNS": "1", "GANON_JOB_BP": "0"}
            one = _child_json([sys.executable, tool, cin, os.path.join(d, "chrom_one"), "stream"], env1, 900,
                              drop=("E2E_WORKERS",))
            def rd(p):   # (a sample without single ends writes no single-end file)
                return open(p, "rb").read() if os.path.exists(p) else None

            def files_equal(a: str, b: str) -> bool:
                return all(rd(os.path.join(d, a, f"{x}_stream{sfx}")) == rd(os.path.join(d, b, f"{x}_stream{sfx}"))
                           for x in ("tumor", "normal") for sfx in (".1.fastq", ".2.fastq", ".single_end.fastq"))
            same = files_equal("chrom_out", "chrom_one") if "error" not in ch and "error" not in one else None
            # the same input through the CPU pipeline (the C oracle masks on the host's cores, the indel
            # restatement tallies, the host C++ formatter formats; verdict r05 item 1): the GPU run's files
            # must equal it byte for byte — a shared planner or kernel bug of the two HIP runs cannot hide
            orc, same_oracle = {}, None
            if not args.no_e2e_oracle:
                stage("e2e: chromosome-scale oracle leg (CPU)")
                cores = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
                wk = max(1, args.e2e_workers)
                orc = _child_json([sys.executable, tool, cin, os.path.join(d, "chrom_oracle"), "stream"],
                                  {"E2E_ENGINE": "oracle", "E2E_RUNS": "0", "E2E_WORKERS": str(wk),
                                   "E2E_THREADS": str(max(1, cores // wk))}, 1200)
                if "error" not in ch and "error" not in orc:
                    same_oracle = files_equal("chrom_out", "chrom_oracle")
            o1 = one.get("stream", {})
            oo = orc.get("stream", {})
            res["e2e"]["chromosome_scale"] = {
                "value": cs.get("reads_per_s"), "unit": "reads/s", "bases_per_sec": cs.get("bases_per_s"),
                "reads": cs.get("reads"), "workers": args.e2e_workers, "wall_s": cs.get("stages_s", {}).get("wall_s"),
                "wall_s_runs": cs.get("wall_s_runs"), "critical_path_s_rank0": cs.get("critical_path_s_rank0"),
                "stages_s_rank0": cs.get("stages_s"), "peak_rss_mb_rank0": cs.get("peak_rss_mb"),
                "output_bytes": cs.get("output_bytes"), "jobs": cs.get("jobs"), "generate_s": round(cgen, 1),
                "disk": ch.get("disk"),
                "files_equal": same,
                "files_equal_oracle": same_oracle,
                "oracle_leg": {"what": "the same input through the CPU pipeline: the C oracle masking (oracle/ganon_oracle.c), "
                                       "the indel restatement (oracle/indel_oracle.py) and the host C++ formatter, same "
                                       "planner, same processes", "reads_per_s": oo.get("reads_per_s"),
                               "wall_s": oo.get("stages_s", {}).get("wall_s"), "error": orc.get("error"),
                               "skipped": bool(args.no_e2e_oracle)},
                "cpu_us_per_read": round(cs["cpu_s"] / cs["reads"] * 1e6, 3) if cs.get("cpu_s") and cs.get("reads") else None,
                "cores_busy": cs.get("cores_busy"),
                "files_equal_against": {"what": "the same input in one process, contig mode (GANON_JOB_BP=0: one job "
                                                "per contig), E2E_WORKERS unset", "reads_per_s": o1.get("reads_per_s"),
                                        "wall_s": o1.get("stages_s", {}).get("wall_s"),
                                        "peak_rss_mb": o1.get("peak_rss_mb"), "error": one.get("error")},
                "workload": f"synth/fastpair.py: 2 contigs x {args.e2e_chrom_len // 1_000_000} Mb, {args.e2e_chrom_pairs} "
                            f"pairs per contig and sample ({cov:.0f}x per sample, configs[2] density; 150 bp, FR), "
                            f"germline SNPs/deletions as above, a window every 20 kb; contigs cut into runs of sections "
                            f"(job mode: about 6 jobs per process, at most 4 Mb each) read by BAI region queries, "
                            f"sharded over {args.e2e_workers} processes sharing the GPU",
                "error": ch.get("error")}
            shutil.rmtree(cin, ignore_errors=True)
            shutil.rmtree(os.path.join(d, "chrom_out"), ignore_errors=True)
            shutil.rmtree(os.path.join(d, "chrom_one"), ignore_errors=True)
            shutil.rmtree(os.path.join(d, "chrom_oracle"), ignore_errors=True)
        # long reads file to file (BASELINE configs[4] shape, verdict r05 "missing" 4): 10-100 kb paired
        # reads with soft clips and tens to hundreds of CIGAR ops, through the same streamed product,
        # then the same input through the CPU pipeline (the C oracle masking): files must be equal
        if args.e2e_long_pairs > 0:
            from genomeanonymizer_amd.synth.longpair import make_long_pair
            t = time.perf_counter()
            lin = os.path.join(d, "long_in")
            stage("e2e: generating the long-read pair")
            make_long_pair(lin, n_contigs=2, contig_len=10_000_000, pairs_per_contig=args.e2e_long_pairs, seed=11)
            lgen = time.perf_counter() - t
            stage("e2e: long-read runs")
            lh = _child_json([sys.executable, tool, lin, os.path.join(d, "long_out"), "stream"],
                             {"E2E_RUNS": "2", "E2E_WORKERS": str(args.e2e_workers)}, 900)
            lo, same_long = {}, None
            if not args.no_e2e_oracle:
                stage("e2e: long-read oracle leg (CPU)")
                cores = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
                wk = max(1, args.e2e_workers)
                lo = _child_json([sys.executable, tool, lin, os.path.join(d, "long_oracle"), "stream"],
                                 {"E2E_ENGINE": "oracle", "E2E_RUNS": "0", "E2E_WORKERS": str(wk),
                                  "E2E_THREADS": str(max(1, cores // wk))}, 1200)
                if "error" not in lh and "error" not in lo:
                    def rdl(p):
                        return open(p, "rb").read() if os.path.exists(p) else None
                    same_long = all(rdl(os.path.join(d, "long_out", f"{x}_stream{sfx}")) ==
                                    rdl(os.path.join(d, "long_oracle", f"{x}_stream{sfx}"))
                                    for x in ("tumor", "normal") for sfx in (".1.fastq", ".2.fastq", ".single_end.fastq"))
            ls, los = lh.get("stream", {}), lo.get("stream", {})
            res["e2e"]["long_reads"] = {
                "value": ls.get("bases_per_s"), "unit": "bases/s", "reads_per_s": ls.get("reads_per_s"),
                "reads": ls.get("reads"), "bases": ls.get("bases"), "workers": args.e2e_workers,
                "wall_s": ls.get("stages_s", {}).get("wall_s"), "wall_s_runs": ls.get("wall_s_runs"),
                "critical_path_s_rank0": ls.get("critical_path_s_rank0"), "cpu_s": ls.get("cpu_s"),
                "generate_s": round(lgen, 1), "files_equal_oracle": same_long,
                "oracle_leg": {"bases_per_s": los.get("bases_per_s"), "wall_s": los.get("stages_s", {}).get("wall_s"),
                               "error": lo.get("error"), "skipped": bool(args.no_e2e_oracle)},
                "workload": f"synth/longpair.py: 2 contigs x 10 Mb, {args.e2e_long_pairs} pairs per contig and sample "
                            f"(read lengths log-normal around 25 kb in [10, 100] kb, 30 % soft-clipped, 0.5 % "
                            f"substitutions, sequencing indels 5e-4/base + the germline deletions: ~30 CIGAR ops per "
                            f"read, up to ~130), germline SNPs 1/kb + deletions 0.1/kb, a window every 20 kb; streamed "
                            f"product in {args.e2e_workers} processes sharing the GPU (job mode, BAI region reads)",
                "error": lh.get("error")}
            shutil.rmtree(lin, ignore_errors=True)
            shutil.rmtree(os.path.join(d, "long_out"), ignore_errors=True)
            shutil.rmtree(os.path.join(d, "long_oracle"), ignore_errors=True)
        # the CPU path on a bounded sample (the first contigs)
        stage("e2e: the CPU pipeline")
        cpu_in = os.path.join(d, "cpu_in")
        make_pair(cpu_in, n_contigs=args.e2e_cpu_contigs, pairs_per_contig=args.e2e_pairs, seed=8)
        cores = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
        wk = max(1, args.e2e_workers)
        cpu = _child_json([sys.executable, tool, cpu_in, os.path.join(d, "cpu_out"), "stream"],
                          {"E2E_ENGINE": "oracle", "E2E_THREADS": str(max(1, cores // wk)), "E2E_RUNS": "1",
                           "E2E_WORKERS": str(wk)}, 900)
        cs = cpu.get("stream", {})
        res["cpu_e2e"] = {"value": cs.get("reads_per_s"), "unit": "reads/s", "bases_per_sec": cs.get("bases_per_s"),
                          "reads": cs.get("reads"), "cores": cores, "kind": "port", "workers": wk,
                          "stages_s": cs.get("stages_s"), "error": cpu.get("error"),
                          "sample": f"the same pipeline ({wk} processes) with the C oracle masking on {cores} host "
                                    f"threads in all, the "
                                    f"indel restatement (Python) and the host C++ formatter, "
                                    f"{args.e2e_cpu_contigs} contigs of the same shape"}
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return res


# the SURVEY §8(d) shapes timed beside the metric's line (child processes, before this process
# initialises the GPU): configs[1] with indel CIGARs at full size, C3 density at a quarter of its
# size, C5 long reads at half of the reads
SIDE_CONFIGS = {
    "c2id": ["--steps", "20", "--warmup", "5"],
    "c3": ["--reads", "10000000", "--genome", "25000000", "--windows", "2500", "--germline", "25000",
           "--steps", "10", "--warmup", "3"],
    "c5": ["--reads", "10000", "--genome", "100000000", "--steps", "5", "--warmup", "2"],
}


def side_config_lines(args) -> dict:
    """The c3 and c5 lines, each a child bench.py run (the same fresh-batch step and roofline), reduced
    to the fields a reader compares."""
    out = {}
    for name, extra in SIDE_CONFIGS.items():
        stage(f"side config {name} (child bench run)")
        r = _child_json([sys.executable, os.path.abspath(__file__), "--config", name, "--no-e2e", "--no-pcie",
                         "--no-fastq", "--no-cpu-baseline", "--no-side-configs"] + extra, {}, 600)
        if "error" in r:
            out[name] = {"error": r["error"]}
            continue
        out[name] = {k: r.get(k) for k in ("value", "unit", "bases_per_sec", "ms_per_step", "run_only_ms_per_step",
                                           "roofline", "batch_shape", "indel", "child_wall_s")}
        out[name]["workload"] = r.get("config", {}).get("workload")
        out[name]["kernels_ms"] = {k: v.get("avg_ms") for k, v in r.get("pass", {}).get("kernels", {}).items()}
    return out


def summary(r: dict) -> dict:
    """The line's headline figures in a few hundred bytes: the metric's step and its roofline, the
    side configs, the formatter, the device record walk, the end-to-end lines with their parity flags
    and the CPU baseline (every figure also sits, with its details, earlier in the line)."""
    def short(msg):
        return msg[-200:] if isinstance(msg, str) else msg

    def rf(x):
        x = x or {}
        dm = x.get("dominant") or {}
        return {"frac": x.get("frac"), "dominant": dm.get("kernel"), "dominant_frac": dm.get("frac"),
                "traffic": x.get("traffic"), "traffic_source": x.get("traffic_source")}
    out = {"c2": {"value": r.get("value"), "ms_per_step": r.get("ms_per_step"), "roofline": rf(r.get("roofline"))}}
    for k, v in (r.get("side_configs") or {}).items():
        out[k] = {"error": v["error"][:200]} if "error" in v else \
            {"value": v.get("value"), "ms_per_step": v.get("ms_per_step"), "roofline": rf(v.get("roofline"))}
    fq = r.get("fastq") or {}
    if fq:
        fr = fq.get("roofline", {})
        out["fastq"] = {"ms_per_run": fq.get("ms_per_run"), "kernel_ms": fr.get("avg_launch_ms"), "frac": fr.get("frac"),
                        "traffic": fr.get("traffic"), "traffic_source": fr.get("traffic_source")}
    bd = r.get("bam_decode") or {}
    if bd:
        out["bam_decode"] = {"records_per_s": bd.get("value"), "device_ms": bd.get("device_ms"),
                             "columns_equal_host_decoder": bd.get("columns_equal_host_decoder"), "error": short(bd.get("error"))}
    e = r.get("e2e") or {}
    if e:
        out["e2e"] = {"value": e.get("value"), "files_equal_whole_sample": e.get("files_equal_whole_sample"),
                      "error": short(e.get("error"))}
        c = e.get("chromosome_scale") or {}
        if c:
            out["e2e_chromosome_scale"] = {"value": c.get("value"), "reads": c.get("reads"), "wall_s": c.get("wall_s"),
                                           "files_equal": c.get("files_equal"),
                                           "files_equal_oracle": c.get("files_equal_oracle"),
                                           "cpu_us_per_read": c.get("cpu_us_per_read"), "error": short(c.get("error")),
                                           "oracle_error": short((c.get("oracle_leg") or {}).get("error"))}
        lr = e.get("long_reads") or {}
        if lr:
            out["e2e_long_reads"] = {"bases_per_s": lr.get("value"), "reads": lr.get("reads"), "wall_s": lr.get("wall_s"),
                                     "files_equal_oracle": lr.get("files_equal_oracle"), "error": short(lr.get("error")),
                                     "oracle_error": short((lr.get("oracle_leg") or {}).get("error"))}
    cb = r.get("cpu_baseline") or {}
    if cb:
        out["cpu_baseline"] = {"value": cb.get("value"), "cores": cb.get("cores"),
                               "single_core_value": cb.get("single_core_value"),
                               "e2e_value": (cb.get("e2e") or {}).get("value")}
    return out


def pmc_summary(config: str, reads: int, explicit: str = None, kind: str = "mask"):
    """The newest PMC summary under profiles/ of this config and size whose kernel-sources digest
    (genomeanonymizer_amd.build.sources_digest, recorded by tools/pmc_step.py) equals the sources this
    bench runs: PMC bytes of older kernels are not cited. Returns (summary, path, note)."""
    import glob
    from genomeanonymizer_amd.build import sources_digest
    want = sources_digest(kind)
    name = f"pmc_step_{config}.json" if kind == "mask" else f"pmc_{config}.json"
    paths = [explicit] if explicit else sorted(glob.glob(os.path.join(REPO, "profiles", "r*", name)), reverse=True)
    note = f"no PMC summary of {config} at {reads} under profiles/"
    for p in paths:
        try:
            pmc = json.load(open(p))
        except (OSError, ValueError):
            continue
        if pmc.get("config") != config or pmc.get("reads") != reads:
            continue
        rel = os.path.relpath(p, REPO)
        if pmc.get("sources_digest") != want:
            if note.startswith("no PMC"):
                note = (f"{rel} was taken on other kernel sources (digest {pmc.get('sources_digest')}, this build "
                        f"{want}): not cited")
            continue
        return pmc, rel, None
    return None, None, note


_STAGE = ["start", time.time()]


def stage(name: str) -> None:
    """Name the bench's current stage (the heartbeat reports it)."""
    _STAGE[0], _STAGE[1] = name, time.time()
    print(f"[bench] {name}", file=sys.stderr, flush=True)


def _heartbeat(every: float = 30.0) -> None:
    """A line on stderr every `every` seconds while the bench runs (its child runs and data generation
    print nothing for minutes; a runner that takes a silent command for a hung one must not kill it)."""
    import threading

    def beat():
        while True:
            time.sleep(every)
            print(f"[bench] ... {_STAGE[0]} ({time.time() - _STAGE[1]:.0f} s)", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True, name="bench-heartbeat").start()


def main() -> None:
    _heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                    help="c2 = BASELINE configs[1] (the metric's workload); c3 / c5 = SURVEY §8(d) density and "
                         "long-read shapes, for their own lines")
    ap.add_argument("--reads", type=int, default=None)
    ap.add_argument("--genome", type=int, default=None)
    ap.add_argument("--windows", type=int, default=None)
    ap.add_argument("--germline", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--unroll", type=int, default=0,
                    help="group kernel chunk width in 16-base blocks (1/2/4/8; 0 auto: 1 for long reads, else 2)")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive measurement")
    ap.add_argument("--target", type=int, default=None, help="GANON_PARAM_GROUP_TARGET (cost units per group)")
    ap.add_argument("--no-fastq", action="store_true", help="skip the FASTQ formatter measurement")
    ap.add_argument("--indel-sort", type=int, default=0, help="GANON_PARAM_INDEL_SORT: 0 segmented, 1 global")
    ap.add_argument("--fastq-kd", type=int, default=None, help="GANON_PARAM_FASTQ_KD (formatter kernel A/B)")
    ap.add_argument("--pipeline", type=int, default=3,
                    help="contexts stepped round-robin, each with its own HIP stream")
    ap.add_argument("--batches", type=int, default=2,
                    help="resident raw batches per context, stepped in turn: every step plans a batch of other "
                         "read / scope / incidence counts than the context's previous one (c5: 1)")
    ap.add_argument("--spec-plan", type=int, default=1, help="GANON_PARAM_SPEC_PLAN: 1 speculative replans "
                    "(no host synchronization inside the step), 0 the replan waits for the scan")
    ap.add_argument("--prep-unroll", type=int, default=0, help="GANON_PARAM_PREP_UNROLL: incidences per thread "
                    "and trip of the one-segment emit (0 auto, 1, 2, 4)")
    ap.add_argument("--fused-flat", type=int, default=1, help="GANON_PARAM_FUSED_FLAT: 1 the group kernel makes "
                    "the one-segment records from the scan's read descriptors, 0 the record pass")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (BAM -> FASTQ) line")
    ap.add_argument("--indel-tally", type=int, default=1, help="diagnostic: 0 leaves the germline indel tally out of "
                    "the step (the line then says so in step_kind; never the metric's setting)")
    ap.add_argument("--no-side-configs", action="store_true", help="skip the c3 / c5 lines (child runs)")
    ap.add_argument("--no-bam-decode", action="store_true",
                    help="skip the device BAM record walk line (tools/bam_cols_bench.py, a child run)")
    ap.add_argument("--e2e-contigs", type=int, default=24)
    ap.add_argument("--e2e-pairs", type=int, default=23_000, help="pairs per contig and sample")
    ap.add_argument("--e2e-cpu-contigs", type=int, default=4)
    ap.add_argument("--e2e-runs", type=int, default=3,
                    help="timed end-to-end runs after a warm run (the best is the line; all are in wall_s_runs: "
                         "the 709 MB of output writes make single runs spread 0.32-0.58 s on one box)")
    ap.add_argument("--e2e-chrom-pairs", type=int, default=2_000_000,
                    help="pairs per contig and sample of the chromosome-scale end-to-end line (2 contigs of "
                         "--e2e-chrom-len; default 30x per sample, configs[2] density; 0: skip)")
    ap.add_argument("--e2e-chrom-len", type=int, default=20_000_000)
    ap.add_argument("--e2e-long-pairs", type=int, default=1500,
                    help="pairs per contig and sample of the long-read end-to-end line (synth/longpair.py: 2 "
                         "contigs of 10 Mb, 10-100 kb reads; 0: skip)")
    ap.add_argument("--no-e2e-oracle", action="store_true",
                    help="skip the chromosome-scale line's CPU-oracle leg (files_equal_oracle)")
    ap.add_argument("--e2e-workers", type=int, default=8,
                    help="processes sharing the GPU in the end-to-end line (the multi-rank path over gloo)")
    ap.add_argument("--resident", action="store_true",
                    help="round-2 step: run only, the plan made once at upload (not a fresh batch)")
    ap.add_argument("--pmc", default=None,
                    help="PMC step summary (tools/pmc_step.py) for the traffic field; default the newest "
                         "profiles/r*/pmc_step_<config>.json of this size taken on these kernel sources")
    args = ap.parse_args()
    for k, v in CONFIGS[args.config]["defaults"].items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    if args.config == "c5" or args.resident:
        args.batches = 1

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    # end to end first: child processes, before this process initialises the GPU (N = 1 only)
    if world == 1 and not args.no_e2e:
        stage("end-to-end lines (child processes)")
    e2e = e2e_lines(args) if world == 1 and not args.no_e2e else {}
    if world == 1 and args.config == "c2" and not args.no_side_configs:
        stage("side configs (child bench runs)")
    side = side_config_lines(args) if world == 1 and args.config == "c2" and not args.no_side_configs else None
    bam_decode = None
    if world == 1 and args.config == "c2" and not args.no_bam_decode:
        stage("device BAM record walk (child run)")
        bam_decode = _child_json([sys.executable, os.path.join(REPO, "tools", "bam_cols_bench.py")], {}, 600)
    stage(f"{args.config}: generating {args.pipeline * args.batches} batches")
    import torch
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = local % max(1, torch.cuda.device_count())   # == local on a node with a GPU per rank
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # GANON_BENCH_BACKEND=gloo: rehearsal of the N > 1 path on one GPU (host-side reductions)
        backend = os.environ.get("GANON_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)

    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import algorithmic_bytes

    # --pipeline S contexts x --batches B resident raw batches: S * B batches of the same sample with
    # their own reads and read counts (make_batch). Step i runs context i % S on its batch
    # (i // S) % B: every step plans a batch of other counts than that context's previous plan (a
    # new batch arriving), and a context's plan (latency-bound scan and emit) runs beside another
    # context's group kernel (bandwidth-bound)
    n_b = args.pipeline * args.batches
    t_gen = time.perf_counter()
    batches = [make_batch(args, rank, k) for k in range(n_b)]
    t_gen = time.perf_counter() - t_gen
    arr, info = batches[0]
    t_up = time.perf_counter()
    slots = []
    shape = None
    for si in range(args.pipeline):
        m = native.HipMasker(dev)
        for prm, val in ((native.PARAM_GROUP_UNROLL, args.unroll), (native.PARAM_INDEL_SORT, args.indel_sort),
                         (native.PARAM_PREP_UNROLL, args.prep_unroll), (native.PARAM_SPEC_PLAN, args.spec_plan),
                         (native.PARAM_FUSED_FLAT, args.fused_flat)):
            m.set_param(prm, val)
        if args.target:
            m.set_param(native.PARAM_GROUP_TARGET, args.target)
        if args.fastq_kd is not None:
            m.set_param(native.PARAM_FASTQ_KD, args.fastq_kd)
        st = torch.cuda.current_stream() if si == 0 else torch.cuda.Stream()
        m.set_stream(st.cuda_stream)
        mine = [batches[si + args.pipeline * b] for b in range(args.batches)]
        # the genome stays resident (ganon_ref_upload), shared by the context's batches of one sample
        r = m.upload_reference(mine[0][0]["ref_nt16"]) if args.config != "c5" or args.batches == 1 else None
        dbs, inds = [], []
        for a, _ in mine:
            if r is None:
                r = m.upload_reference(a["ref_nt16"])
            d = m.upload({k: v for k, v in a.items() if k != "ref_nt16"}, ref=r)
            sh = d.shape()
            shape = shape or sh
            dbs.append(d)
            # germline indel tally: part of every step when the device scan found I/D ops
            inds.append(d.indel_tally(a) if sh["id_ops"] and args.indel_tally else None)
        slots.append({"m": m, "st": st, "ref": r, "dbs": dbs, "inds": inds, "arrs": [a for a, _ in mine],
                      "reads": [i["reads"] for _, i in mine]})
    masker, stream, db, ind = slots[0]["m"], slots[0]["st"], slots[0]["dbs"][0], slots[0]["inds"][0]
    ref = slots[0]["ref"]
    t_up = time.perf_counter() - t_up

    def pick(i: int):
        sl = slots[i % len(slots)]
        b = (i // len(slots)) % args.batches
        return sl, b
    # totals all-reduce (RCCL) of every step, double-buffered: the reduction of step i runs beside
    # step i + 1's kernels; a buffer is reused only after its previous reduction completed
    tots = [torch.zeros(8, dtype=torch.int64, device="cuda") for _ in range(2)]
    works = [None, None]
    host_reduce = dist is not None and dist.get_backend() != "nccl"

    def step(i: int):
        sl, b = pick(i)
        st_i, db_i, ind_i = sl["st"], sl["dbs"][b], sl["inds"][b]
        if not args.resident:
            db_i.replan()     # a fresh batch: the plan from the raw arrays, every step
        db_i.run()
        if ind_i is not None:
            ind_i.run()
        if dist is not None:
            if host_reduce:
                dist.all_reduce(torch.from_numpy(db_i.totals()))
                return
            b = i & 1
            if works[b] is not None:
                works[b].wait()
            with torch.cuda.stream(st_i):   # (the reduction is ordered after this batch's kernels)
                db_i.copy_totals_to(tots[b].data_ptr())
                works[b] = dist.all_reduce(tots[b], async_op=True)

    def drain():
        for b in range(2):
            if works[b] is not None:
                works[b].wait()
                works[b] = None

    stage("warmup and timed steps")
    for i in range(args.warmup):
        step(i)
    drain()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    gated0 = sum(d.gated_runs() for sl in slots for d in sl["dbs"])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_s = 0.0   # host time inside step(): the launches (a host-bound step shows host_s ~ dt)
    for i in range(args.steps):
        th = time.perf_counter()
        step(i)
        host_s += time.perf_counter() - th
    drain()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    # every timed step really ran: a speculative plan a batch did not fit runs nothing (its download
    # would plan it again), so such a step must not count
    gated = sum(d.gated_runs() for sl in slots for d in sl["dbs"]) - gated0
    if gated:
        raise RuntimeError(f"{gated} timed steps ran nothing (speculative plans their batches did not fit)")
    reads_timed = sum(pick(i)[0]["reads"][pick(i)[1]] for i in range(args.steps))
    dt_t = torch.tensor([dt], dtype=torch.float64, device="cpu" if host_reduce else "cuda")
    if dist is not None:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())

    # the same steps on one context and one stream (its batches in turn, no overlap), for comparison
    one_stream_ms = None
    if len(slots) > 1:
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(args.steps):
            step(i * len(slots))
        drain()
        torch.cuda.synchronize()
        one_stream_ms = (time.perf_counter() - t) / args.steps * 1e3
    # the same pipelined steps with every plan synchronous (GANON_PARAM_SPEC_PLAN 0: the host waits
    # for each scan before it launches the run), for comparison
    sync_ms = None
    if not args.resident and args.spec_plan:
        for sl in slots:
            sl["m"].set_param(native.PARAM_SPEC_PLAN, 0)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(args.steps):
            step(i)
        drain()
        torch.cuda.synchronize()
        sync_ms = (time.perf_counter() - t) / args.steps * 1e3
        for sl in slots:
            sl["m"].set_param(native.PARAM_SPEC_PLAN, args.spec_plan)

    # per-kernel durations: context 0's steps again (its batches in turn) with a HIP event pair
    # around each launch
    masker.set_profiling(True)
    ktimes: dict = {}
    for i in range(args.steps):
        b = i % args.batches
        db_i, ind_i = slots[0]["dbs"][b], slots[0]["inds"][b]
        if not args.resident:
            db_i.replan()
        db_i.run()
        if ind_i is not None:
            ind_i.run()
        db_i.sync()
        for name, launches, ms in db_i.kernel_times():
            k = ktimes.setdefault(name, [0, 0.0])
            k[0] += launches
            k[1] += ms
    masker.set_profiling(False)
    stage("pcie / fastq / cpu baseline")
    pcie = None if args.no_pcie else pcie_bench(masker, db, arr, args, torch)
    fastq = None if args.no_fastq else fastq_bench(masker, db, arr, args, torch, rank)
    # the run-only step of round 2 (plan kept from the previous step), for comparison
    run_only_ms = None
    if not args.resident:
        db.replan()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.steps):
            db.run()
        torch.cuda.synchronize()
        run_only_ms = (time.perf_counter() - t) / args.steps * 1e3
    totals = db.totals()     # (also reports any check the runs made: a bad batch raises here)
    batch_info = db.info()
    if ind is not None:
        irecs = ind.download()
        indel_info = ind.info()
        ind.free()
    else:
        irecs = np.zeros(0, native.INDEL_REC)
        indel_info = {"observations": 0, "emitted": 0, "incidences": 0}
    if dist is not None and host_reduce:
        t_host = torch.from_numpy(totals.copy())
        dist.all_reduce(t_host)
        job_totals = t_host.numpy()
    elif dist is not None:
        db.copy_totals_to(tots[0].data_ptr())
        dist.all_reduce(tots[0])
        torch.cuda.synchronize()
        job_totals = tots[0].cpu().numpy()
    else:
        job_totals = totals
    # every batch's last (speculative) result equals a full synchronous plan + run of it
    per_batch = []
    for sl in slots:
        spec_tots = []
        for rnd in range(2):    # (round 0 leaves every batch planned after another: round 1 is a new-batch plan)
            spec_tots = []
            for d in sl["dbs"]:
                d.replan()
                d.run()
                g0 = d.gated_runs()
                spec_tots.append((d.totals(), g0))
        sl["m"].set_param(native.PARAM_SPEC_PLAN, 0)
        for d, (spec_tot, g0) in zip(sl["dbs"], spec_tots):
            d.replan()
            d.run()
            if not (d.totals() == spec_tot).all():
                raise RuntimeError("a speculative step's totals differ from its batch's full plan")
            per_batch.append({"reads": int(spec_tot[2]), "written": int(spec_tot[3]), "scopes": int(spec_tot[4]),
                              "masked_snv_calls": int(spec_tot[0]), "gated_runs_since_upload": g0})
    for sl in slots:
        for x in sl["inds"]:
            if x is not None and x is not ind:
                x.free()
        for d in sl["dbs"]:
            if d is not db:
                d.free()
        if sl is not slots[0]:
            sl["ref"].free()
            sl["m"].close()
    db.free()
    ref.free()

    # algorithmic bytes of the profiled steps: context 0's batches, one step each in turn
    prof_arrs = slots[0]["arrs"]
    kbs = [kernel_bytes(a) for a in prof_arrs]
    kb = {k: sum(x[k] for x in kbs) // len(kbs) for k in kbs[0]}
    kb.update(indel_bytes(arr, indel_info["observations"], indel_info["emitted"]))
    per_kernel = {n: {"launches": c, "avg_ms": ms / c} for n, (c, ms) in ktimes.items()}
    # the dominant kernel: the longest one the algorithmic bytes are counted for (the group kernel;
    # a prep kernel can take longer on long reads, but it has no byte count of its own)
    counted = [n for n in per_kernel if kb.get(kernel_class(n))] or list(per_kernel)
    dom = max(counted, key=lambda n: per_kernel[n]["avg_ms"] * per_kernel[n]["launches"])
    indel_ms = sum(v["avg_ms"] * v["launches"] for n, v in per_kernel.items() if "indel" in n) / args.steps
    dom_bytes = kb.get(kernel_class(dom), 0)
    dom_ms = per_kernel[dom]["avg_ms"]
    pass_ms = sum(v["avg_ms"] * v["launches"] for v in per_kernel.values()) / args.steps
    alg_total = sum(algorithmic_bytes(a) for a in prof_arrs) // len(prof_arrs)
    achieved = alg_total / (pass_ms * 1e-3) / 1e9
    traffic = dom_traffic = None
    # the newest PMC summary of this config and size taken on these kernel sources (tools/pmc_step.py)
    pmc, pmc_used, pmc_note = pmc_summary(args.config, args.reads, args.pmc)
    if pmc is not None:
        traffic = pmc.get("step_hbm_bytes")
        dom_traffic = pmc.get("kernels", {}).get("k_group", {}).get("hbm_bytes_per_launch")

    reads_total = reads_timed * world
    value = reads_total / dt
    mean_len = float(arr["read_len"].astype(np.int64).mean()) if len(arr["read_len"]) else 0.0
    cfg = CONFIGS[args.config]
    result = {
        "metric": "reads/sec + bases/sec anonymized, 150 bp paired BAM, 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "reads/s",
        "bases_per_sec": round(value * mean_len, 1),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic ({cfg['generator']}, seed {cfg['seed']}+rank)",
        "config": {"workload": cfg["workload"].format(**vars(args), c5_germline=args.genome // 1000,
                                                     c5_windows=args.genome // 10_000), "name": args.config,
                   "reads_per_gpu": info["reads"], "mean_read_len": round(mean_len, 1),
                   "scopes_per_gpu": info["scopes"], "incidences_per_gpu": info.get("incidences"),
                   "window_scopes": info.get("window_scopes"), "union_scopes": info.get("union_scopes"),
                   "passthrough_reads": info.get("passthrough_reads"), "parallelism": f"contig-shard x{world}",
                   "pipeline": args.pipeline},
        "roofline": {"bound": "hbm", "kernel": "step: " + " + ".join(per_kernel), "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic, "traffic_source": pmc_used, "traffic_note": pmc_note,
                     "algorithmic_bytes_per_launch": alg_total,
                     "avg_launch_ms": round(pass_ms, 5),
                     "dominant": {"kernel": dom, "algorithmic_bytes_per_launch": dom_bytes,
                                  "avg_launch_ms": round(dom_ms, 5),
                                  "achieved": round(dom_bytes / (dom_ms * 1e-3) / 1e9, 1),
                                  "traffic": dom_traffic if "k_group" in dom else None,
                                  "frac": round(dom_bytes / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}},
        "step_kind": ("DIAGNOSTIC: the indel tally left out; " if not args.indel_tally else "") +
                     ("resident batch, plan kept (run only)" if args.resident else
                     (f"fresh batch: device plan (replan: validation scan, group table, shape checks) + run every "
                      f"step, over {n_b} resident raw batches of the sample with their own reads ({args.pipeline} "
                      f"contexts on their own HIP streams x {args.batches} batches each, stepped in turn; read counts "
                      f"{sorted(set(batch_reads(args, k) for k in range(n_b)))}): every plan is of other read / scope / "
                      f"incidence counts than its context's previous one; "
                      + ("speculative plan (the run is enqueued behind the scan, buffers sized on the host from the "
                         "batch's counts for the context's last shape; the scan gates the run; gated timed steps: 0)"
                         if args.spec_plan else "the plan waits for the scan"))),
        "batches": per_batch,
        "host_launch_ms_per_step": round(host_s / args.steps * 1e3, 4),
        "sync_plan_ms_per_step": round(sync_ms, 4) if sync_ms else None,
        "run_only_ms_per_step": round(run_only_ms, 4) if run_only_ms else None,
        "one_stream_ms_per_step": round(one_stream_ms, 4) if one_stream_ms else None,
        "batch_shape": shape,
        "pass": {"kernel_ms": round(pass_ms, 4), "algorithmic_bytes": alg_total,
                 "prep_ms": round(sum(v["avg_ms"] * v["launches"] for n, v in per_kernel.items()
                                      if n in PREP_KERNELS) / args.steps, 4),
                 "kernels": {n: {"avg_ms": round(v["avg_ms"], 5), "launches_per_step": v["launches"] // args.steps,
                                 "alg_bytes": kb.get(kernel_class(n))} for n, v in per_kernel.items()}},
        "indel": {"observations": indel_info["observations"], "emitted": indel_info["emitted"],
                  "incidences": indel_info["incidences"],
                  "masked_calls": int((irecs["kind"] == native.INDEL_CALL).sum()),
                  "support_records": int((irecs["kind"] == native.INDEL_SUPPORT).sum()),
                  "ms_per_step": round(indel_ms, 4)},
        "e2e": e2e.get("e2e"),
        "side_configs": side,
        "bam_decode": bam_decode,
        "pcie_inclusive": pcie,
        "fastq": fastq,
        "totals": {k: int(v) for k, v in zip(native.TOTAL_NAMES, job_totals)},
        "batch": batch_info,
        "setup_s": {"generate": round(t_gen, 1), "upload_pcie": round(t_up, 2)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(arr, info["reads"])
        cb = result["cpu_baseline"]
        fmt_rate = (fastq or {}).get("cpu_host_formatter", {}).get("value")
        if fmt_rate:   # ref-cpu-1 with FASTQ formatting: mask then format, one core
            cb["single_core_mask_plus_format"] = round(1.0 / (1.0 / cb["single_core_value"] + 1.0 / fmt_rate), 1)
        cb["e2e"] = e2e.get("cpu_e2e")
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        # last: the compact figures a reader compares (a runner that keeps only the line's tail keeps these)
        result["summary"] = summary(result)
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
