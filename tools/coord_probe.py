#!/usr/bin/env python3
"""Multi-rank readiness evidence on the CPU (verdict r04 item 8, ADVICE r04 stream.py redo rate):
the streamed product in P gloo ranks (the C oracle masking: no GPU) on a chromosome-scale-shaped
pair, reporting rank 0's coordinator busy seconds against the wall, every rank's exchange bytes,
and the job redos that off-contig secondary alignments cause.

    python tools/coord_probe.py OUT.json [RANKS=8] [N_CONTIGS=4] [CONTIG_LEN=8000000] [PAIRS=400000] [SEC_FRAC=0.01]

The input is synth/fastpair.py's (job mode: 4 Mb runs of sections, BAI region reads); SEC_FRAC of
the pairs get a secondary alignment of read 1 on another contig. The one-process run of the same
input (contig mode, GANON_JOB_BP=0) is the files' reference.
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def run(tool, inp, out, env):
    e = {k: v for k, v in os.environ.items() if k != "E2E_WORKERS"}
    e.update(env)
    r = subprocess.run([sys.executable, tool, inp, out, "stream"], env=e, capture_output=True, text=True, timeout=3000)
    if r.returncode:
        raise RuntimeError(r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    a = sys.argv[1:]
    out_json = a[0]
    ranks, nc, cl, pairs, sec = (int(a[1]) if len(a) > 1 else 8, int(a[2]) if len(a) > 2 else 4,
                                 int(a[3]) if len(a) > 3 else 8_000_000, int(a[4]) if len(a) > 4 else 400_000,
                                 float(a[5]) if len(a) > 5 else 0.01)
    from genomeanonymizer_amd.synth.fastpair import make_pair
    d = tempfile.mkdtemp(prefix="ganon_coord_")
    try:
        t = time.time()
        make_pair(os.path.join(d, "in"), n_contigs=nc, contig_len=cl, pairs_per_contig=pairs, sec_frac=sec,
                  window_every=20_000, seed=13)
        gen = time.time() - t
        tool = os.path.join(REPO, "tools", "e2e_bench.py")
        base = {"E2E_ENGINE": "oracle", "E2E_RUNS": "1"}
        multi = run(tool, os.path.join(d, "in"), os.path.join(d, "multi"),
                    dict(base, E2E_WORKERS=str(ranks), E2E_THREADS="1"))
        one = run(tool, os.path.join(d, "in"), os.path.join(d, "one"), dict(base, GANON_JOB_BP="0", E2E_THREADS="8"))
        def rd(p):   # (a sample without single ends writes no single-end file)
            return open(p, "rb").read() if os.path.exists(p) else None
        same = all(rd(os.path.join(d, "multi", f"{x}_stream{s}")) == rd(os.path.join(d, "one", f"{x}_stream{s}"))
                   for x in ("tumor", "normal") for s in (".1.fastq", ".2.fastq", ".single_end.fastq"))
        m = multi["stream"]
        wall = m["stages_s"]["wall_s"]
        res = {"ranks": ranks, "engine": "C oracle (CPU)", "reads": m["reads"], "jobs": m["jobs"],
               "input": f"synth/fastpair.py: {nc} contigs x {cl} bp, {pairs} pairs per contig and sample, "
                        f"{sec:.3f} of the pairs with an off-contig secondary of read 1, BAI-indexed (job mode, "
                        f"GANON_JOB_BP default 4 Mb)",
               "generate_s": round(gen, 1), "wall_s": wall,
               "coordinator_busy_s": m.get("coordinator_busy_s"),
               "coordinator_busy_frac": round((m.get("coordinator_busy_s") or 0) / wall, 4) if wall else None,
               "redos": m.get("redos"), "redos_unchanged": m.get("redos_unchanged"),
               "exchange_bytes_per_rank": [{"sent": r["exchange_sent_bytes"], "recv": r["exchange_recv_bytes"],
                                            "jobs": r["jobs"], "wait_s": round(r["wait_s"], 3),
                                            "wall_s": round(r["wall_s"], 3)} for r in m["per_rank"]],
               "critical_path_s_rank0": m.get("critical_path_s_rank0"),
               # every rank's wall split (stream.py critical_path) and rank 0's tail, part by part
               "critical_path_s_per_rank": [r.get("critical_path") for r in m["per_rank"]],
               "tail_parts_s_per_rank": [r.get("tail_parts") for r in m["per_rank"]],
               "one_process_contig_mode": {"wall_s": one["stream"]["stages_s"]["wall_s"],
                                           "reads_per_s": one["stream"]["reads_per_s"]},
               "files_equal_one_process": same, "host": {"nproc": os.cpu_count()}}
        with open(out_json, "w") as fh:
            json.dump(res, fh, indent=1)
        print(json.dumps(res))
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
