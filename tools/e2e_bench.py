#!/usr/bin/env python3
"""End-to-end timing of the product pipeline on one tumor/normal pair (BAM decode -> native
planner -> GPU masking + indel tally -> GPU FASTQ formatting -> files), the path a user of the
CLI runs: the streamed path (per contig, bounded memory; the default) and the whole-sample path.
Prints one JSON line with per-stage seconds, reads/s, bases/s and the process's peak RSS per mode.

    python tools/e2e_bench.py DIR [OUTDIR] [stream,whole]   # DIR: tumor.bam normal.bam ref.fa variants.vcf
                                                             # (tools/e2e_data.py, synth/fastpair.py)
    E2E_ENGINE=oracle ...    # the CPU path: the C oracle (E2E_THREADS threads) masks, the host C++
                             # formatter formats (bench.py's CPU end-to-end baseline; test infrastructure)
    E2E_RUNS=N ...           # timed runs per mode after one untimed warm run (default 1; 0: one run only)
    E2E_PROFILE=PREFIX ...   # cProfile of the timed run of each mode -> PREFIX_<mode>.txt (main thread)
    E2E_SAMPLE=PREFIX ...    # CPU attribution of the last timed run, every thread (tools/cpu_sampler.py)
                             # -> PREFIX_<mode>_r<rank>.json
    GANON_PREFETCH=N ...     # look-ahead planning threads of the streamed path (0: in line)
    E2E_DECODE_THREADS=T ... # host decode threads per process (default 16 / E2E_WORKERS)
    E2E_WORKERS=P ...        # the streamed path in P processes sharing the GPU (torch.distributed.run,
                             # gloo; the contigs sharded over them as over the ranks of a multi-GPU run,
                             # host decode threads 16 / P each); wall = the slowest rank's
    E2E_DISK_PROBE=1 ...     # also time 2 GiB of pwrite into OUTDIR (4 files at once, as the product
                             # writes; page cache, then with fsync): the box's write bandwidth
"""
import json
import os
import resource
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _engine():
    from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
    if os.environ.get("E2E_ENGINE", "hip") == "oracle":
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        from pyoracle import OracleEngine
        from genomeanonymizer_amd import native

        class CpuEngine(OracleEngine):
            """The C oracle's masking + the host C++ formatter (libganon_host.so)."""

            def format_fastq(self, recs):
                return native.host_format_fastq(recs)
        eng = CpuEngine()
        eng.threads = int(os.environ.get("E2E_THREADS", "16"))
        return CompleteGermlineAnonymizer(engine=eng)
    anon = CompleteGermlineAnonymizer(device=int(os.environ.get("GANON_DEVICE", "0")))
    anon.engine   # context creation outside the timed stages
    return anon


def disk_probe(out: str, total: int = 2 << 30) -> dict:
    """Write bandwidth of OUTDIR's file system as the product sees it: four files written at once in
    16 MiB pwrites (the page cache: what an un-synced run's wall pays), then the same with an fsync
    of each file (the device)."""
    from concurrent.futures import ThreadPoolExecutor
    buf = os.urandom(16 << 20)
    res = {}
    for sync in (False, True):
        paths = [os.path.join(out, f"_probe{k}") for k in range(4)]
        fds = [os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644) for p in paths]

        def one(fd):
            for o in range(0, total // 4, len(buf)):
                os.pwrite(fd, buf, o)
            if sync:
                os.fsync(fd)
        t = time.time()
        with ThreadPoolExecutor(4) as ex:
            list(ex.map(one, fds))
        dt = time.time() - t
        for fd, p in zip(fds, paths):
            os.close(fd)
            os.unlink(p)
        res["fsync_gb_per_s" if sync else "page_cache_gb_per_s"] = round(total / dt / 1e9, 2)
    res["bytes"] = total
    res["dir"] = out
    return res


def _relaunch(workers: int) -> None:
    """This script again under torch.distributed.run with ``workers`` ranks (a child process: this
    one has not touched the GPU); exits with its code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={workers}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def main():
    workers = int(os.environ.get("E2E_WORKERS", "1"))
    if workers > 1 and "RANK" not in os.environ:
        _relaunch(workers)
    dist = None
    rank = 0
    if workers > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        rank = dist.get_rank()
        os.environ.setdefault("GANON_DEVICE", str(int(os.environ.get("LOCAL_RANK", 0)) % max(1, torch.cuda.device_count())))
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out", "e2e")
    os.makedirs(out, exist_ok=True)
    from genomeanonymizer_amd import short_read_tumor_normal_anonymizer as sr
    from genomeanonymizer_amd.io.fasta import FastaRef
    from genomeanonymizer_amd.io.vcf import read_vcf
    from genomeanonymizer_amd.planner import get_windows
    t0 = time.time()
    fasta = FastaRef(os.path.join(d, "ref.fa"))
    windows = get_windows(read_vcf(os.path.join(d, "variants.vcf")), dict(fasta.index))
    t_win = time.time() - t0
    anon = _engine()
    res = {"windows_s": round(t_win, 3), "engine": os.environ.get("E2E_ENGINE", "hip")}
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["stream", "whole"]
    if dist is not None and modes != ["stream"]:
        sys.exit("E2E_WORKERS > 1 runs the streamed path only")
    threads = int(os.environ.get("E2E_DECODE_THREADS", "0")) or max(1, 16 // workers)
    n_timed = int(os.environ.get("E2E_RUNS", "1"))
    for mode in modes:
        runs = []
        for it in range(1 + n_timed):    # the first run pays one-time costs (module loads, device init)
            prof = None
            if it == n_timed and os.environ.get("E2E_PROFILE"):   # cProfile of the last timed run
                import cProfile
                prof = cProfile.Profile()
                prof.enable()
            # a run writes new files: the previous run's outputs go first (truncating 0.7 GB of
            # files inside the timed region cost ~75 ms)
            if rank == 0:
                for x in ("tumor", "normal"):
                    for sfx in (".1.fastq", ".2.fastq", ".single_end.fastq"):
                        try:
                            os.unlink(os.path.join(out, f"{x}_{mode}{sfx}"))
                        except FileNotFoundError:
                            pass
            if dist is not None:
                dist.barrier()
            sampler = None
            if it == n_timed and os.environ.get("E2E_SAMPLE"):   # CPU attribution of the last timed run
                sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
                from cpu_sampler import Sampler
                sampler = Sampler().__enter__()
            from genomeanonymizer_amd import native as _nat
            _nat.decode_phase_times(reset=True)
            pin0 = _nat.pinned_stats()
            t1, c1 = time.time(), os.times()
            tim = sr.anonymize_genome(windows, os.path.join(d, "tumor.bam"), os.path.join(d, "normal.bam"),
                                      os.path.join(d, "ref.fa"), anon, os.path.join(out, f"tumor_{mode}"),
                                      os.path.join(out, f"normal_{mode}"), True, threads, fasta=fasta,
                                      streaming=(mode == "stream"), dist=dist)
            tim["wall_s"] = time.time() - t1
            tim["decode_phases"] = _nat.decode_phase_times()
            pin1 = _nat.pinned_stats()
            tim["pinned"] = {k: round(pin1[k] - pin0.get(k, 0), 4) for k in pin1}
            if sampler is not None:
                sampler.__exit__(None, None, None)
                sampler.report(f"{os.environ['E2E_SAMPLE']}_{mode}_r{rank}.json")
            c2 = os.times()   # this process's CPU time over the run (all its threads)
            tim["cpu_s"] = (c2.user - c1.user) + (c2.system - c1.system)
            if dist is not None:   # every rank's exchange and waits, then the slowest rank's wall
                per_rank = [None] * dist.get_world_size()
                dist.all_gather_object(per_rank, {k: tim.get(k) for k in (
                    "wall_s", "exchange_sent_bytes", "exchange_recv_bytes", "wait_s", "writer_wait_s", "jobs",
                    "decode_s", "mask_s", "format_s", "write_s", "redos_skipped", "critical_path", "cpu_s", "fastq_device",
                    "setup_s", "groups_s", "tail_parts", "prep_parts", "decode_thread_s", "prefetch_s", "decode_phases",
                    "pinned")})
                tim["per_rank"] = per_rank
                import torch
                w = torch.tensor([tim["wall_s"]], dtype=torch.float64)
                dist.all_reduce(w, op=dist.ReduceOp.MAX)
                rb = torch.tensor([tim["reads"], tim.get("bases", 0), tim.get("jobs", 0)], dtype=torch.int64)
                dist.all_reduce(rb)
                tim["cpu_s"] = sum(p["cpu_s"] for p in per_rank)
                tim["wall_s"], tim["reads"], tim["bases"], tim["jobs"] = float(w[0]), int(rb[0]), int(rb[1]), int(rb[2])
            if prof is not None:
                import pstats
                prof.disable()
                sfx = f"_r{rank}" if dist is not None else ""
                with open(f"{os.environ['E2E_PROFILE']}_{mode}{sfx}.txt", "w") as f:
                    pstats.Stats(prof, stream=f).sort_stats("cumulative").print_stats(60)
                    pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(40)
            runs.append(tim)
        timed = runs[1:] or runs   # (E2E_RUNS=0: the one run, a parity leg)
        best = min(timed, key=lambda t: t["wall_s"])
        bases = int(best.get("bases", 0))
        res[mode] = {"reads": best["reads"], "bases": bases, "jobs": best.get("jobs"),
                     "stages_s": {k: round(v, 3) for k, v in best.items() if k.endswith("_s")},
                     "reads_per_s": round(best["reads"] / best["wall_s"], 1),
                     "bases_per_s": round(bases / best["wall_s"], 1),
                     "wall_s_runs": [round(t["wall_s"], 3) for t in timed],
                     "peak_rss_mb": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss // 1024,
                     "workers": workers,
                     "critical_path_s_rank0": best.get("critical_path"),
                     "fastq_device_rank0": best.get("fastq_device"),
                     "decode_phases_rank0": best.get("decode_phases"),
                     "per_rank": best.get("per_rank"),
                     "coordinator_busy_s": best.get("resolve_s"),
                     "redos": best.get("redos"), "redos_unchanged": best.get("redos_unchanged"),
                     "first_run_wall_s": round(runs[0]["wall_s"], 3),
                     # host CPU seconds of all ranks over the run, and the cores that kept busy
                     "cpu_s": round(best["cpu_s"], 2), "cores_busy": round(best["cpu_s"] / best["wall_s"], 2),
                     "cpus_available": len(os.sched_getaffinity(0)),
                     "output_bytes": sum(os.path.getsize(os.path.join(out, f"{x}_{mode}{s}"))
                                         for x in ("tumor", "normal") for s in (".1.fastq", ".2.fastq"))}
        if rank == 0:
            print(json.dumps({mode: res[mode]}), file=sys.stderr, flush=True)
    if "stream" in res and "whole" in res:
        same = all(open(os.path.join(out, f"{x}_stream{s}"), "rb").read() ==
                   open(os.path.join(out, f"{x}_whole{s}"), "rb").read()
                   for x in ("tumor", "normal") for s in (".1.fastq", ".2.fastq"))
        res["stream_equals_whole"] = same
    if rank == 0 and os.environ.get("E2E_DIGEST") == "1":   # (outside the timed runs: A/B parity of settings)
        import hashlib
        dig = hashlib.sha1()
        for mode in res:
            if not isinstance(res[mode], dict):
                continue
            for x in ("tumor", "normal"):
                for sfx in (".1.fastq", ".2.fastq", ".single_end.fastq"):
                    p = os.path.join(out, f"{x}_{mode}{sfx}")
                    if os.path.exists(p):
                        with open(p, "rb") as f:
                            for blk in iter(lambda: f.read(1 << 24), b""):
                                dig.update(blk)
        res["output_sha1"] = dig.hexdigest()
    if rank == 0 and os.environ.get("E2E_DISK_PROBE") == "1":
        res["disk"] = disk_probe(out)
    if rank == 0:
        print(json.dumps(res))
    if dist is not None:
        from genomeanonymizer_amd.distributed import release_side_groups
        release_side_groups(dist)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
