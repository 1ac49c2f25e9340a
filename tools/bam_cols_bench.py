"""Device BAM record walk (ganon_bam_columns) against the host decoder on one large stream.

The stream: the records of a generated configs[0] BAM tiled to about --mb MB of inflated records
(150 bp paired reads, ~265 bytes a record). The device side is timed per kernel with HIP events
(ganon_last_kernel_times: k_bam_guess, k_bam_check, k_bam_fix, k_bam_offsets, k_bam_sizes, the
five scans, k_bam_scatter) with the stream already in device memory; the host side is
libganon_host.so's ganon_bam_open on the same records written as stored (level-0) BGZF blocks, so
that its inflate is a copy and the time is mostly the record walk's (one thread and --threads
threads; the file read included). Every device column must equal the host decoder's. Prints one
JSON line (bench.py's `bam_decode` side line runs this as a child).
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

COLS = ("tid", "pos", "end", "flag", "mapq", "l_seq", "n_cigar", "mate_tid", "mate_pos", "tlen", "name_len", "aux_len",
        "name_off", "cig_off", "seq_off", "qual_off", "aux_off")
BLOBS = ("names_blob", "cigar", "seq", "qual", "aux")
HBM_PEAK_GBPS = 8000.0


def measure(mb: int = 256, threads: int = 16, reps: int = 3) -> dict:
    import gzip
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.io.bam import ReadTable
    from genomeanonymizer_amd.synth.bamwriter import first_record_offset, write_bgzf
    from genomeanonymizer_amd.synth.generate import generate, scenario
    tmp = tempfile.mkdtemp(prefix="bamcols_")
    try:
        paths = generate(scenario("config1"), os.path.join(tmp, "in"))
        d = gzip.decompress(open(paths["T"], "rb").read())
        p = first_record_offset(d)
        head, recs = d[:p], d[p:]
        tiles = max(1, (mb << 20) // max(1, len(recs)))
        stream = np.frombuffer(head + recs * tiles, np.uint8)
        g = native.GpuInflater(0, min_blocks=1)
        lib = native.hip_lib()
        g.set_profiling(True)
        runs = []
        cols, _ = native.bam_columns_device(g.handle, stream, p, len(stream), on_host=True)   # (warm: blocks cached)
        for _ in range(reps):
            t0 = time.perf_counter()
            cols, fixes = native.bam_columns_device(g.handle, stream, p, len(stream), on_host=True)
            wall = time.perf_counter() - t0
            arr = (native.KernelTime * 32)()
            k = lib.ganon_last_kernel_times(g.handle, arr, 32)
            per = {}
            for i in range(min(k, 32)):
                name = arr[i].name.decode()
                per[name] = per.get(name, 0.0) + float(arr[i].ms)
            runs.append((sum(per.values()), per, wall, fixes))
        g.close()
        best = min(runs, key=lambda x: x[0])
        nr = len(cols["pos"])
        path = os.path.join(tmp, "big0.bam")
        write_bgzf(path, stream.tobytes(), level=0)
        host = {}
        t = None
        for th in (1, threads):
            t0 = time.perf_counter()
            t = ReadTable(path, threads=th)
            host[th] = time.perf_counter() - t0
        equal = len(cols["pos"]) == t.n and all(np.array_equal(cols[f], getattr(t, f)) for f in COLS + BLOBS)
        out_bytes = sum(cols[f].nbytes for f in COLS + BLOBS) + cols["rec_off"].nbytes
        alg = (len(stream) - p) + out_bytes   # the records read once, the columns written once
        ms = best[0]
        return {
            "metric": "BAM records decoded to columns per second (device record walk)", "unit": "records/s",
            "value": round(nr / (ms / 1e3), 1), "records": nr, "stream_MB": round(len(stream) / 2**20, 1),
            "device_ms": round(ms, 3), "device_kernels_ms": {k: round(v, 3) for k, v in best[1].items()},
            "roofline": {"bound": "hbm", "achieved": round(alg / (ms / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                         "algorithmic_bytes": int(alg), "traffic": None},
            "device_call_wall_s": round(best[2], 3), "guess_fixes": best[3],
            "host_decoder_s": {str(k): round(v, 3) for k, v in host.items()},
            "host_records_per_s": {str(k): round(nr / v, 1) for k, v in host.items()},
            "columns_equal_host_decoder": bool(equal),
            "workload": f"configs[0] tumor BAM records tiled x{tiles} ({nr} records, 150 bp); device: the stream "
                        f"resident in HBM, kernels only (HIP events on the context's stream); call wall adds the H2D "
                        f"copy, the scans' host reads and the D2H of the columns; host: ganon_bam_open of the same "
                        f"records as stored BGZF blocks (inflate = copy), file read included",
        }
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=256)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    print(json.dumps(measure(args.mb, args.threads, args.reps)))


if __name__ == "__main__":
    main()
