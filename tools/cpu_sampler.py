#!/usr/bin/env python3
"""CPU attribution of a multi-threaded Python + native run (no perf on the box): a sampler thread
reads, every PERIOD seconds, each thread's on-CPU nanoseconds (/proc/self/task/<tid>/schedstat) and
charges the delta since its previous sample to that thread's current Python stack (the innermost
frames; native code is charged to the Python call that entered it). Threads the sampler does not know
as Python threads (the native libraries' own pools) are charged as a whole, per thread name. The
report lists the top call sites by CPU seconds and the process's CPU total, so the attributed share
is visible.

    with Sampler() as s: ...;  s.report(path)        (tools/e2e_bench.py: E2E_SAMPLE=PREFIX)
"""
import collections
import json
import os
import sys
import threading
import time


def _task_cpu_ns(tid: int) -> int:
    try:
        with open(f"/proc/self/task/{tid}/schedstat") as fh:
            return int(fh.read().split()[0])
    except (OSError, ValueError, IndexError):
        return -1


def _task_name(tid: int) -> str:
    try:
        with open(f"/proc/self/task/{tid}/comm") as fh:
            return fh.read().strip()
    except OSError:
        return "?"


class Sampler:
    def __init__(self, period: float = 0.002, depth: int = 3):
        self.period = period
        self.depth = depth
        self.by_site = collections.Counter()     # (thread name, frames) -> ns
        self.by_thread = collections.Counter()   # thread name -> ns
        self.native = collections.Counter()      # native thread name -> ns
        self._last = {}
        self._stop = threading.Event()
        self._t = None
        self.wall = 0.0
        self.cpu0 = None

    def _frames(self, frame) -> str:
        out = []
        while frame is not None and len(out) < self.depth:
            co = frame.f_code
            out.append(f"{os.path.basename(co.co_filename)}:{co.co_name}:{frame.f_lineno}")
            frame = frame.f_back
        return " < ".join(out)

    def _sample(self) -> None:
        me = threading.get_native_id()
        py = {t.native_id: t for t in threading.enumerate() if t.native_id is not None}
        frames = sys._current_frames()
        try:
            tids = [int(x) for x in os.listdir("/proc/self/task")]
        except OSError:
            return
        for tid in tids:
            if tid == me:
                continue
            ns = _task_cpu_ns(tid)
            if ns < 0:
                continue
            prev = self._last.get(tid)
            self._last[tid] = ns
            if prev is None:
                continue
            d = ns - prev
            if d <= 0:
                continue
            t = py.get(tid)
            if t is None:
                self.native[_task_name(tid)] += d
                continue
            name = t.name.split("_")[0] if t.name.startswith("ThreadPoolExecutor") else t.name
            self.by_thread[name] += d
            f = frames.get(t.ident)
            self.by_site[(name, self._frames(f) if f is not None else "?")] += d

    def _run(self) -> None:
        while not self._stop.wait(self.period):
            self._sample()

    def __enter__(self):
        self.cpu0 = os.times()
        self.t0 = time.time()
        self._sample()
        self._t = threading.Thread(target=self._run, daemon=True, name="cpu-sampler")
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join()
        self._sample()
        self.wall = time.time() - self.t0
        c1 = self.cpu0, os.times()
        self.cpu_s = (c1[1].user - c1[0].user) + (c1[1].system - c1[0].system)
        return False

    def report(self, path: str, top: int = 60) -> dict:
        tot = sum(self.by_thread.values()) + sum(self.native.values())
        res = {"wall_s": round(self.wall, 3), "process_cpu_s": round(self.cpu_s, 3),
               "sampled_cpu_s": round(tot / 1e9, 3),
               "threads_s": {k: round(v / 1e9, 3) for k, v in self.by_thread.most_common()},
               "native_threads_s": {k: round(v / 1e9, 3) for k, v in self.native.most_common(20)},
               "sites_s": [[k[0], k[1], round(v / 1e9, 4)] for k, v in self.by_site.most_common(top)]}
        with open(path, "w") as fh:
            json.dump(res, fh, indent=1)
        return res
