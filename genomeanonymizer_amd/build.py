"""In-tree build of the native libraries (no JIT cache: the .so files travel with the repo
snapshot to the GPU box).

* ``genomeanonymizer_amd/libganon_hip.so``  — HIP kernels (masking, FASTQ formatter) + C ABI
  (include/ganon.h), gfx950
* ``genomeanonymizer_amd/libganon_host.so`` — BAM decoder + FASTQ formatter (include/ganon_host.h)
* ``oracle/build/libganon_oracle.so``       — CPU restatement used by tests/bench only
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
HIP_LIB = os.path.join(PKG, "libganon_hip.so")
HOST_LIB = os.path.join(PKG, "libganon_host.so")
ORACLE_LIB = os.path.join(REPO, "oracle", "build", "libganon_oracle.so")
ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP library cannot be built")


def _stale(target: str, sources) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd) -> None:
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError(f"build failed: {' '.join(cmd)}")


HIP_SOURCES = ("ganon_hip.hip", "ganon_prep.hip", "ganon_fastq.hip", "ganon_indel.hip", "ganon_inflate.hip",
               "ganon_bam.hip")


def build_hip(force: bool = False) -> str:
    """One object per source, compiled in parallel, then linked (the rocPRIM sort in
    ganon_indel.hip is the slowest unit)."""
    srcs = [os.path.join(CSRC, s) for s in HIP_SOURCES]
    hdrs = [os.path.join(REPO, "include", "ganon.h"), os.path.join(CSRC, "ganon_ctx.h"), os.path.join(CSRC, "ganon_batch.h"),
            __file__]
    if not (force or _stale(HIP_LIB, srcs + hdrs)):
        return HIP_LIB
    objdir = os.path.join(PKG, "build")
    os.makedirs(objdir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
             "-Wno-unused-result", "-Wno-unused-value"]
    objs, procs = [], []
    for src in srcs:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            cmd = [_hipcc()] + flags + ["-c", "-o", obj + ".tmp", src]
            procs.append((cmd, obj, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                                     text=True)))
    failed = None
    for cmd, obj, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out)
            failed = failed or cmd
        else:
            os.replace(obj + ".tmp", obj)
    if failed:
        raise RuntimeError(f"build failed: {' '.join(failed)}")
    tmp = f"{HIP_LIB}.{os.getpid()}.tmp"
    _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs)
    os.replace(tmp, HIP_LIB)
    return HIP_LIB


HOST_SOURCES = ("ganon_host.cpp", "ganon_plan.cpp", "ganon_objects.cpp")


def build_host(force: bool = False) -> str:
    srcs = [os.path.join(CSRC, s) for s in HOST_SOURCES]
    hdr = os.path.join(REPO, "include", "ganon_host.h")
    if force or _stale(HOST_LIB, srcs + [hdr, __file__]):
        tmp = f"{HOST_LIB}.{os.getpid()}.tmp"
        _run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-pthread",
              "-o", tmp] + srcs + ["-lz", "-ldl"])
        os.replace(tmp, HOST_LIB)
    return HOST_LIB


def build_oracle(force: bool = False) -> str:
    src = os.path.join(REPO, "oracle", "ganon_oracle.c")
    hdr = os.path.join(REPO, "include", "ganon.h")
    os.makedirs(os.path.dirname(ORACLE_LIB), exist_ok=True)
    if force or _stale(ORACLE_LIB, [src, hdr, __file__]):
        tmp = f"{ORACLE_LIB}.{os.getpid()}.tmp"
        _run(["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-pthread", "-o", tmp, src])
        os.replace(tmp, ORACLE_LIB)
    return ORACLE_LIB


# the sources a PMC summary describes (tools/pmc_step.py, tools/fq_pmc_summary.py record their digest;
# bench.py cites a summary only while the digest still matches: PMC bytes of older kernels are not
# evidence for these)
DIGEST_SOURCES = {
    "mask": ("csrc/ganon_hip.hip", "csrc/ganon_prep.hip", "csrc/ganon_indel.hip", "csrc/ganon_ctx.h",
             "csrc/ganon_batch.h", "../include/ganon.h"),
    "fastq": ("csrc/ganon_fastq.hip", "csrc/ganon_ctx.h", "csrc/ganon_batch.h", "../include/ganon.h"),
}


def sources_digest(kind: str = "mask") -> str:
    """sha256 over the kernel sources of ``kind`` (DIGEST_SOURCES), in a fixed order."""
    import hashlib
    h = hashlib.sha256()
    for rel in DIGEST_SOURCES[kind]:
        p = os.path.normpath(os.path.join(PKG, rel))
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_all(force: bool = False) -> None:
    build_host(force)
    build_oracle(force)
    build_hip(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("built:", HIP_LIB, HOST_LIB, ORACLE_LIB)
