#!/usr/bin/env python3
"""Build an A/B variant of libganon_hip.so with extra compile-time defines (tuning only), e.g.
    python tools/build_variant.py ke5 -DGANON_KE_BLOCKS=5
writes genomeanonymizer_amd/variants/libganon_hip_ke5.so; select it at run time with
GANON_HIP_LIB=<path> (native.py). The product always loads the default in-tree build."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from genomeanonymizer_amd.build import ARCH, CSRC, HIP_SOURCES, PKG, _hipcc  # noqa: E402


def main() -> None:
    tag, defines = sys.argv[1], sys.argv[2:]
    out_dir = os.path.join(PKG, "variants")
    obj_dir = os.path.join(out_dir, "obj_" + tag)
    os.makedirs(obj_dir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wno-unused-result",
             "-Wno-unused-value"] + defines
    procs, objs = [], []
    for s in HIP_SOURCES:
        o = os.path.join(obj_dir, s + ".o")
        objs.append(o)
        procs.append(subprocess.Popen([_hipcc()] + flags + ["-c", "-o", o, os.path.join(CSRC, s)]))
    if any(p.wait() for p in procs):
        sys.exit("variant build failed")
    lib = os.path.join(out_dir, f"libganon_hip_{tag}.so")
    subprocess.check_call([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs)
    print(lib)


if __name__ == "__main__":
    main()
