"""ASan/UBSan build of the host code that parses untrusted input or follows untrusted indices
(ADVICE r1): the BGZF/BAM decoder and FASTQ formatter (csrc/ganon_host.cpp), the scope
planner (csrc/ganon_plan.cpp) and the C oracle (oracle/ganon_oracle.c), linked into one driver
executable (tests/sanitize/sanitize_driver.cpp) — no preloading, the sanitizer runtime is linked
in. Valid pairs are planned and formatted; malformed BGZF/BAM files must be rejected with an error
code, never read out of bounds. CPU only."""
import os
import shutil
import struct
import subprocess
import zlib

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-O1", "-g"]


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if not shutil.which("g++") or not shutil.which("gcc"):
        pytest.skip("no host compiler")
    d = tmp_path_factory.mktemp("san")
    obj = str(d / "oracle.o")
    exe = str(d / "sanitize_driver")
    subprocess.run(["gcc", *SAN, "-std=c11", "-c", os.path.join(REPO, "oracle", "ganon_oracle.c"), "-o", obj],
                   check=True, capture_output=True)
    r = subprocess.run(["g++", *SAN, "-std=c++17", "-pthread", "-o", exe,
                        os.path.join(REPO, "tests", "sanitize", "sanitize_driver.cpp"),
                        os.path.join(REPO, "genomeanonymizer_amd", "csrc", "ganon_host.cpp"),
                        os.path.join(REPO, "genomeanonymizer_amd", "csrc", "ganon_plan.cpp"), obj, "-lz"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def _run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, *args], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


def _bgzf_block(payload: bytes, isize=None, bsize_override=None, xlen_extra=b"") -> bytes:
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    cdata = c.compress(payload) + c.flush()
    extra = b"BC" + struct.pack("<H", 2) + struct.pack("<H", 0) + xlen_extra
    bsize = 12 + len(extra) + len(cdata) + 8 - 1
    extra = b"BC" + struct.pack("<H", 2) + struct.pack("<H", bsize if bsize_override is None else bsize_override) + xlen_extra
    head = bytes([31, 139, 8, 4, 0, 0, 0, 0, 0, 255]) + struct.pack("<H", len(extra))
    tail = struct.pack("<I", zlib.crc32(payload)) + struct.pack("<I", len(payload) if isize is None else isize)
    return head + extra + cdata + tail


def test_oracle_under_sanitizers(driver):
    for seed in (1, 2, 3, 4):
        assert "calls" in _run(driver, "oracle", str(seed))


@pytest.mark.parametrize("name", ["tiny", "edge"])
def test_decoder_planner_formatter_under_sanitizers(driver, name, tmp_path):
    from genomeanonymizer_amd.io.fasta import FastaRef
    from genomeanonymizer_amd.io.vcf import read_vcf
    from genomeanonymizer_amd.planner import get_windows
    from genomeanonymizer_amd.synth.generate import generate, scenario
    paths = generate(scenario(name), str(tmp_path / "in"))
    fa = FastaRef(paths["ref"])
    refs = list(fa.references)
    wins = get_windows(read_vcf(paths["vcf"]), fa.index)
    spec = tmp_path / "spec.txt"
    lines = [str(len(refs))] + [f"{c} {n}" for c, n in zip(refs, fa.lengths)] + [str(len(wins))]
    lines += [f"{refs.index(w.sequence)} {w.first} {w.last}" for w in wins]
    spec.write_text("\n".join(lines) + "\n")
    out = _run(driver, "plan", paths["T"], paths["N"], str(spec))
    assert "plan:" in out and "fastq 1:" in out


def test_malformed_bam_files_are_rejected_cleanly(driver, tmp_path):
    from genomeanonymizer_amd.synth.generate import generate, scenario
    paths = generate(scenario("tiny"), str(tmp_path / "in"))
    good = open(paths["T"], "rb").read()
    files = []

    def put(tag, data):
        p = tmp_path / f"bad_{tag}.bam"
        p.write_bytes(data)
        files.append(str(p))

    for cut in (1, 17, 18, 30, len(good) // 3, len(good) - 1):
        put(f"trunc{cut}", good[:cut])
    b = bytearray(good)
    b[10:12] = struct.pack("<H", 0xFFFF)             # XLEN past the end of the file
    put("xlen", bytes(b))
    b = bytearray(good)
    b[16:18] = struct.pack("<H", 3)                   # BSIZE smaller than the block header
    put("bsize", bytes(b))
    b = bytearray(good)
    b[12:14] = b"XY"                                   # no BC subfield
    put("nobc", bytes(b))
    bam = b"BAM\x01" + struct.pack("<i", -5) + b"\x00" * 8
    put("ltext", _bgzf_block(bam))                    # negative l_text
    bam = b"BAM\x01" + struct.pack("<i", 0) + struct.pack("<i", -3)
    put("nref", _bgzf_block(bam))                     # negative n_ref
    bam = b"BAM\x01" + struct.pack("<i", 0) + struct.pack("<i", 0) + struct.pack("<i", 40) + b"\x00" * 36
    put("recsize", _bgzf_block(bam))                  # record larger than the stream
    bam = b"BAM\x01" + struct.pack("<i", 0) + struct.pack("<i", 0) + struct.pack("<i", 32) + b"\xff" * 32
    put("fields", _bgzf_block(bam))                   # record fields past its size
    put("isize", _bgzf_block(b"BAM\x01" + b"\x00" * 8, isize=0xFFFFFFF0))   # ISIZE over 64 KiB
    put("subfield", _bgzf_block(b"BAM\x01" + b"\x00" * 8, xlen_extra=b"ZZ\xff\x00"))  # subfield past XLEN
    rng = np.random.default_rng(5)
    for k in range(24):                               # random byte flips in the first block
        b = bytearray(good)
        for _ in range(4):
            b[int(rng.integers(0, min(len(b), 400)))] = int(rng.integers(0, 256))
        put(f"flip{k}", bytes(b))
    out = _run(driver, "bam", paths["T"], *files)
    assert f"decoded " in out
    dec, rej = out.strip().split("\n")[-1].split()[1::2]
    assert int(rej) >= 14


def test_fastq_edit_and_gather_under_sanitizers(driver):
    """ganon_fastq_edit on random, truncated and oddly edited records, ganon_gather_ranges in and out
    of bounds: no sanitizer report, malformed input refused with an error code."""
    for seed in (1, 2):
        out = _run(driver, "edit", str(seed))
        ok, refused = (int(x.split("=")[1]) for x in out.split()[1:3])
        assert ok > 1000 and refused > 100, out       # both paths exercised
