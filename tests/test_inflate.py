"""BGZF inflate offload: the host BAM reader's inflater hook
(ganon_bam_reader_set_inflater, include/ganon_host.h) and the GPU inflate (ganon_inflate,
include/ganon.h).

Parity: DEFLATE is a fixed format (RFC 1951), so Python's zlib — the library htslib's bgzf_read
calls behind the reference's AlignmentFile (pileup_io.pyx:12-17) — is the oracle: every stream
here is made by zlib (all block types: stored, fixed and dynamic Huffman; every strategy) or taken
from a BAM our writer made with it, and the GPU output must equal zlib's byte for byte.
"""
import ctypes as C
import dataclasses
import os
import zlib

import numpy as np
import pytest


def _bgzf_blocks(path):
    """(payloads, isizes) of a BGZF file's non-empty blocks, parsed in Python."""
    data = open(path, "rb").read()
    pay, isz, off = [], [], 0
    while off < len(data):
        xlen = data[off + 10] | (data[off + 11] << 8)
        bsize = None
        x = off + 12
        while x < off + 12 + xlen:
            slen = data[x + 2] | (data[x + 3] << 8)
            if data[x] == 66 and data[x + 1] == 67:
                bsize = data[x + 4] | (data[x + 5] << 8)
            x += 4 + slen
        blen = bsize + 1
        n = int.from_bytes(data[off + blen - 4:off + blen], "little")
        if n:
            pay.append(data[off + 12 + xlen:off + blen - 8])
            isz.append(n)
        off += blen
    return pay, isz


def _zlib_streams():
    """Raw DEFLATE streams of every block type and strategy, with their inflated bytes."""
    rng = np.random.default_rng(7)
    texts = [
        b"",
        b"A",
        bytes(rng.integers(0, 256, 65536, dtype=np.uint8)),                      # incompressible
        rng.choice(np.frombuffer(b"ACGTN", np.uint8), 65536, p=[.3, .2, .2, .29, .01]).tobytes(),   # bases
        b"\x00" * 65536,                                                          # one long run
        (b"@read_%d\nACGTACGTTTGA\n+\nIIIIHHHG#\n" * 2500)[:65536],              # FASTQ-like repeats
        bytes(rng.integers(30, 42, 40000, dtype=np.uint8)),                      # qualities
        np.repeat(rng.integers(0, 256, 3000, dtype=np.uint8), rng.integers(1, 40, 3000)).tobytes()[:65536],
    ]
    out = []
    for t in texts:
        for level, strategy in ((0, zlib.Z_DEFAULT_STRATEGY), (1, zlib.Z_DEFAULT_STRATEGY),
                                (6, zlib.Z_DEFAULT_STRATEGY), (9, zlib.Z_DEFAULT_STRATEGY), (6, zlib.Z_FIXED),
                                (6, zlib.Z_HUFFMAN_ONLY), (6, zlib.Z_RLE), (9, zlib.Z_FILTERED)):
            c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
            out.append((c.compress(t) + c.flush(), t))
    # several deflate blocks in one stream (flushes), a stored block between Huffman ones
    t = rng.choice(np.frombuffer(b"ACGT", np.uint8), 60000).tobytes()
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    parts = [c.compress(t[:20000]), c.flush(zlib.Z_FULL_FLUSH), c.compress(t[20000:40000]),
             c.flush(zlib.Z_SYNC_FLUSH), c.compress(t[40000:]), c.flush()]
    out.append((b"".join(parts), t))
    return out


def _soa(streams):
    comp = b"".join(s for s, _ in streams)
    in_len = np.array([len(s) for s, _ in streams], np.int32)
    in_off = np.zeros(len(streams), np.int64)
    in_off[1:] = np.cumsum(in_len[:-1])
    out_len = np.array([len(t) for _, t in streams], np.int32)
    return np.frombuffer(comp, np.uint8), in_off, in_len, out_len


class _ZlibInflater:
    """An inflater callback in Python (zlib): exercises the reader's hook without a GPU."""
    FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint8), C.c_int64, C.POINTER(C.c_int64),
                     C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.c_int64,
                     C.POINTER(C.c_uint8), C.c_int64)

    def __init__(self, fail=False):
        self.calls, self.blocks, self.fail = 0, 0, fail
        self._cb = self.FN(self._inflate)
        self.fn = C.cast(self._cb, C.c_void_p)
        self.handle = None
        self.min_blocks = 1

    def _inflate(self, user, comp, comp_len, in_off, in_len, out_off, out_len, n, out, out_total):
        self.calls += 1
        self.blocks += n
        if self.fail:
            return 1
        src = C.string_at(comp, comp_len)
        dst = (C.c_uint8 * out_total).from_address(C.addressof(out.contents))
        for i in range(n):
            b = zlib.decompress(src[in_off[i]:in_off[i] + in_len[i]], -15)
            if len(b) != out_len[i]:
                return 1
            dst[out_off[i]:out_off[i] + out_len[i]] = b
        return 0


def test_reader_inflater_hook_matches_zlib_threads(tmp_path):
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.io.bam import BamReader
    from genomeanonymizer_amd.synth.generate import generate, scenario
    paths = generate(dataclasses.replace(scenario("config1"), bam_index=False), str(tmp_path / "in"))
    ref = BamReader(paths["T"], threads=2, window=1 << 17)
    inf = _ZlibInflater()
    R = BamReader(paths["T"], threads=2, window=1 << 17, inflater=inf)
    for tid in range(len(ref.ref_names)):
        a, b = ref.contig(tid), R.contig(tid)
        assert a.n == b.n
        for f in ("pos", "flag", "l_seq", "cigar", "seq", "qual", "aux", "names_blob"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert inf.calls > 0 and inf.blocks > 0
    R.close()
    ref.close()
    bad = _ZlibInflater(fail=True)
    R = BamReader(paths["T"], threads=2, window=1 << 17, inflater=bad)
    with pytest.raises(native.GanonError, match="inflate"):
        R.contig(0)
    R.close()


def _bad_cases(rng):
    t = rng.choice(np.frombuffer(b"ACGT", np.uint8), 30000).tobytes()
    good = zlib.compress(t, 6)[2:-4]
    return t, good, [
        (good, len(t) + 1),                                    # ISIZE disagrees
        (good[:len(good) // 2], len(t)),                       # truncated
        (b"\x07" + good[1:], len(t)),                          # BTYPE 3 (reserved)
        (bytes([0x01, 0x05, 0x00, 0x00, 0x00]) + b"abcde", 5),  # stored LEN/NLEN mismatch
        (bytes(rng.integers(0, 256, 4000, dtype=np.uint8)), 65536),   # noise
    ]


@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    """tools/inflate_host_check.cpp built with hipcc: the kernel's decoder source run on the host."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc is not available")
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    exe = str(tmp_path_factory.mktemp("ihc") / "inflate_host_check")
    subprocess.run([hipcc, "-O2", "-std=c++17", "--offload-arch=gfx950", "-x", "hip",
                    os.path.join(root, "tools", "inflate_host_check.cpp"), "-o", exe], check=True)
    d = tmp_path_factory.mktemp("ihc_io")

    def run(streams):
        comp, in_off, in_len, out_len = _soa(streams)
        comp.tofile(d / "comp.bin")
        meta = np.stack([in_off, in_len.astype(np.int64), out_len.astype(np.int64)], 1).ravel()
        np.concatenate([[len(streams)], meta]).astype(np.int64).tofile(d / "meta.bin")
        r = subprocess.run([exe, str(d / "comp.bin"), str(d / "meta.bin"), str(d / "out.bin")], check=True,
                           capture_output=True, text=True)
        return [int(x) for x in r.stdout.split()], open(d / "out.bin", "rb").read()
    return run


def test_decoder_source_matches_zlib_on_host(host_check):
    streams = _zlib_streams()
    status, out = host_check(streams)
    assert status == [0] * len(streams)
    assert out == b"".join(t for _, t in streams)
    _, _, bad = _bad_cases(np.random.default_rng(3))
    status, _ = host_check([(s, b"\x00" * n) for s, n in bad])
    assert all(x != 0 for x in status)


def test_zlib_streams_cover_every_block_type():
    """The fixture streams hold stored (BTYPE 0), fixed (1) and dynamic (2) first blocks."""
    kinds = {(s[0] >> 1) & 3 for s, _ in _zlib_streams() if s}
    assert kinds == {0, 1, 2}


@pytest.fixture(scope="module")
def gpu_inflater(hip_built):
    from genomeanonymizer_amd import native
    g = native.GpuInflater(0, min_blocks=1)
    yield g
    g.close()


@pytest.mark.gpu
def test_gpu_inflate_matches_zlib(gpu_inflater):
    streams = _zlib_streams()
    comp, in_off, in_len, out_len = _soa(streams)
    out = gpu_inflater.inflate(comp, in_off, in_len, out_len)
    assert out.tobytes() == b"".join(t for _, t in streams)
    # one at a time too (a grid of one block; buffers reused at a smaller size)
    for s, t in streams[::7]:
        c, a, b, o = _soa([(s, t)])
        assert gpu_inflater.inflate(c, a, b, o).tobytes() == t


@pytest.mark.gpu
def test_gpu_inflate_real_bgzf_blocks(gpu_inflater, tmp_path):
    from genomeanonymizer_amd.synth.generate import generate, scenario
    paths = generate(scenario("config1"), str(tmp_path / "in"))
    pay, isz = _bgzf_blocks(paths["T"])
    streams = [(p, zlib.decompress(p, -15)) for p in pay]
    assert [len(t) for _, t in streams] == isz
    comp, in_off, in_len, out_len = _soa(streams * 40)   # thousands of blocks in one launch
    out = gpu_inflater.inflate(comp, in_off, in_len, out_len)
    assert out.tobytes() == b"".join(t for _, t in streams) * 40


@pytest.mark.gpu
def test_gpu_inflate_rejects_bad_streams(gpu_inflater):
    from genomeanonymizer_amd import native
    t, good, cases = _bad_cases(np.random.default_rng(3))
    for k, (s, n) in enumerate(cases):
        streams = [(good, t), (s, b"\x00" * n)]
        comp, in_off, in_len, out_len = _soa(streams)
        with pytest.raises(native.GanonError, match="block 1"):
            gpu_inflater.inflate(comp, in_off, in_len, out_len)
    # the context still works after failures
    comp, in_off, in_len, out_len = _soa([(good, t)])
    assert gpu_inflater.inflate(comp, in_off, in_len, out_len).tobytes() == t


@pytest.mark.gpu
def test_gpu_inflater_in_the_contig_reader(hip_built, tmp_path):
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.io.bam import BamReader
    from genomeanonymizer_amd.synth.generate import generate, scenario
    paths = generate(scenario("config1"), str(tmp_path / "in"))
    g = native.GpuInflater(0, min_blocks=1)
    ref = BamReader(paths["N"], threads=2, window=1 << 17)
    R = BamReader(paths["N"], threads=2, window=1 << 17, inflater=g)
    for tid in range(len(ref.ref_names)):
        a, b = ref.contig(tid), R.contig(tid)
        assert a.n == b.n
        for f in ("pos", "flag", "cigar", "seq", "qual", "aux", "names_blob"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), f
    R.close()
    ref.close()
    g.close()
