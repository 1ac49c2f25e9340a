"""The C-ABI libraries load and export every symbol their headers declare (no compute
calls without a GPU), and the product fails loudly instead of falling back."""
import ctypes
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header, macro):
    text = open(os.path.join(REPO, "include", header)).read()
    return set(re.findall(r"^" + macro + r"\s+[\w\s\*]*?\b(\w+)\s*\(", text, flags=re.M))


def test_hip_library_exports_header(hip_built):
    names = _declared("ganon.h", "GANON_API")
    assert len(names) >= 15
    lib = ctypes.CDLL(hip_built)
    for n in sorted(names):
        assert hasattr(lib, n), n
    from genomeanonymizer_amd import native
    assert set(native.EXPORTED_HIP_SYMBOLS) == names


def test_host_library_exports_header():
    from genomeanonymizer_amd import native
    names = _declared("ganon_host.h", "GANON_HOST_API")
    lib = ctypes.CDLL(native.HOST_LIB_PATH)
    for n in sorted(names):
        assert hasattr(lib, n), n
    assert set(native.EXPORTED_HOST_SYMBOLS) == names


def test_abi_version_and_struct_layout(hip_built):
    from genomeanonymizer_amd import native
    lib = native.hip_lib()
    assert lib.ganon_abi_version() == 5
    # ganon_batch: 2 int32 + 4 int64 + 17 pointers, naturally aligned
    assert ctypes.sizeof(native.GanonBatch) == 8 + 32 + 17 * 8
    # ganon_fastq_records: int64 + 2 int32 + 15 pointers
    assert ctypes.sizeof(native.GanonFastqRecords) == 8 + 8 + 15 * 8


def test_no_cpu_fallback_without_gpu(hip_built):
    """Without a gfx950 device the context cannot be created: GanonError, never a CPU path."""
    import os
    if os.path.exists("/dev/kfd"):   # an AMD GPU driver is present (torch may not see it here)
        pytest.skip("a GPU is present")
    from genomeanonymizer_amd import native
    with pytest.raises(native.GanonError):
        native.HipMasker(0)
    from genomeanonymizer_amd.anonymizer_methods import CompleteGermlineAnonymizer
    with pytest.raises(native.GanonError):
        CompleteGermlineAnonymizer().engine


def test_fastq_formatter_q1_q7():
    """Reverse reads: reverse-complemented bases, qualities in stored order (Q1);
    a non-ACGTN base on a reverse read is an error (Q7)."""
    from genomeanonymizer_amd import native
    from genomeanonymizer_amd.synth.batch import pack_nibbles
    lib = native.host_lib()
    C = ctypes
    seq = pack_nibbles(np.array([1, 2, 4, 8, 15, 1], np.uint8))   # ACGTNA
    qual = np.array([0, 1, 2, 3, 4, 5], np.uint8)
    u8p = C.POINTER(C.c_uint8)
    sb = (u8p * 1)(seq.ctypes.data_as(u8p))
    qb = (u8p * 1)(qual.ctypes.data_as(u8p))
    out = C.create_string_buffer(256)

    def fmt(rev, s=sb):
        one = lambda v, t: (t * 1)(v)
        return lib.ganon_fastq_format(1, s, one(0, C.c_uint8), one(0, C.c_int64), one(6, C.c_int32),
                                      one(rev, C.c_uint8), qb, one(0, C.c_uint8), one(0, C.c_int64),
                                      one(6, C.c_int32), one(0, C.c_uint8), b"rd", one(0, C.c_int64),
                                      one(2, C.c_int32), one(2, C.c_uint8), out, 256)
    n = fmt(0)
    assert out.raw[:n] == b"@rd/2\nACGTNA\n+\n!\"#$%&\n"
    n = fmt(1)
    assert out.raw[:n] == b"@rd/2\nTNACGT\n+\n!\"#$%&\n"
    bad = pack_nibbles(np.array([1, 5, 4, 8, 15, 1], np.uint8))     # R on a reverse read
    sb2 = (u8p * 1)(bad.ctypes.data_as(u8p))
    assert fmt(1, sb2) == -1
