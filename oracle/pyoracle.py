"""ctypes wrapper of oracle/build/libganon_oracle.so (see ganon_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker or the timed CPU baseline — never by the product.
``OracleEngine.mask`` has the signature of ``genomeanonymizer_amd.native.HipMasker.mask``
so the host planner can be checked on machines without a GPU.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libganon_oracle.so")
N_TOTALS = 8


class OracleEngine:
    def __init__(self):
        if not os.path.exists(LIB):
            import sys
            sys.path.insert(0, os.path.dirname(HERE))
            from genomeanonymizer_amd.build import build_oracle
            build_oracle()
        from genomeanonymizer_amd.native import GanonBatch
        self._lib = C.CDLL(LIB)
        self._lib.oracle_mask_batch.argtypes = [C.POINTER(GanonBatch), C.POINTER(C.c_uint8),
                                                C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                                C.POINTER(C.c_int64)]
        self._lib.oracle_mask_batch_mt.argtypes = self._lib.oracle_mask_batch.argtypes + [C.c_int]
        self.threads = 1

    def format_fastq(self, recs: dict) -> bytes:
        """The FASTQ restatement (fastq_oracle.py) with HipMasker.format_fastq's contract."""
        import fastq_oracle
        from genomeanonymizer_amd.native import FastqBadRecord
        try:
            return fastq_oracle.format_records(recs)
        except fastq_oracle.BadRecord as e:
            raise FastqBadRecord(e.index, str(e)) from None

    def mask(self, arrays: dict, indels: bool = False):
        from genomeanonymizer_amd.native import make_c_batch
        if indels:
            import indel_oracle
            from genomeanonymizer_amd.native import indel_records_array
            return self.mask(arrays) + (indel_records_array(indel_oracle.indel_records(arrays)),)
        b = make_c_batch(arrays)
        out = np.empty(b.seq_bytes, np.uint8)
        calls = np.zeros(b.n_scopes, np.int32)
        bases = np.zeros(b.n_scopes, np.int32)
        tot = np.zeros(N_TOTALS, np.int64)
        args = (C.byref(b), out.ctypes.data_as(C.POINTER(C.c_uint8)), calls.ctypes.data_as(C.POINTER(C.c_int32)),
                bases.ctypes.data_as(C.POINTER(C.c_int32)), tot.ctypes.data_as(C.POINTER(C.c_int64)))
        rc = (self._lib.oracle_mask_batch(*args) if self.threads == 1
              else self._lib.oracle_mask_batch_mt(*args, int(self.threads)))
        if rc != 0:
            raise RuntimeError(f"oracle_mask_batch failed: {rc}")
        return out, calls, bases, tot
