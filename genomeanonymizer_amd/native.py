"""ctypes bindings of the two in-tree native libraries.

* ``libganon_hip.so`` (include/ganon.h): the HIP masking kernels and the HIP FASTQ
  formatter (``ganon_fastq_*``). There is no CPU
  implementation behind it; loading or creating a context fails loudly without a gfx950
  device (``GanonError``), never falls back.
* ``libganon_host.so`` (include/ganon_host.h): BAM decoder and FASTQ formatter.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import weakref
import time
from typing import Dict, Optional, Tuple

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
# GANON_HIP_LIB: another in-tree build of the same sources (compile-time tuning A/B only)
HIP_LIB_PATH = os.environ.get("GANON_HIP_LIB") or os.path.join(_PKG, "libganon_hip.so")
HOST_LIB_PATH = os.path.join(_PKG, "libganon_host.so")

GANON_N_TOTALS = 8
TOTAL_NAMES = ("masked_snv_calls", "masked_bases", "reads_in", "reads_written", "scopes",
               "rare_scopes", "large_tiles", "reserved")


class GanonError(RuntimeError):
    pass


_p = C.c_void_p
# a fresh, unshared bytes object of n bytes (contents undefined) for a library to fill in place
_new_bytes = C.pythonapi.PyBytes_FromStringAndSize
_new_bytes.restype = C.py_object
_new_bytes.argtypes = [C.c_void_p, C.c_ssize_t]
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_u8p = C.POINTER(C.c_uint8)
# ganon_bam_cols member order (include/ganon.h)
BAM_I32_COLS = ("tid", "pos", "end", "flag", "mapq", "l_seq", "n_cigar", "mate_tid", "mate_pos", "tlen", "name_len",
                "aux_len")
BAM_I64_COLS = ("name_off", "cig_off", "seq_off", "qual_off", "aux_off", "rec_off")
_u32p = C.POINTER(C.c_uint32)


class GanonBatch(C.Structure):
    """Mirror of ``ganon_batch`` (include/ganon.h)."""
    _fields_ = [
        ("n_reads", C.c_int32), ("n_scopes", C.c_int32), ("n_incid", C.c_int64),
        ("seq_bytes", C.c_int64), ("n_cigar_ops", C.c_int64), ("ref_bytes", C.c_int64),
        ("ref_start", _i32p), ("read_len", _i32p), ("seq_off", _i64p), ("seq_nt16", _u8p),
        ("cig_off", _i64p), ("n_cig", _i32p), ("cigar", _u32p), ("dataset", _u8p),
        ("write_scope", _i32p),
        ("scope_incid_off", _i64p), ("incid_read", _i32p), ("scope_span_start", _i32p),
        ("scope_span_len", _i32p), ("scope_ref_off", _i64p), ("ref_nt16", _u8p),
        ("keep_pos", _i32p), ("keep_code", _u8p),
    ]


class GanonFastqRecords(C.Structure):
    """Mirror of ``ganon_fastq_records`` (include/ganon.h)."""
    _fields_ = [
        ("n", C.c_int64), ("n_seq_bufs", C.c_int32), ("n_qual_bufs", C.c_int32),
        ("seq_buf", C.POINTER(_u8p)), ("seq_batch", _p), ("seq_sel", _u8p), ("seq_nib_off", _i64p),
        ("seq_len", _i32p), ("reverse", _u8p), ("qual_buf", C.POINTER(_u8p)), ("qual_sel", _u8p),
        ("qual_off", _i64p), ("qual_len", _i32p), ("qual_rev", _u8p), ("names", C.c_char_p),
        ("name_off", _i64p), ("name_len", _i32p), ("mate", _u8p),
    ]


# ganon_indel_rec (include/ganon.h): one masked TN indel call (kind 0) or one support of it by
# a read its scope writes (kind 1)
INDEL_REC = np.dtype([("scope", np.int32), ("pos", np.int32), ("length", np.int32), ("type", np.int32),
                      ("rank", np.int32), ("kind", np.int32), ("read", np.int32), ("in_read_pos", np.int32)])
INDEL_DEL, INDEL_INS = 2, 3
INDEL_CALL, INDEL_SUPPORT = 0, 1


def indel_records_array(rows) -> np.ndarray:
    """Records as a structured array sorted by (scope, pos, rank, kind, read): the device's order
    is not part of the contract."""
    a = np.array([tuple(r) for r in rows], INDEL_REC) if not isinstance(rows, np.ndarray) else rows
    if len(a) == 0:
        return np.zeros(0, INDEL_REC)
    o = np.lexsort((a["in_read_pos"], a["read"], a["kind"], a["rank"], a["pos"], a["scope"]))
    return a[o]


class KernelTime(C.Structure):
    _fields_ = [("name", C.c_char * 48), ("launches", C.c_int32), ("ms", C.c_float)]


# numpy field spec of a batch: name -> dtype
BATCH_ARRAYS = {
    "ref_start": np.int32, "read_len": np.int32, "seq_off": np.int64, "seq_nt16": np.uint8,
    "cig_off": np.int64, "n_cig": np.int32, "cigar": np.uint32, "dataset": np.uint8,
    "write_scope": np.int32, "scope_incid_off": np.int64, "incid_read": np.int32,
    "scope_span_start": np.int32, "scope_span_len": np.int32, "scope_ref_off": np.int64,
    "ref_nt16": np.uint8, "keep_pos": np.int32, "keep_code": np.uint8,
}


_PTR_OF = {np.int32: _i32p, np.int64: _i64p, np.uint8: _u8p, np.uint32: _u32p}


def indel_view(arrays: dict) -> dict:
    """The batch as the indel tally sees it: ``indel_incid_off``/``indel_incid_read`` (when the
    plan leaves later alignments of a read out, anonymizer_methods.build_batch) replace the
    incidence CSR."""
    if "indel_incid_off" not in arrays:
        return arrays
    a = dict(arrays)
    a["scope_incid_off"] = arrays["indel_incid_off"]
    a["incid_read"] = arrays["indel_incid_read"]
    return a


def make_c_batch(arrays: dict, with_ref: bool = True) -> GanonBatch:
    """Build a GanonBatch over numpy arrays (kept alive by the caller's dict). ``with_ref`` False:
    the reference is resident on the device, ``ref_nt16`` may be absent."""
    b = GanonBatch()
    for name, dt in BATCH_ARRAYS.items():
        if name == "ref_nt16" and not with_ref and name not in arrays:
            continue
        a = arrays[name]
        if a.dtype != dt or not a.flags["C_CONTIGUOUS"]:
            raise GanonError(f"batch array {name} must be C-contiguous {np.dtype(dt)}")
        setattr(b, name, a.ctypes.data_as(_PTR_OF[dt]))
    b.n_reads = len(arrays["read_len"])
    b.n_scopes = len(arrays["scope_span_len"])
    b.n_incid = len(arrays["incid_read"])
    b.seq_bytes = len(arrays["seq_nt16"])
    b.n_cigar_ops = len(arrays["cigar"])
    b.ref_bytes = len(arrays["ref_nt16"]) if "ref_nt16" in arrays else 0
    return b


_hip = None
_host = None


_HIP_CONTEXTS = [0]   # HipMasker contexts created in this process (page-locked buffers need a GPU)


def hip_loaded() -> bool:
    """Whether this process drives the GPU (a HipMasker exists): page-locked staging only then."""
    return _HIP_CONTEXTS[0] > 0


def hip_lib():
    """Load libganon_hip.so (raises GanonError if it is missing)."""
    global _hip
    if _hip is not None:
        return _hip
    if not os.path.exists(HIP_LIB_PATH):
        raise GanonError(f"{HIP_LIB_PATH} is missing: run __graft_entry__.build() (hipcc, gfx950)")
    lib = C.CDLL(HIP_LIB_PATH)
    lib.ganon_abi_version.restype = C.c_int
    lib.ganon_ctx_create.argtypes = [C.c_int, C.POINTER(_p)]
    lib.ganon_ctx_destroy.argtypes = [_p]
    lib.ganon_last_error.argtypes = [_p]
    lib.ganon_last_error.restype = C.c_char_p
    lib.ganon_ctx_set_stream.argtypes = [_p, _p]
    lib.ganon_ctx_set_profiling.argtypes = [_p, C.c_int]
    lib.ganon_ctx_set_variant.argtypes = [_p, C.c_int]
    lib.ganon_ctx_set_param.argtypes = [_p, C.c_int, C.c_int]
    lib.ganon_mask_batch.argtypes = [_p, C.POINTER(GanonBatch), _u8p, _i32p, _i32p, _i64p]
    lib.ganon_batch_upload.argtypes = [_p, C.POINTER(GanonBatch), C.POINTER(_p)]
    lib.ganon_batch_upload_ref.argtypes = [_p, C.POINTER(GanonBatch), _p, C.POINTER(_p)]
    lib.ganon_batch_reload.argtypes = [_p, _p, C.POINTER(GanonBatch)]
    lib.ganon_batch_replan.argtypes = [_p, _p]
    lib.ganon_ref_upload.argtypes = [_p, _u8p, C.c_int64, C.POINTER(_p)]
    lib.ganon_ref_free.argtypes = [_p, _p]
    lib.ganon_batch_run.argtypes = [_p, _p]
    lib.ganon_batch_sync.argtypes = [_p]
    lib.ganon_batch_download.argtypes = [_p, _p, _u8p, _i32p, _i32p, _i64p]
    lib.ganon_batch_free.argtypes = [_p, _p]
    lib.ganon_batch_device_totals.argtypes = [_p, C.POINTER(_p)]
    lib.ganon_batch_copy_totals.argtypes = [_p, _p, _p]
    lib.ganon_last_kernel_times.argtypes = [_p, C.POINTER(KernelTime), C.c_int]
    lib.ganon_batch_info.argtypes = [_p, _i64p]
    lib.ganon_batch_shape.argtypes = [_p, _i64p]
    lib.ganon_batch_path_counts.argtypes = [_p, _p, _i64p]
    lib.ganon_batch_gated_runs.argtypes = [_p, _p, _i64p]
    lib.ganon_fastq_upload.argtypes = [_p, C.POINTER(GanonFastqRecords), C.POINTER(_p)]
    lib.ganon_fastq_run.argtypes = [_p, _p]
    lib.ganon_fastq_bytes.argtypes = [_p]
    lib.ganon_fastq_bytes.restype = C.c_int64
    lib.ganon_fastq_device_output.argtypes = [_p, C.POINTER(_p)]
    lib.ganon_fastq_download.argtypes = [_p, _p, C.c_void_p, C.c_int64]
    lib.ganon_pinned_alloc.argtypes = [C.c_int64, C.POINTER(_p)]
    lib.ganon_pinned_free.argtypes = [_p]
    lib.ganon_pinned_stats.argtypes = [_i64p]
    lib.ganon_fastq_download.restype = C.c_int64
    lib.ganon_fastq_free.argtypes = [_p, _p]
    lib.ganon_fastq_format_hip.restype = C.c_int64
    lib.ganon_fastq_format_hip.argtypes = [_p, C.c_int64, C.POINTER(_u8p), _u8p, _i64p, _i32p, _u8p,
                                           C.POINTER(_u8p), _u8p, _i64p, _i32p, _u8p, C.c_char_p, _i64p,
                                           _i32p, _u8p, C.c_char_p, C.c_int64]
    lib.ganon_indel_upload.argtypes = [_p, C.POINTER(GanonBatch), _p, C.POINTER(_p)]
    lib.ganon_indel_run.argtypes = [_p, _p]
    lib.ganon_indel_download.argtypes = [_p, _p, _p, C.c_int64]
    lib.ganon_indel_download.restype = C.c_int64
    lib.ganon_indel_info.argtypes = [_p, _i64p]
    lib.ganon_indel_free.argtypes = [_p, _p]
    lib.ganon_inflate.argtypes = [_p, _u8p, C.c_int64, _i64p, _i32p, _i64p, _i32p, C.c_int64, _u8p, C.c_int64,
                                  _i64p]
    lib.ganon_inflate_device_output.argtypes = [_p, C.POINTER(_p), _i64p]
    lib.ganon_bam_columns.argtypes = [_p, _p, C.c_int64, C.c_int64, C.c_int, C.POINTER(_p)]
    lib.ganon_bam_dcols_get.argtypes = [_p, C.POINTER(BamCols), _i64p]
    lib.ganon_bam_dcols_download.argtypes = [_p, _p, C.POINTER(BamCols)]
    lib.ganon_bam_dcols_free.argtypes = [_p, _p]
    if lib.ganon_abi_version() != 5:
        raise GanonError("libganon_hip.so ABI version mismatch")
    _hip = lib
    return lib


PARAM_GROUP_UNROLL = 1   # include/ganon.h GANON_PARAM_GROUP_UNROLL
PARAM_GROUP_SKIP = 2     # include/ganon.h GANON_PARAM_GROUP_SKIP (phase timing only)
PARAM_GROUP_TARGET = 3   # include/ganon.h GANON_PARAM_GROUP_TARGET (cost units per group, at upload)
PARAM_NT_COPY = 4        # include/ganon.h GANON_PARAM_NT_COPY
PARAM_REF2 = 5           # include/ganon.h GANON_PARAM_REF2
PARAM_FASTQ_SKIP = 6     # include/ganon.h GANON_PARAM_FASTQ_SKIP (phase timing only)
PARAM_FASTQ_KD = 7       # include/ganon.h GANON_PARAM_FASTQ_KD
PARAM_INDEL_SORT = 8     # include/ganon.h GANON_PARAM_INDEL_SORT (0 segmented, 1 global)
PARAM_PREP_LONG = 9      # include/ganon.h GANON_PARAM_PREP_LONG (-1 auto, 0 never, 1 always; at upload)
PARAM_GROUP_OBS = 10     # include/ganon.h GANON_PARAM_GROUP_OBS (0 auto, 512, 1024)
PARAM_PREP_UNROLL = 11   # include/ganon.h GANON_PARAM_PREP_UNROLL (0 auto, 1, 2, 4)
PARAM_FAR_INIT = 12      # include/ganon.h GANON_PARAM_FAR_INIT (first far-mask list capacity; 0 auto)
PARAM_SPEC_PLAN = 13     # include/ganon.h GANON_PARAM_SPEC_PLAN (1 speculative replans, 0 synchronous)
PARAM_FUSED_FLAT = 14    # include/ganon.h GANON_PARAM_FUSED_FLAT (1 one-segment records in the group kernel, 0 record pass)
PARAM_XREC_INIT = 15     # include/ganon.h GANON_PARAM_XREC_INIT (first extras list capacity; 0 auto)

EXPORTED_HIP_SYMBOLS = (
    "ganon_ctx_create", "ganon_ctx_destroy", "ganon_last_error", "ganon_abi_version",
    "ganon_ctx_set_stream", "ganon_ctx_set_profiling", "ganon_ctx_set_variant", "ganon_ctx_set_param", "ganon_mask_batch",
    "ganon_ref_upload", "ganon_ref_free", "ganon_batch_upload", "ganon_batch_upload_ref", "ganon_batch_reload", "ganon_batch_replan",
    "ganon_batch_run", "ganon_batch_sync", "ganon_batch_download", "ganon_batch_free",
    "ganon_batch_device_totals", "ganon_batch_copy_totals", "ganon_last_kernel_times", "ganon_batch_info",
    "ganon_batch_shape",
    "ganon_batch_path_counts", "ganon_batch_gated_runs",
    "ganon_fastq_upload", "ganon_fastq_run", "ganon_fastq_bytes", "ganon_fastq_device_output",
    "ganon_fastq_download", "ganon_fastq_free", "ganon_fastq_format_hip",
    "ganon_indel_upload", "ganon_indel_run", "ganon_indel_download", "ganon_indel_info", "ganon_indel_free",
    "ganon_inflate", "ganon_inflate_hostcb", "ganon_inflate_device_output",
    "ganon_bam_columns", "ganon_bam_dcols_get", "ganon_bam_dcols_download", "ganon_bam_dcols_free",
    "ganon_pinned_alloc", "ganon_pinned_free", "ganon_pinned_stats", "ganon_region_decode",
)
EXPORTED_HOST_SYMBOLS = (
    "ganon_bam_open", "ganon_bam_view_get", "ganon_bam_error", "ganon_bam_close",
    "ganon_host_last_error", "ganon_host_inflate_backend", "ganon_fastq_format", "ganon_pack_nt16",
    "ganon_plan_run", "ganon_plan_view_get", "ganon_plan_free", "ganon_plan_last_error", "ganon_io_replay",
    "ganon_bam_reader_open", "ganon_bam_reader_set_window", "ganon_bam_reader_has_index", "ganon_bam_reader_header",
    "ganon_bam_reader_contig", "ganon_bam_reader_region", "ganon_bam_reader_close",
    "ganon_resolver_create", "ganon_resolver_free", "ganon_resolver_contig", "ganon_resolver_pending",
    "ganon_resolver_finish", "ganon_resolver_take_log", "ganon_resolver_mark_written", "ganon_objects_pack", "ganon_blob_size", "ganon_blob_data",
    "ganon_blob_free", "ganon_objects_create", "ganon_objects_free", "ganon_objects_add_job", "ganon_objects_add_plain",
    "ganon_objects_run", "ganon_objects_take", "ganon_objects_settle", "ganon_objects_last_error",
    "ganon_objects_take_all", "ganon_aux_sa_count", "ganon_fastq_edit", "ganon_gather_ranges", "ganon_gather_ranges2", "ganon_host_phase_times",
    "ganon_bam_reader_set_inflater", "ganon_bam_reader_set_buffer_alloc", "ganon_bam_reader_set_region_decoder",
)


def _ptr(a: np.ndarray, ty):
    return a.ctypes.data_as(ty) if a is not None else None


class BamCols(C.Structure):
    """Mirror of ``ganon_bam_cols`` (include/ganon.h): device pointers, or host arrays for a download."""
    _fields_ = [("n_records", C.c_int64)] + [(f, _i32p) for f in BAM_I32_COLS] + [(f, _i64p) for f in BAM_I64_COLS] + [
        ("names", _p), ("names_bytes", C.c_int64), ("cigar", _p), ("cigar_ops", C.c_int64),
        ("seq", _p), ("seq_bytes", C.c_int64), ("qual", _p), ("qual_bytes", C.c_int64),
        ("aux", _p), ("aux_bytes", C.c_int64)]


def bam_columns_device(ctx, stream, p: int, n: int, on_host: bool) -> Tuple[Dict[str, np.ndarray], int]:
    """``ganon_bam_columns`` on context ``ctx`` (a ``ganon_ctx`` handle): the records at stream[p, n)
    decoded to columns on the device, downloaded as numpy arrays named as ``io.bam.ReadTable``'s
    (blobs: names_blob, cigar, seq, qual, aux; plus rec_off). ``stream`` is a host uint8 array
    (``on_host``) or a device address. Returns (columns, boundary fix rounds)."""
    lib = hip_lib()
    h = _p()
    if on_host:
        arr = np.ascontiguousarray(stream, np.uint8)
        addr = arr.ctypes.data
    else:
        addr = int(stream)
    rc = lib.ganon_bam_columns(ctx, _p(addr), int(p), int(n), 1 if on_host else 0, C.byref(h))
    if rc != 0:
        raise GanonError(f"ganon_bam_columns failed ({rc}): {lib.ganon_last_error(ctx).decode(errors='replace')}")
    try:
        dv = BamCols()
        fixes = C.c_int64(0)
        lib.ganon_bam_dcols_get(h, C.byref(dv), C.byref(fixes))
        nr = int(dv.n_records)
        cols: Dict[str, np.ndarray] = {}
        hv = BamCols()
        hv.n_records = nr
        for f in BAM_I32_COLS:
            cols[f] = np.empty(nr, np.int32)
            setattr(hv, f, _ptr(cols[f], _i32p))
        for f in BAM_I64_COLS:
            cols[f] = np.empty(nr, np.int64)
            setattr(hv, f, _ptr(cols[f], _i64p))
        for f, key, dt, cnt in (("names", "names_blob", np.uint8, "names_bytes"), ("cigar", "cigar", np.uint32, "cigar_ops"),
                                ("seq", "seq", np.uint8, "seq_bytes"), ("qual", "qual", np.uint8, "qual_bytes"),
                                ("aux", "aux", np.uint8, "aux_bytes")):
            cols[key] = np.empty(int(getattr(dv, cnt)), dt)
            setattr(hv, f, _p(cols[key].ctypes.data))
            setattr(hv, cnt, int(getattr(dv, cnt)))
        if lib.ganon_bam_dcols_download(ctx, h, C.byref(hv)) != 0:
            raise GanonError(f"ganon_bam_dcols_download failed: {lib.ganon_last_error(ctx).decode(errors='replace')}")
        return cols, int(fixes.value)
    finally:
        lib.ganon_bam_dcols_free(ctx, h)


class GpuInflater:
    """BGZF inflate on the GPU (``ganon_inflate``, include/ganon.h): a device
    context of its own (own stream, own grow-only buffers), used by one thread at a time — the
    BamReader decode thread hands it its block windows (``BamReader(..., inflater=)``). Windows
    of fewer than ``min_blocks`` blocks stay on the reader's host threads: the decoder is one wave
    per block (token rounds, ten blocks per CU, 2,560 in flight; a 64 KiB block takes several ms on
    its wave), so a call pays off only when it carries hundreds of blocks."""

    def __init__(self, device: int = 0, min_blocks: int = 512):
        lib = hip_lib()
        self._lib = lib
        h = _p()
        if lib.ganon_ctx_create(int(device), C.byref(h)) != 0:
            raise GanonError(f"ganon_ctx_create(device={device}) failed: no usable gfx950 device")
        self._h = h
        self.device = device
        self.min_blocks = int(min_blocks)
        self.fn = C.cast(lib.ganon_inflate_hostcb, _p)   # the reader's callback, user = the context
        self.region_fn = C.cast(lib.ganon_region_decode, _p)   # the reader's region decoder, same user

    @property
    def handle(self):
        return self._h

    def set_profiling(self, on: bool) -> None:
        self._lib.ganon_ctx_set_profiling(self._h, 1 if on else 0)

    def kernel_ms(self) -> float:
        """k_inflate's time in the last profiled inflate (HIP events on the context's stream)."""
        arr = (KernelTime * 4)()
        n = self._lib.ganon_last_kernel_times(self._h, arr, 4)
        return sum(float(arr[i].ms) for i in range(min(n, 4)) if arr[i].name == b"k_inflate")

    def inflate(self, comp: np.ndarray, in_off: np.ndarray, in_len: np.ndarray, out_len: np.ndarray) -> np.ndarray:
        """Inflate raw DEFLATE payloads comp[in_off[i]:+in_len[i]] (each to out_len[i] bytes),
        concatenated; raises GanonError naming the first bad block."""
        comp = np.ascontiguousarray(comp, np.uint8)
        in_off = np.ascontiguousarray(in_off, np.int64)
        in_len = np.ascontiguousarray(in_len, np.int32)
        out_len = np.ascontiguousarray(out_len, np.int32)
        out_off = np.zeros(len(out_len), np.int64)
        if len(out_len) > 1:
            np.cumsum(out_len[:-1], out=out_off[1:])
        total = int(out_len.sum()) if len(out_len) else 0
        out = np.empty(total, np.uint8)
        bad = np.full(1, -1, np.int64)
        rc = self._lib.ganon_inflate(self._h, _ptr(comp, _u8p), len(comp), _ptr(in_off, _i64p), _ptr(in_len, _i32p),
                                     _ptr(out_off, _i64p), _ptr(out_len, _i32p), len(out_len), _ptr(out, _u8p),
                                     total, _ptr(bad, _i64p))
        if rc != 0:
            msg = self._lib.ganon_last_error(self._h).decode(errors="replace")
            raise GanonError(f"ganon_inflate failed ({rc}, block {int(bad[0])}): {msg}")
        return out

    def device_output(self) -> Tuple[int, int]:
        """(device address, bytes) of the last inflate's output, still on the device
        (``ganon_inflate_device_output``): valid until the next ``inflate``."""
        addr, nb = _p(), C.c_int64(0)
        if self._lib.ganon_inflate_device_output(self._h, C.byref(addr), C.byref(nb)) != 0:
            raise GanonError(self._lib.ganon_last_error(self._h).decode(errors="replace"))
        return int(addr.value or 0), int(nb.value)

    def bam_columns(self, p: int, n: int) -> Tuple[Dict[str, np.ndarray], int]:
        """The BAM records at [p, n) of the last inflate's output, decoded to columns on the device
        where the inflate left them (``ganon_bam_columns``, include/ganon.h)."""
        addr, nb = self.device_output()
        if not 0 <= p <= n <= nb:
            raise GanonError(f"bam_columns: [{p}, {n}) outside the inflated {nb} bytes")
        return bam_columns_device(self._h, addr, p, n, on_host=False)

    def close(self) -> None:
        if self._h:
            self._lib.ganon_ctx_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class PinnedPool:
    """Page-locked host blocks (ganon_pinned_alloc: cached per process in libganon_hip.so) handed out
    as numpy uint8 views and given back when the last view is gone (weakref.finalize on the block):
    the device formatter's records of a job land in one by DMA — into pageable memory the runtime
    staged every byte through a host copy, ~1 CPU-second per 5 GB of FASTQ (tools/cpu_sampler.py on
    the 30x line). Sizes are rounded to 16 MiB so that blocks are reused across jobs."""

    def take(self, n: int) -> np.ndarray:
        cap = max(16 << 20, -(-n // (16 << 20)) * (16 << 20))
        ptr = _p()
        if hip_lib().ganon_pinned_alloc(cap, C.byref(ptr)) != 0 or not ptr.value:
            return np.empty(n, np.uint8)      # (no page-locked memory left: pageable)
        block = (C.c_uint8 * cap).from_address(ptr.value)
        weakref.finalize(block, PinnedPool._give_back, ptr.value)
        return np.frombuffer(block, np.uint8, count=n)

    @staticmethod
    def _give_back(addr: int) -> None:
        hip_lib().ganon_pinned_free(_p(addr))


PINNED = PinnedPool()


class HipMasker:
    """One device context (one GPU, one HIP stream) of libganon_hip.so."""

    def __init__(self, device: int = 0):
        lib = hip_lib()
        self._lib = lib
        h = _p()
        rc = lib.ganon_ctx_create(int(device), C.byref(h))
        if rc != 0:
            raise GanonError(f"ganon_ctx_create(device={device}) failed with {rc}: "
                             "no usable gfx950 device (there is no CPU fallback)")
        self._h = h
        _HIP_CONTEXTS[0] += 1
        self.device = device
        self._ref = None            # (the host array, its DeviceRef): the genome stays resident
        self._job_db = None         # the device batch of the last mask(indels=True), reloaded per job
        self.job_gen = 0            # increments with every job batch: a MaskResult's batch is live while equal

    def resident_reference(self, ref_nt16: np.ndarray) -> "DeviceRef":
        """The packed genome in HBM, uploaded once per array object (stream.py masks one contig
        batch after another against the same genome)."""
        if self._ref is None or self._ref[0] is not ref_nt16:
            if getattr(self, "_job_db", None) is not None:   # it reads the reference being replaced
                self._job_db.free()
                self._job_db = None
            if self._ref is not None:
                self._ref[1].free()
            self._ref = (ref_nt16, self.upload_reference(ref_nt16))
        return self._ref[1]

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            msg = self._lib.ganon_last_error(self._h).decode(errors="replace")
            raise GanonError(f"{what} failed ({rc}): {msg}")

    def close(self) -> None:
        if getattr(self, "_job_db", None) is not None:
            self._job_db.free()
            self._job_db = None
        if getattr(self, "_ref", None) is not None:
            self._ref[1].free()
            self._ref = None
        if getattr(self, "_h", None):
            self._lib.ganon_ctx_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, hip_stream_ptr: Optional[int]) -> None:
        self._check(self._lib.ganon_ctx_set_stream(self._h, _p(hip_stream_ptr or 0)), "set_stream")

    def set_variant(self, variant: int) -> None:
        """include/ganon.h GANON_VARIANT_*: 0 (default) or 5 (the same fused group kernel); the
        round-1 A/B kernels are retired and raise GanonError."""
        self._check(self._lib.ganon_ctx_set_variant(self._h, int(variant)), "set_variant")

    def set_param(self, param: int, value: int) -> None:
        """include/ganon.h GANON_PARAM_* tuning knob (never changes results)."""
        self._check(self._lib.ganon_ctx_set_param(self._h, int(param), int(value)), "set_param")

    def set_profiling(self, on: bool) -> None:
        self._check(self._lib.ganon_ctx_set_profiling(self._h, 1 if on else 0), "set_profiling")

    def mask(self, arrays: dict, indels: bool = False, fetch_seq: bool = True):
        """Synchronous one-shot: returns (seq_out, scope_calls, scope_bases, totals), plus the
        germline indel records (``INDEL_REC``, sorted) when ``indels``. ``fetch_seq`` False (job
        path): seq_out is None, the masked bases stay in the job batch (``job_seq``)."""
        if indels:
            # one device batch per context, reloaded job after job (grow-only buffers: no allocation
            # once the largest job has been seen); it stays valid — for formatting from the device
            # (format_fastq_batch) — until the next job
            ref = self.resident_reference(arrays["ref_nt16"])
            self.job_gen += 1
            db = self._job_db
            if db is None:
                db = self._job_db = self.upload(arrays, ref=ref)
            else:
                try:
                    db.reload(arrays)
                except GanonError:
                    self._job_db = None
                    db.free()
                    raise
            t = db.indel_tally(arrays) if db.shape()["id_ops"] else None   # (no I/D op: nothing to tally)
            try:
                db.run()
                if t is not None:
                    t.run()
                res = db.download(with_seq=fetch_seq)
                recs = t.download() if t is not None else np.zeros(0, INDEL_REC)
            finally:
                if t is not None:
                    t.free()
            return res + (recs,)
        b = make_c_batch(arrays)
        out = np.empty(b.seq_bytes, np.uint8)
        calls = np.zeros(b.n_scopes, np.int32)
        bases = np.zeros(b.n_scopes, np.int32)
        tot = np.zeros(GANON_N_TOTALS, np.int64)
        self._check(self._lib.ganon_mask_batch(self._h, C.byref(b), _ptr(out, _u8p), _ptr(calls, _i32p),
                                               _ptr(bases, _i32p), _ptr(tot, _i64p)), "ganon_mask_batch")
        return out, calls, bases, tot

    def job_seq(self, gen: int) -> np.ndarray:
        """The masked bases of job ``gen`` from the job batch (it holds only the last job's)."""
        db = self._job_db
        if db is None or gen != self.job_gen:
            raise GanonError(f"the masked bases of job {gen} are no longer on the device (job {self.job_gen} is)")
        out = np.empty(db.seq_bytes, np.uint8)
        db.download_seq(out)
        return out

    # -- device-resident path ------------------------------------------------------------
    def upload(self, arrays: dict, ref: "DeviceRef" = None) -> "DeviceBatch":
        """Copy the raw batch arrays to HBM; validation and planning run on the device. With
        ``ref`` the scopes read that resident reference (the batch's ``ref_nt16`` is ignored)."""
        b = make_c_batch(arrays, with_ref=ref is None)
        h = _p()
        if ref is None:
            self._check(self._lib.ganon_batch_upload(self._h, C.byref(b), C.byref(h)), "ganon_batch_upload")
        else:
            self._check(self._lib.ganon_batch_upload_ref(self._h, C.byref(b), ref.h, C.byref(h)),
                        "ganon_batch_upload_ref")
        return DeviceBatch(self, h, b.seq_bytes, b.n_scopes, resident_ref=ref is not None)

    def upload_reference(self, ref_nt16: np.ndarray) -> "DeviceRef":
        """ganon_ref_upload: a genome resident in HBM for every batch of this context."""
        a = np.ascontiguousarray(ref_nt16, dtype=np.uint8)
        h = _p()
        self._check(self._lib.ganon_ref_upload(self._h, a.ctypes.data_as(_u8p), len(a), C.byref(h)), "ganon_ref_upload")
        return DeviceRef(self, h, len(a))

    # -- FASTQ formatter -------------------------------------------------------------------
    def fastq_upload(self, recs: dict, seq_batch: "DeviceBatch" = None) -> "DeviceFastq":
        """Upload a record set (``fastq_records`` layout); with ``seq_batch`` the sequences are
        read from that device batch (buffer 0 = masked output, 1 = input) without a copy."""
        c, keep = _c_fastq_records(recs, seq_batch)
        h = _p()
        self._check(self._lib.ganon_fastq_upload(self._h, C.byref(c), C.byref(h)), "ganon_fastq_upload")
        del keep
        return DeviceFastq(self, h)

    def format_fastq_batch(self, recs: dict, gen: int) -> Optional[bytes]:
        """Format records whose sequences are in the last job batch (``recs`` as FastqFormatter
        builds them: buffer 0 = that batch's masked output, 1 / 2 = the tumor / normal blobs, which
        are the batch's input at offsets 0 / ``recs['seq_base1']``), reading the bases in place on
        the device: no upload of the sequences. None when the batch is no longer job ``gen``'s."""
        db = self._job_db
        if db is None or gen != self.job_gen:
            return None
        r = dict(recs)
        sel = recs["seq_sel"]
        r["seq_nib_off"] = recs["seq_nib_off"] + np.where(sel == 2, 2 * int(recs["seq_base1"]), 0).astype(np.int64)
        r["seq_sel"] = np.minimum(sel, 1).astype(np.uint8)
        t0 = time.perf_counter()
        c, keep = _c_fastq_records(r, seq_batch=db)
        h = _p()
        self._check(self._lib.ganon_fastq_upload(self._h, C.byref(c), C.byref(h)), "ganon_fastq_upload")
        del keep
        try:
            t1 = time.perf_counter()
            self._check(self._lib.ganon_fastq_run(self._h, h), "ganon_fastq_run")
            n_bytes = int(self._lib.ganon_fastq_bytes(h))
            # page-locked: the records come down by DMA (a numpy view; the job's pre-formatted blob)
            out = PINNED.take(n_bytes) if n_bytes >= (8 << 20) else _new_bytes(None, n_bytes)
            t2 = time.perf_counter()
            w = self._lib.ganon_fastq_download(self._h, h, _addr(out), n_bytes)
            w = _fastq_result(w, lambda: self._lib.ganon_last_error(self._h).decode(errors="replace"))
            t3 = time.perf_counter()
            FQ_TIMES["upload_s"] += t1 - t0   # (where a job's formatting goes: the stream's timing)
            FQ_TIMES["run_s"] += t2 - t1
            FQ_TIMES["download_s"] += t3 - t2
            FQ_TIMES["bytes"] += n_bytes
        finally:
            self._lib.ganon_fastq_free(self._h, h)
        return out if w == n_bytes else out[:w]

    def format_fastq(self, recs: dict) -> bytes:
        """One-shot ``ganon_fastq_format_hip`` (the host formatter's arguments)."""
        a = _fastq_args(recs)
        n_bytes = fastq_bytes(recs)
        out = _new_bytes(None, n_bytes)    # filled in place: no zero-fill, no copy out
        w = self._lib.ganon_fastq_format_hip(self._h, *a, out, n_bytes)
        w = _fastq_result(w, lambda: self._lib.ganon_last_error(self._h).decode(errors="replace"))
        return out if w == n_bytes else out[:w]


class FastqBadRecord(GanonError):
    """A reverse read with a base outside ACGTN (the reference's KeyError)."""

    def __init__(self, index: int, msg: str):
        super().__init__(msg)
        self.index = index


FASTQ_FAILED = -(1 << 63) + 1   # include/ganon.h GANON_FASTQ_FAILED

# per process: the device formatter's record upload, run (kernels + sync) and download of the bytes
FQ_TIMES = {"upload_s": 0.0, "run_s": 0.0, "download_s": 0.0, "bytes": 0}


def _fastq_result(w: int, err) -> int:
    if w >= 0:
        return w
    if w == -(1 << 63):
        raise GanonError("FASTQ output buffer too small")
    if w == FASTQ_FAILED:
        raise GanonError(f"FASTQ formatter failed: {err()}")
    raise FastqBadRecord(-w - 1, f"record {-w - 1}: reverse read with a base outside ACGTN (SURVEY Q7)")


FASTQ_ARRAYS = {"seq_sel": np.uint8, "seq_nib_off": np.int64, "seq_len": np.int32, "reverse": np.uint8,
                "qual_sel": np.uint8, "qual_off": np.int64, "qual_len": np.int32, "qual_rev": np.uint8,
                "name_off": np.int64, "name_len": np.int32, "mate": np.uint8}


def fastq_bytes(recs: dict) -> int:
    return int(8 * len(recs["seq_len"]) + recs["name_len"].sum(dtype=np.int64) +
               recs["seq_len"].sum(dtype=np.int64) + recs["qual_len"].sum(dtype=np.int64))


def _check_fastq(recs: dict) -> None:
    for k, dt in FASTQ_ARRAYS.items():
        a = recs[k]
        if a.dtype != dt or not a.flags["C_CONTIGUOUS"]:
            raise GanonError(f"FASTQ record array {k} must be C-contiguous {np.dtype(dt)}")


def _names_ptr(names):
    """The names blob (bytes or a uint8 array) as the formatter's char pointer, without a copy."""
    if isinstance(names, np.ndarray) and names.dtype == np.uint8 and names.flags["C_CONTIGUOUS"]:
        return C.cast(_addr(names), C.c_char_p)    # (alive in the caller's record dict)
    return names if isinstance(names, bytes) else bytes(names)


def _fastq_args(recs: dict) -> tuple:
    """The host formatter's argument list (minus out/cap) over a ``fastq_records`` dict."""
    _check_fastq(recs)
    seq_ptrs = (_u8p * len(recs["seq_bufs"]))(*[b.ctypes.data_as(_u8p) for b in recs["seq_bufs"]])
    qual_ptrs = (_u8p * len(recs["qual_bufs"]))(*[b.ctypes.data_as(_u8p) for b in recs["qual_bufs"]])
    P = lambda k, t: recs[k].ctypes.data_as(t)
    return (len(recs["seq_len"]), seq_ptrs, P("seq_sel", _u8p), P("seq_nib_off", _i64p), P("seq_len", _i32p),
            P("reverse", _u8p), qual_ptrs, P("qual_sel", _u8p), P("qual_off", _i64p), P("qual_len", _i32p),
            P("qual_rev", _u8p), _names_ptr(recs["names"]), P("name_off", _i64p), P("name_len", _i32p),
            P("mate", _u8p))


def _c_fastq_records(recs: dict, seq_batch=None):
    _check_fastq(recs)
    c = GanonFastqRecords()
    c.n = len(recs["seq_len"])
    nsb = 2 if seq_batch is not None else len(recs["seq_bufs"])
    c.n_seq_bufs, c.n_qual_bufs = nsb, len(recs["qual_bufs"])
    keep = []
    if seq_batch is None:
        sp = (_u8p * nsb)(*[b.ctypes.data_as(_u8p) for b in recs["seq_bufs"]])
        keep.append(sp)
        c.seq_buf = sp
    else:
        c.seq_batch = seq_batch.h
    qp = (_u8p * len(recs["qual_bufs"]))(*[b.ctypes.data_as(_u8p) for b in recs["qual_bufs"]])
    keep.append(qp)
    c.qual_buf = qp
    names = recs["names"]
    if not isinstance(names, (bytes, np.ndarray)):
        names = bytes(names)
    keep.append(names)
    c.names = C.cast(_addr(names), C.c_char_p)     # (in place: a job's names blob is not copied)
    for k, dt in FASTQ_ARRAYS.items():
        setattr(c, k, recs[k].ctypes.data_as(_PTR_OF[dt]))
    return c, keep


def host_format_fastq(recs: dict) -> bytes:
    """libganon_host.so ganon_fastq_format over a ``fastq_records`` dict (same contract)."""
    a = _fastq_args(recs)
    n_bytes = fastq_bytes(recs)
    out = _new_bytes(None, n_bytes)
    w = _fastq_result(host_lib().ganon_fastq_format(*a, out, n_bytes), lambda: "host formatter")
    return out if w == n_bytes else out[:w]


def _addr(buf) -> int:
    """Address of a bytes object's, a ctypes array's or a contiguous numpy array's data."""
    if isinstance(buf, np.ndarray):
        return buf.ctypes.data
    if isinstance(buf, C.Array):
        return C.addressof(buf)
    return C.cast(C.c_char_p(buf), C.c_void_p).value or 0


def gather_ranges(src, off: np.ndarray, length: np.ndarray) -> bytes:
    """libganon_host.so ganon_gather_ranges: src[off[i]:off[i] + length[i]] back to back (src: bytes or a
    uint8 array)."""
    off = np.ascontiguousarray(off, np.int64)
    length = np.ascontiguousarray(length, np.int64)
    total = int(length.sum())
    out = _new_bytes(None, total)      # a fresh, unshared bytes object the library fills in place
    w = host_lib().ganon_gather_ranges(_addr(src), len(src), len(off), off.ctypes.data_as(_i64p),
                                       length.ctypes.data_as(_i64p), out, total)
    if w != total:
        raise GanonError("gather_ranges: range outside the source")
    return out


def gather_ranges2(src0, src1, sel: np.ndarray, off: np.ndarray, length: np.ndarray) -> bytes:
    """libganon_host.so ganon_gather_ranges2: range i from src0 (sel 0) or src1 (sel 1), back to back."""
    sel = np.ascontiguousarray(sel, np.uint8)
    off = np.ascontiguousarray(off, np.int64)
    length = np.ascontiguousarray(length, np.int64)
    total = int(length.sum())
    out = _new_bytes(None, total)
    w = host_lib().ganon_gather_ranges2(_addr(src0), len(src0), _addr(src1), len(src1), len(off), sel.ctypes.data_as(_u8p),
                                        off.ctypes.data_as(_i64p), length.ctypes.data_as(_i64p), out, total)
    if w != total:
        raise GanonError("gather_ranges2: bad selector or range outside its source")
    return out


# (then two counts: region reads the device decoder finished, and those it handed back to the host)
DECODE_PHASES = ("parse", "inflate", "region_walk", "kept_copy", "record_walk", "sizes", "columns", "device_region",
                 "read", "device_region_cpu", "device_regions", "device_fallbacks")


def pinned_stats() -> dict:
    """ganon_pinned_stats: the process's page-locked blocks pinned anew (count, bytes, seconds) and
    the requests its cache served (an empty dict without the HIP library loaded)."""
    if _hip is None:
        return {}
    out = np.zeros(4, np.int64)
    hip_lib().ganon_pinned_stats(_ptr(out, _i64p))
    return {"new_blocks": int(out[0]), "new_bytes": int(out[1]), "pin_s": round(out[2] * 1e-9, 4),
            "cache_hits": int(out[3])}


def decode_phase_times(reset: bool = False) -> dict:
    """ganon_host_phase_times: seconds the BAM readers' calling threads spent per decode phase."""
    out = (C.c_double * 16)()
    n = host_lib().ganon_host_phase_times(out, 16, int(reset))
    return {DECODE_PHASES[i] if i < len(DECODE_PHASES) else f"p{i}": round(out[i], 4) for i in range(min(n, 16))}


class FastqEditError(GanonError):
    """ganon_fastq_edit refused record ``index``: code 1 = reverse read with a base outside ACGTN
    (SURVEY Q7), 2 = sequence/quality lengths diverge, 3 = DEL on a read without qualities."""

    def __init__(self, code: int, index: int):
        super().__init__(f"record {index}: left-over edit failed (code {code})")
        self.code, self.index = code, index


def fastq_edit(recs: bytes, rec_off: np.ndarray, reverse: np.ndarray, times: np.ndarray, edit_off: np.ndarray,
               edits: np.ndarray, alleles: bytes, allele_off: np.ndarray, cap: int) -> Tuple[bytes, np.ndarray]:
    """libganon_host.so ganon_fastq_edit: the indel left-overs applied to unedited records (host
    side of row A4). Returns (edited records back to back, per-record lengths)."""
    n = len(reverse)
    rec_off = np.ascontiguousarray(rec_off, np.int64)
    reverse = np.ascontiguousarray(reverse, np.uint8)
    times = np.ascontiguousarray(times, np.int32)
    edit_off = np.ascontiguousarray(edit_off, np.int64)
    edits = np.ascontiguousarray(edits, np.int64).reshape(-1)
    allele_off = np.ascontiguousarray(allele_off, np.int64)
    if len(rec_off) != n + 1 or len(edit_off) != n + 1 or len(edits) != 3 * int(edit_off[-1]) or \
            len(allele_off) != int(edit_off[-1]) + 1:
        raise GanonError("fastq_edit: inconsistent array sizes")
    out = C.create_string_buffer(max(int(cap), 1))
    out_len = np.zeros(n, np.int64)
    bad = C.c_int64(-1)
    P = lambda a, t: a.ctypes.data_as(t)
    rc = host_lib().ganon_fastq_edit(n, recs, P(rec_off, _i64p), P(reverse, _u8p), P(times, _i32p),
                                     P(edit_off, _i64p), P(edits, _i64p), alleles, P(allele_off, _i64p),
                                     C.cast(out, _p), int(cap), P(out_len, _i64p), C.byref(bad))
    if rc > 0:
        raise FastqEditError(rc, int(bad.value))
    if rc < 0:
        raise GanonError("fastq_edit: output too small" if rc == -2 else "fastq_edit: bad arguments")
    return out.raw[:int(out_len.sum())], out_len


class DeviceFastq:
    """A record set resident on the device (ganon_fastq_upload)."""

    def __init__(self, masker: HipMasker, handle):
        self.m = masker
        self.h = handle
        self.n_bytes = int(masker._lib.ganon_fastq_bytes(handle))

    def run(self) -> None:
        self.m._check(self.m._lib.ganon_fastq_run(self.m._h, self.h), "ganon_fastq_run")

    def sync(self) -> None:
        self.m._check(self.m._lib.ganon_batch_sync(self.m._h), "ganon_batch_sync")

    def device_output_ptr(self) -> int:
        p = _p()
        self.m._check(self.m._lib.ganon_fastq_device_output(self.h, C.byref(p)), "fastq_device_output")
        return p.value

    def download(self) -> bytes:
        out = C.create_string_buffer(max(self.n_bytes, 1))
        w = self.m._lib.ganon_fastq_download(self.m._h, self.h, _addr(out), self.n_bytes)
        return out.raw[:_fastq_result(w, lambda: self.m._lib.ganon_last_error(self.m._h).decode(errors="replace"))]

    def kernel_times(self) -> list:
        arr = (KernelTime * 32)()
        n = self.m._lib.ganon_last_kernel_times(self.m._h, arr, 32)
        return [(arr[i].name.decode(), int(arr[i].launches), float(arr[i].ms)) for i in range(min(n, 32))]

    def free(self) -> None:
        if self.h:
            self.m._lib.ganon_fastq_free(self.m._h, self.h)
            self.h = None


class DeviceRef:
    """A reference genome resident on the device (ganon_ref_upload)."""

    def __init__(self, masker: HipMasker, handle, n_bytes: int):
        self.m = masker
        self.h = handle
        self.n_bytes = n_bytes

    def free(self) -> None:
        if self.h:
            self.m._lib.ganon_ref_free(self.m._h, self.h)
            self.h = None


class DeviceBatch:
    def __init__(self, masker: HipMasker, handle, seq_bytes: int, n_scopes: int, resident_ref: bool = False):
        self.m = masker
        self.h = handle
        self.seq_bytes = seq_bytes
        self.n_scopes = n_scopes
        self.resident_ref = resident_ref

    def reload(self, arrays: dict) -> None:
        """ganon_batch_reload: replace the contents with another host batch (device buffers reused)."""
        b = make_c_batch(arrays, with_ref=not self.resident_ref)
        self.m._check(self.m._lib.ganon_batch_reload(self.m._h, self.h, C.byref(b)), "ganon_batch_reload")
        self.seq_bytes = b.seq_bytes
        self.n_scopes = b.n_scopes

    def replan(self) -> None:
        """ganon_batch_replan: plan the device arrays again exactly as a fresh upload would
        (validation scan, prep mode, sizes; speculative — no synchronization — when the previous
        plan's one-segment shape still applies; errors then come from download)."""
        self.m._check(self.m._lib.ganon_batch_replan(self.m._h, self.h), "ganon_batch_replan")

    def run(self) -> None:
        self.m._check(self.m._lib.ganon_batch_run(self.m._h, self.h), "ganon_batch_run")

    def sync(self) -> None:
        self.m._check(self.m._lib.ganon_batch_sync(self.m._h), "ganon_batch_sync")

    def download(self, with_seq: bool = True):
        """(masked bases or None, per-scope calls, per-scope bases, totals)."""
        out = np.empty(self.seq_bytes, np.uint8) if with_seq else None
        calls = np.zeros(self.n_scopes, np.int32)
        bases = np.zeros(self.n_scopes, np.int32)
        tot = np.zeros(GANON_N_TOTALS, np.int64)
        self.m._check(self.m._lib.ganon_batch_download(self.m._h, self.h, _ptr(out, _u8p) if with_seq else None,
                                                       _ptr(calls, _i32p), _ptr(bases, _i32p), _ptr(tot, _i64p)),
                      "download")
        return out, calls, bases, tot

    def download_seq(self, out: np.ndarray) -> None:
        """The masked bases into ``out`` (uint8, seq_bytes long; pinned memory for full PCIe rate)."""
        if out.dtype != np.uint8 or len(out) < self.seq_bytes or not out.flags["C_CONTIGUOUS"]:
            raise GanonError("download_seq: need a C-contiguous uint8 buffer of seq_bytes")
        self.m._check(self.m._lib.ganon_batch_download(self.m._h, self.h, _ptr(out, _u8p), None, None, None),
                      "download")

    def totals(self) -> np.ndarray:
        tot = np.zeros(GANON_N_TOTALS, np.int64)
        self.m._check(self.m._lib.ganon_batch_download(self.m._h, self.h, None, None, None, _ptr(tot, _i64p)),
                      "download totals")
        return tot

    def copy_totals_to(self, dev_ptr: int) -> None:
        self.m._check(self.m._lib.ganon_batch_copy_totals(self.m._h, self.h, _p(dev_ptr)), "copy_totals")

    def device_totals_ptr(self) -> int:
        p = _p()
        self.m._check(self.m._lib.ganon_batch_device_totals(self.h, C.byref(p)), "device_totals")
        return p.value

    def info(self) -> dict:
        a = np.zeros(8, np.int64)
        self.m._check(self.m._lib.ganon_batch_info(self.h, _ptr(a, _i64p)), "batch_info")
        keys = ("groups", "segments", "huge_scopes", "huge_tiles", "far_capacity", "huge_written_reads",
                "overflow_region", "written_reads")
        return dict(zip(keys, a.tolist()))

    def shape(self) -> dict:
        """ganon_batch_shape: what the device scan of the last plan found."""
        a = np.zeros(4, np.int64)
        self.m._check(self.m._lib.ganon_batch_shape(self.h, _ptr(a, _i64p)), "batch_shape")
        return {"id_ops": int(a[0]), "max_len": int(a[1]), "max_seg": int(a[2]),
                "prep_mode": ("two_pass", "long_read", "one_segment", "one_segment_fused",
                              "multi_segment_fused")[int(a[3])]}

    def kernel_times(self) -> list:
        arr = (KernelTime * 32)()
        n = self.m._lib.ganon_last_kernel_times(self.m._h, arr, 32)
        return [(arr[i].name.decode(), int(arr[i].launches), float(arr[i].ms)) for i in range(min(n, 32))]

    def path_counts(self) -> dict:
        """ganon_batch_path_counts: the group kernel's rarer paths taken since upload."""
        a = np.zeros(4, np.int64)
        self.m._check(self.m._lib.ganon_batch_path_counts(self.m._h, self.h, _ptr(a, _i64p)), "path_counts")
        return {"sorted_lists": int(a[0]), "overflowing_lists": int(a[1]), "key_range_splits": int(a[2]),
                "filtered_into_lds": int(a[3])}

    def gated_runs(self) -> int:
        """ganon_batch_gated_runs: runs since upload whose speculative plan the batch did not fit
        (they ran nothing; the download planned and ran the batch in full)."""
        a = np.zeros(1, np.int64)
        self.m._check(self.m._lib.ganon_batch_gated_runs(self.m._h, self.h, _ptr(a, _i64p)), "gated_runs")
        return int(a[0])

    def indel_tally(self, arrays: dict) -> "DeviceIndels":
        """Plan the germline indel tally of this batch (``arrays`` = the batch it was uploaded from)."""
        iv = indel_view(arrays)
        b = make_c_batch(iv)
        h = _p()
        self.m._check(self.m._lib.ganon_indel_upload(self.m._h, C.byref(b), self.h, C.byref(h)), "ganon_indel_upload")
        return DeviceIndels(self.m, h)

    def free(self) -> None:
        if self.h:
            self.m._lib.ganon_batch_free(self.m._h, self.h)
            self.h = None


class DeviceIndels:
    """ganon_indel_* handle: observation emission, sort and classification on the device."""

    def __init__(self, masker: HipMasker, handle):
        self.m = masker
        self.h = handle

    def run(self) -> None:
        self.m._check(self.m._lib.ganon_indel_run(self.m._h, self.h), "ganon_indel_run")

    def download(self) -> np.ndarray:
        lib = self.m._lib
        n = lib.ganon_indel_download(self.m._h, self.h, None, 0)
        if n < 0:
            self.m._check(int(n), "ganon_indel_download")
        out = np.zeros(n, INDEL_REC)
        if n:
            w = lib.ganon_indel_download(self.m._h, self.h, out.ctypes.data_as(_p), n)
            if w != n:
                self.m._check(int(w) if w < 0 else -4, "ganon_indel_download")
        return indel_records_array(out)

    def info(self) -> dict:
        a = np.zeros(8, np.int64)
        self.m._check(self.m._lib.ganon_indel_info(self.h, _ptr(a, _i64p)), "ganon_indel_info")
        return dict(zip(("observations", "incidences", "key_bits", "records", "emitted", "reads", "global_sort"),
                        a.tolist()))

    def free(self) -> None:
        if self.h:
            self.m._lib.ganon_indel_free(self.m._h, self.h)
            self.h = None


# ---- host library ---------------------------------------------------------------------

class BamView(C.Structure):
    _fields_ = [
        ("n_records", C.c_int64), ("n_ref", C.c_int32), ("ref_names", _p),
        ("ref_name_off", _i64p), ("ref_len", _i64p),
        ("tid", _i32p), ("pos", _i32p), ("end", _i32p), ("flag", _i32p), ("mapq", _i32p),
        ("l_seq", _i32p), ("n_cigar", _i32p), ("mate_tid", _i32p), ("mate_pos", _i32p), ("tlen", _i32p),
        ("name_off", _i64p), ("name_len", _i32p), ("cig_off", _i64p), ("seq_off", _i64p),
        ("qual_off", _i64p), ("aux_off", _i64p), ("aux_len", _i32p),
        ("names", _p), ("names_bytes", C.c_int64), ("cigar", _u32p), ("cigar_ops", C.c_int64),
        ("seq", _u8p), ("seq_bytes", C.c_int64), ("qual", _u8p), ("qual_bytes", C.c_int64),
        ("aux", _u8p), ("aux_bytes", C.c_int64),
    ]


class PlanTable(C.Structure):
    """Mirror of ``ganon_plan_table`` (include/ganon_host.h)."""
    _fields_ = [("n", C.c_int64), ("tid", _i32p), ("pos", _i32p), ("end", _i32p), ("flag", _i32p),
                ("l_seq", _i32p), ("n_cigar", _i32p), ("names", _p), ("name_off", _i64p), ("name_len", _i32p),
                ("n_ref", C.c_int32), ("ref_len", _i64p), ("tid_of_contig", _i32p), ("mate_tid", _i32p),
                ("mate_pos", _i32p), ("n_sa", _i32p)]


class PlanInput(C.Structure):
    _fields_ = [("tables", PlanTable * 2), ("n_contigs", C.c_int32), ("contig_len", _i64p),
                ("contig_names", _p), ("contig_name_off", _i64p), ("n_windows", C.c_int32),
                ("win_contig", _i32p), ("win_first", _i64p), ("win_last", _i64p),
                ("contig_mode", C.c_int32), ("only_contig", C.c_int32), ("n_force", C.c_int64),
                ("force_names", _p), ("force_off", _i64p), ("force_len", _i32p),
                ("sec_lo", C.c_int32), ("sec_hi", C.c_int32), ("reg_lo", C.c_int64), ("reg_hi", C.c_int64)]


class PlanView(C.Structure):
    _fields_ = [("n_scopes", C.c_int32), ("scope_contig", _i32p), ("scope_window", _i32p),
                ("scope_first", _i64p), ("scope_last", _i64p), ("scope_span_start", _i64p),
                ("scope_span_end", _i64p), ("scope_t_off", _i64p), ("scope_n_off", _i64p),
                ("t_rows", _i64p), ("n_rows", _i64p), ("n_events", C.c_int64), ("events", _i32p),
                ("event_rows", _i64p), ("n_stats", C.c_int64), ("stats", _i32p),
                ("n_single", C.c_int64 * 2), ("single", _i64p * 2), ("write_single_end", C.c_int32),
                ("n_left", C.c_int64), ("left", _i64p), ("n_cand", C.c_int64), ("cand", _i64p),
                ("n_objs", C.c_int64), ("objs", _i64p), ("n_obj_rows", C.c_int64), ("obj_rows", _i64p),
                ("n_skip", C.c_int64), ("skip", _i64p)]


PLAN_E_VALUE, PLAN_E_TYPE, PLAN_E_UNSUPPORTED, PLAN_E_INDEX = -10, -11, -12, -13


def _np_copy(ptr, n: int, dtype) -> np.ndarray:
    if n <= 0:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(ptr, shape=(int(n),)).astype(dtype, copy=True)


def plan_sample(tables, contig_names, contig_lens, win_contig, win_first, win_last, only_contig=None,
                force_names=(), job=None) -> dict:
    """``ganon_plan_run`` over two ReadTables (io/bam.py) and the variant windows. Returns the
    plan's column arrays (copies); raises ValueError / TypeError / planner.UnsupportedInput as
    the reference's own code would (message from the library). ``only_contig``: contig mode for
    that FASTA contig (tables holding its records only), see include/ganon_host.h; ``force_names``
    (bytes): names planned as cross names there (``ganon_plan_input.force_names``); ``job``:
    (first section, end section, region start, region end) of job mode (``ganon_plan_input.sec_lo``)."""
    lib = host_lib()
    keep = []

    def arr(a, dt):
        a = np.ascontiguousarray(a, dtype=dt)
        keep.append(a)
        return a.ctypes.data_as(_PTR_OF[dt])

    inp = PlanInput()
    for d, t in enumerate(tables):
        pt = inp.tables[d]
        pt.n = t.n
        for f in ("tid", "pos", "end", "flag", "l_seq", "n_cigar"):
            setattr(pt, f, arr(getattr(t, f), np.int32))
        nb = np.ascontiguousarray(t.names_blob)
        keep.append(nb)
        pt.names = nb.ctypes.data_as(_p)
        pt.name_off = arr(t.name_off, np.int64)
        pt.name_len = arr(t.name_len, np.int32)
        pt.n_ref = len(t.ref_names)
        pt.ref_len = arr(t.ref_lens, np.int64)
        idx = {nm: i for i, nm in enumerate(t.ref_names)}
        pt.tid_of_contig = arr([idx.get(c, -1) for c in contig_names], np.int32)
        pt.mate_tid = arr(t.mate_tid, np.int32)
        pt.mate_pos = arr(t.mate_pos, np.int32)
        if only_contig is not None or t.may_be_complex():
            pt.n_sa = arr(t.sa_count(), np.int32)
    inp.n_contigs = len(contig_names)
    inp.contig_len = arr(contig_lens, np.int64)
    blob = b"".join(c.encode() + b"\0" for c in contig_names) or b"\0"
    cb = np.frombuffer(blob, np.uint8).copy()
    keep.append(cb)
    inp.contig_names = cb.ctypes.data_as(_p)
    offs = np.cumsum([0] + [len(c.encode()) + 1 for c in contig_names])[:-1] if contig_names else [0]
    inp.contig_name_off = arr(offs, np.int64)
    inp.n_windows = len(win_contig)
    inp.win_contig = arr(win_contig, np.int32)
    inp.win_first = arr(win_first, np.int64)
    inp.win_last = arr(win_last, np.int64)
    inp.contig_mode = 0 if only_contig is None else 1
    inp.only_contig = -1 if only_contig is None else int(only_contig)
    inp.sec_lo, inp.sec_hi, inp.reg_lo, inp.reg_hi = (-1, -1, 0, 0) if job is None else tuple(int(x) for x in job)
    force_names = list(force_names)
    if force_names:
        inp.n_force = len(force_names)
        inp.force_names, inp.force_off, inp.force_len = _names_args(force_names, keep)
    h = _p()
    rc = lib.ganon_plan_run(C.byref(inp), C.byref(h))
    if rc != 0:
        msg = lib.ganon_plan_last_error().decode(errors="replace")
        if rc == PLAN_E_VALUE:
            raise ValueError(msg)
        if rc == PLAN_E_TYPE:
            raise TypeError(msg)
        if rc == PLAN_E_UNSUPPORTED:
            from .planner import UnsupportedInput
            raise UnsupportedInput(msg)
        raise GanonError(f"ganon_plan_run failed ({rc}): {msg}")
    try:
        v = PlanView()
        lib.ganon_plan_view_get(h, C.byref(v))
        ns = int(v.n_scopes)
        out = {
            "scope_contig": _np_copy(v.scope_contig, ns, np.int32),
            "scope_window": _np_copy(v.scope_window, ns, np.int32),
            "scope_first": _np_copy(v.scope_first, ns, np.int64),
            "scope_last": _np_copy(v.scope_last, ns, np.int64),
            "scope_span_start": _np_copy(v.scope_span_start, ns, np.int64),
            "scope_span_end": _np_copy(v.scope_span_end, ns, np.int64),
            "scope_t_off": _np_copy(v.scope_t_off, ns + 1, np.int64),
            "scope_n_off": _np_copy(v.scope_n_off, ns + 1, np.int64),
        }
        out["t_rows"] = _np_copy(v.t_rows, int(out["scope_t_off"][-1]), np.int64)
        out["n_rows"] = _np_copy(v.n_rows, int(out["scope_n_off"][-1]), np.int64)
        ne = int(v.n_events)
        out["events"] = _np_copy(v.events, 7 * ne, np.int32).reshape(ne, 7)
        out["event_rows"] = _np_copy(v.event_rows, ne, np.int64)
        out["stats"] = _np_copy(v.stats, 2 * int(v.n_stats), np.int32).reshape(-1, 2)
        out["single"] = [_np_copy(v.single[d], 3 * int(v.n_single[d]), np.int64).reshape(-1, 3) for d in (0, 1)]
        out["write_single_end"] = bool(v.write_single_end)
        out["left"] = _np_copy(v.left, 11 * int(v.n_left), np.int64).reshape(-1, 11)
        out["cand"] = _np_copy(v.cand, 6 * int(v.n_cand), np.int64).reshape(-1, 6)
        out["objs"] = _np_copy(v.objs, 10 * int(v.n_objs), np.int64).reshape(-1, 10)
        out["obj_rows"] = _np_copy(v.obj_rows, int(v.n_obj_rows), np.int64)
        out["skip"] = _np_copy(v.skip, 3 * int(v.n_skip), np.int64).reshape(-1, 3)
    finally:
        lib.ganon_plan_free(h)
    return out


def _names_args(names: list, keep: list):
    """(blob, offsets, lengths) ctypes arguments of a list of bytes names."""
    lens = np.array([len(x) for x in names], np.int32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.int64)]).astype(np.int64) if len(names) else np.zeros(1, np.int64)
    blob = np.frombuffer(b"".join(names) + b"\0", np.uint8).copy()
    lens = lens if len(names) else np.zeros(1, np.int32)
    keep += [blob, offs, lens]
    return blob.ctypes.data_as(_p), offs.ctypes.data_as(_i64p), lens.ctypes.data_as(_i32p)


class Resolver:
    """``ganon_resolver_*`` (include/ganon_host.h): the sample-wide pairing state across contig
    plans. Writes come back as int64 rows (file dataset, file slot, job, dataset, scope, row)."""

    def __init__(self):
        self._lib = host_lib()
        h = _p()
        if self._lib.ganon_resolver_create(C.byref(h)) != 0:
            raise GanonError("ganon_resolver_create failed")
        self._h = h

    def _err(self, rc: int):
        msg = self._lib.ganon_plan_last_error().decode(errors="replace")
        if rc == PLAN_E_VALUE:
            raise ValueError(msg)
        if rc == PLAN_E_TYPE:
            raise TypeError(msg)
        raise GanonError(f"resolver failed ({rc}): {msg}")

    def contig(self, job: int, ops: np.ndarray, op_rows: np.ndarray, op_names: list, left: np.ndarray,
               left_names: list, objs: np.ndarray = None, obj_rows: np.ndarray = None, obj_ids: np.ndarray = None):
        """Returns (n_writes per op, writes [n_ops, 2, 7]); ``objs``/``obj_rows``: the plan's
        objects of complex names (their log: ``take_log``)."""
        keep = []
        ops = np.ascontiguousarray(ops, np.int32).reshape(-1, 7)
        rows = np.ascontiguousarray(op_rows, np.int64)
        left = np.ascontiguousarray(left, np.int64).reshape(-1, 11)
        objs = np.ascontiguousarray(np.zeros((0, 10), np.int64) if objs is None else objs, np.int64).reshape(-1, 10)
        obj_rows = np.ascontiguousarray(np.zeros(0, np.int64) if obj_rows is None else obj_rows, np.int64)
        ids = None if obj_ids is None else np.ascontiguousarray(obj_ids, np.int64)
        if ids is not None and len(ids) != len(obj_rows):
            raise ValueError("obj_ids: one per obj_rows entry")
        keep += [objs, obj_rows, ids]
        n = len(ops)
        out_n = np.zeros(max(n, 1), np.int32)
        out_w = np.zeros((max(n, 1), 2, 7), np.int64)
        on, oo, ol = _names_args(op_names, keep)
        ln, lo, ll = _names_args(left_names, keep)
        rc = self._lib.ganon_resolver_contig(self._h, int(job), n, ops.ctypes.data_as(_i32p), rows.ctypes.data_as(_i64p),
                                             on, oo, ol, len(left), left.ctypes.data_as(_i64p), ln, lo, ll,
                                             len(objs), objs.ctypes.data_as(_i64p), obj_rows.ctypes.data_as(_i64p),
                                             None if ids is None or not len(ids) else ids.ctypes.data_as(_i64p),
                                             out_n.ctypes.data_as(_i32p), out_w.ctypes.data_as(_i64p))
        if rc != 0:
            self._err(rc)
        return out_n[:n], out_w[:n]

    def mark_written(self, names: list) -> int:
        """``ganon_resolver_mark_written``: the names it has no state for count as written (their
        contig planned them locally and wrote them); returns how many were marked."""
        if not names:
            return 0
        keep = []
        nb, no, nl = _names_args(list(names), keep)
        rc = self._lib.ganon_resolver_mark_written(self._h, len(names), nb, no, nl)
        if rc < 0:
            self._err(rc)
        return int(rc)

    def take_log(self) -> np.ndarray:
        """The object log entries made since the last call ([n, 8] int64, include/ganon_host.h)."""
        n = self._lib.ganon_resolver_take_log(self._h, None, 0)
        out = np.zeros((max(n, 1), 8), np.int64)
        self._lib.ganon_resolver_take_log(self._h, out.ctypes.data_as(_i64p), n)
        return out[:n]

    def pending(self) -> np.ndarray:
        k = self._lib.ganon_resolver_pending(self._h, None, 0)
        out = np.zeros((max(k, 1), 4), np.int64)
        self._lib.ganon_resolver_pending(self._h, out.ctypes.data_as(_i64p), k)
        return out[:k]

    def finish(self, cand: np.ndarray, names: list):
        """Returns (tail writes [n, 7], single ends per dataset [m, 5] (job, ds, scope, row,
        reapply), write_single_end)."""
        keep = []
        cand = np.ascontiguousarray(cand, np.int64).reshape(-1, 8)
        n_pend = self._lib.ganon_resolver_pending(self._h, None, 0)
        tail = np.zeros((max(2 * len(cand), 1), 7), np.int64)
        s0 = np.zeros((max(n_pend, 1), 5), np.int64)
        s1 = np.zeros((max(n_pend, 1), 5), np.int64)
        n_tail = C.c_int64(0)
        n_single = np.zeros(2, np.int64)
        wse = C.c_int32(0)
        nb, no, nl = _names_args(names, keep)
        rc = self._lib.ganon_resolver_finish(self._h, len(cand), cand.ctypes.data_as(_i64p), nb, no, nl,
                                             tail.ctypes.data_as(_i64p), C.byref(n_tail), s0.ctypes.data_as(_i64p),
                                             s1.ctypes.data_as(_i64p), n_single.ctypes.data_as(_i64p), C.byref(wse))
        if rc != 0:
            self._err(rc)
        return tail[:n_tail.value], [s0[:n_single[0]], s1[:n_single[1]]], bool(wse.value)

    def close(self):
        if self._h:
            self._lib.ganon_resolver_free(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class ObjectsTable(C.Structure):
    """Mirror of ``ganon_objects_table`` (include/ganon_host.h)."""
    _fields_ = [("n", C.c_int64), ("flag", _i32p), ("pos", _i32p), ("l_seq", _i32p), ("n_cigar", _i32p),
                ("name_len", _i32p), ("seq_off", _i64p), ("qual_off", _i64p), ("name_off", _i64p),
                ("cig_off", _i64p), ("seq", _u8p), ("qual", _u8p), ("names", _p), ("cigar", _u32p)]


class ObjectsSrc(C.Structure):
    _fields_ = [("tables", ObjectsTable * 2), ("n_objs", C.c_int64), ("objs", _i64p), ("n_obj_rows", C.c_int64),
                ("obj_rows", _i64p), ("n_inc", C.c_int64), ("inc", _i64p), ("inc_nib", _i64p), ("masked", _u8p),
                ("n_ind", C.c_int64), ("ind", _i64p), ("ind_ref", _p), ("ind_ref_off", _i64p),
                ("ind_ref_len", _i32p)]


def _indel_args(entries, keep: list):
    """(n, ind int64 array, ref blob, offsets, lengths) of left-over entries [(prefix..., irp, call)]."""
    rows, refs = [], []
    for pre, irp, call in entries:
        rows.append(list(pre) + [int(irp), int(call.variant_type.value), int(call.length)])
        refs.append(call.ref_allele.encode())
    width = len(rows[0]) if rows else 1
    ind = np.ascontiguousarray(np.array(rows, np.int64).reshape(-1, width) if rows else np.zeros((1, width), np.int64))
    lens = np.array([len(r) for r in refs] or [0], np.int32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.int64)]).astype(np.int64)
    blob = np.frombuffer(b"".join(refs) + b"\0", np.uint8).copy()
    keep += [ind, lens, offs, blob]
    return len(rows), ind.ctypes.data_as(_i64p), blob.ctypes.data_as(_p), offs.ctypes.data_as(_i64p), \
        lens.ctypes.data_as(_i32p)


def objects_pack(tables, objs: np.ndarray, obj_rows: np.ndarray, inc: np.ndarray, inc_nib: np.ndarray,
                 masked: np.ndarray, leftovers: dict) -> bytes:
    """``ganon_objects_pack``: one contig plan's complex-name ingredients as a blob (objects.py)."""
    lib = host_lib()
    keep = []

    def arr(a, dt):
        a = np.ascontiguousarray(a, dtype=dt)
        if a.size == 0:
            a = np.zeros(1, dt)
        keep.append(a)
        return a.ctypes.data_as(_PTR_OF[dt])

    src = ObjectsSrc()
    for d, t in enumerate(tables):
        ot = src.tables[d]
        ot.n = t.n
        for f in ("flag", "pos", "l_seq", "n_cigar", "name_len"):
            setattr(ot, f, arr(getattr(t, f), np.int32))
        for f in ("seq_off", "qual_off", "name_off", "cig_off"):
            setattr(ot, f, arr(getattr(t, f), np.int64))
        ot.seq = arr(t.seq, np.uint8)
        ot.qual = arr(t.qual, np.uint8)
        nb = np.ascontiguousarray(t.names_blob if len(t.names_blob) else np.zeros(1, np.uint8))
        keep.append(nb)
        ot.names = nb.ctypes.data_as(_p)
        ot.cigar = arr(t.cigar, np.uint32)
    src.n_objs = len(objs)
    src.objs = arr(objs, np.int64)
    src.n_obj_rows = len(obj_rows)
    src.obj_rows = arr(obj_rows, np.int64)
    src.n_inc = len(inc)
    src.inc = arr(inc, np.int64)
    src.inc_nib = arr(inc_nib, np.int64)
    src.masked = arr(masked, np.uint8)
    entries = [((d, r, sc), irp, call) for (d, r, sc), lst in leftovers.items() for irp, call in lst]
    src.n_ind, src.ind, src.ind_ref, src.ind_ref_off, src.ind_ref_len = _indel_args(entries, keep)
    h = _p()
    rc = lib.ganon_objects_pack(C.byref(src), C.byref(h))
    if rc != 0:
        raise GanonError(f"ganon_objects_pack failed ({rc}): {lib.ganon_objects_last_error().decode(errors='replace')}")
    try:
        n = lib.ganon_blob_size(h)
        return C.string_at(lib.ganon_blob_data(h), n) if n else b""
    finally:
        lib.ganon_blob_free(h)


class ObjectStore:
    """``ganon_objects_*``: the content replay of the resolver log in libganon_host.so (objects.py
    restates it in Python)."""

    def __init__(self):
        self._lib = host_lib()
        h = _p()
        if self._lib.ganon_objects_create(C.byref(h)) != 0:
            raise GanonError("ganon_objects_create failed")
        self._h = h

    def _check(self, rc: int) -> None:
        if rc == 0:
            return
        msg = self._lib.ganon_objects_last_error().decode(errors="replace")
        if rc == PLAN_E_VALUE:
            raise ValueError(msg)
        if rc == PLAN_E_TYPE:
            raise TypeError(msg)
        if rc == PLAN_E_INDEX:
            raise IndexError(msg)
        if rc == PLAN_E_UNSUPPORTED:
            from .planner import UnsupportedInput
            raise UnsupportedInput(msg)
        raise GanonError(f"objects failed ({rc}): {msg}")

    def add_job(self, job: int, blob: bytes) -> None:
        self._check(self._lib.ganon_objects_add_job(self._h, int(job), blob, len(blob)))

    def add_plain(self, job, ds, scope, row, flag, fastq: bytes, edits) -> None:
        keep = []
        n, ind, ref, ro, rl = _indel_args([((), irp, call) for irp, call in edits], keep)
        self._check(self._lib.ganon_objects_add_plain(self._h, int(job), int(ds), int(scope), int(row), int(flag),
                                                      fastq, len(fastq), n, ind, ref, ro, rl))

    def run(self, log: np.ndarray) -> None:
        lg = np.ascontiguousarray(log, np.int64).reshape(-1, 8)
        if len(lg):
            self._check(self._lib.ganon_objects_run(self._h, len(lg), lg.ctypes.data_as(_i64p)))

    def take_all(self) -> dict:
        """serial -> FASTQ bytes of every object written since the last call."""
        tot = C.c_int64(0)
        n = self._lib.ganon_objects_take_all(self._h, None, None, None, 0, C.byref(tot))
        if n <= 0:
            return {}
        ser = np.zeros(n, np.int64)
        lens = np.zeros(n, np.int64)
        buf = C.create_string_buffer(max(tot.value, 1))
        self._lib.ganon_objects_take_all(self._h, ser.ctypes.data_as(_i64p), lens.ctypes.data_as(_i64p), buf,
                                         tot.value, C.byref(tot))
        raw = buf.raw
        off = np.concatenate([[0], np.cumsum(lens)]).tolist()
        return {s: raw[off[i]:off[i + 1]] for i, s in enumerate(ser.tolist())}

    def take(self, serial: int) -> bytes:
        n = self._lib.ganon_objects_take(self._h, int(serial), None, 0)
        if n < 0:
            raise KeyError(serial)
        buf = C.create_string_buffer(max(int(n), 1))
        self._lib.ganon_objects_take(self._h, int(serial), buf, int(n))
        return buf.raw[:n]

    def settle(self, live_ids: np.ndarray) -> None:
        ids = np.ascontiguousarray(live_ids, np.int64)
        self._check(self._lib.ganon_objects_settle(self._h, len(ids), ids.ctypes.data_as(_i64p) if len(ids) else None))

    def close(self) -> None:
        if self._h:
            self._lib.ganon_objects_free(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def io_replay(events: np.ndarray, rec_len: np.ndarray, block: int):
    """``ganon_io_replay``: per output file (dataset * 2 + slot) the write-event indices in the
    order they reach the file."""
    lib = host_lib()
    ev = np.ascontiguousarray(events, np.int32).reshape(-1, 7)
    rl = np.ascontiguousarray(rec_len, np.int64)
    order = np.zeros(max(len(ev), 1), np.int64)
    cnt = np.zeros(4, np.int64)
    k = lib.ganon_io_replay(len(ev), ev.ctypes.data_as(_i32p), rl.ctypes.data_as(_i64p), int(block),
                            order.ctypes.data_as(_i64p), cnt.ctypes.data_as(_i64p))
    if k < 0:
        raise RuntimeError(lib.ganon_plan_last_error().decode(errors="replace"))
    bounds = np.concatenate([[0], np.cumsum(cnt)])
    return [order[bounds[f]:bounds[f + 1]] for f in range(4)]


def host_lib():
    global _host
    if _host is not None:
        return _host
    if not os.path.exists(HOST_LIB_PATH):
        raise GanonError(f"{HOST_LIB_PATH} is missing: run __graft_entry__.build()")
    lib = C.CDLL(HOST_LIB_PATH)
    lib.ganon_bam_open.argtypes = [C.c_char_p, C.c_int, C.POINTER(_p)]
    lib.ganon_bam_view_get.argtypes = [_p, C.POINTER(BamView)]
    lib.ganon_bam_close.argtypes = [_p]
    lib.ganon_bam_reader_open.argtypes = [C.c_char_p, C.c_int, C.POINTER(_p)]
    lib.ganon_bam_reader_has_index.argtypes = [_p]
    lib.ganon_bam_reader_set_window.argtypes = [_p, C.c_int64]
    lib.ganon_bam_reader_header.argtypes = [_p, C.POINTER(BamView)]
    lib.ganon_bam_reader_contig.argtypes = [_p, C.c_int32, C.POINTER(_p)]
    lib.ganon_bam_reader_region.argtypes = [_p, C.c_int32, C.c_int64, C.c_int64, C.POINTER(_p)]
    lib.ganon_bam_reader_close.argtypes = [_p]
    lib.ganon_bam_reader_set_inflater.argtypes = [_p, _p, _p, C.c_int64]
    lib.ganon_host_last_error.restype = C.c_char_p
    lib.ganon_host_inflate_backend.restype = C.c_char_p
    lib.ganon_fastq_format.restype = C.c_int64
    lib.ganon_fastq_format.argtypes = [C.c_int64, C.POINTER(_u8p), _u8p, _i64p, _i32p, _u8p, C.POINTER(_u8p),
                                       _u8p, _i64p, _i32p, _u8p, C.c_char_p, _i64p, _i32p, _u8p, C.c_char_p,
                                       C.c_int64]
    lib.ganon_pack_nt16.argtypes = [C.c_char_p, C.c_int64, _u8p]
    lib.ganon_plan_run.argtypes = [C.POINTER(PlanInput), C.POINTER(_p)]
    lib.ganon_plan_view_get.argtypes = [_p, C.POINTER(PlanView)]
    lib.ganon_plan_free.argtypes = [_p]
    lib.ganon_plan_last_error.restype = C.c_char_p
    lib.ganon_io_replay.argtypes = [C.c_int64, _i32p, _i64p, C.c_int64, _i64p, _i64p]
    lib.ganon_resolver_create.argtypes = [C.POINTER(_p)]
    lib.ganon_resolver_free.argtypes = [_p]
    lib.ganon_resolver_contig.argtypes = [_p, C.c_int32, C.c_int64, _i32p, _i64p, _p, _i64p, _i32p, C.c_int64, _i64p,
                                          _p, _i64p, _i32p, C.c_int64, _i64p, _i64p, _i64p, _i32p, _i64p]
    lib.ganon_objects_pack.argtypes = [C.POINTER(ObjectsSrc), C.POINTER(_p)]
    lib.ganon_blob_size.argtypes = [_p]
    lib.ganon_blob_size.restype = C.c_int64
    lib.ganon_blob_data.argtypes = [_p]
    lib.ganon_blob_data.restype = C.c_void_p
    lib.ganon_blob_free.argtypes = [_p]
    lib.ganon_objects_create.argtypes = [C.POINTER(_p)]
    lib.ganon_objects_free.argtypes = [_p]
    lib.ganon_objects_add_job.argtypes = [_p, C.c_int32, C.c_char_p, C.c_int64]
    lib.ganon_objects_add_plain.argtypes = [_p, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int32, C.c_char_p,
                                            C.c_int64, C.c_int64, _i64p, _p, _i64p, _i32p]
    lib.ganon_objects_run.argtypes = [_p, C.c_int64, _i64p]
    lib.ganon_objects_take.argtypes = [_p, C.c_int64, C.c_char_p, C.c_int64]
    lib.ganon_objects_take.restype = C.c_int64
    lib.ganon_objects_settle.argtypes = [_p, C.c_int64, _i64p]
    lib.ganon_objects_take_all.argtypes = [_p, _i64p, _i64p, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
    lib.ganon_objects_take_all.restype = C.c_int64
    lib.ganon_aux_sa_count.argtypes = [_u8p, _i64p, _i32p, C.c_int64, _i32p]
    lib.ganon_gather_ranges.argtypes = [C.c_void_p, C.c_int64, C.c_int64, _i64p, _i64p, C.c_char_p, C.c_int64]
    lib.ganon_gather_ranges.restype = C.c_int64
    lib.ganon_gather_ranges2.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int64, _u8p, _i64p, _i64p,
                                         C.c_char_p, C.c_int64]
    lib.ganon_gather_ranges2.restype = C.c_int64
    lib.ganon_bam_reader_set_buffer_alloc.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.ganon_bam_reader_set_region_decoder.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    lib.ganon_host_phase_times.argtypes = [C.POINTER(C.c_double), C.c_int, C.c_int]
    lib.ganon_host_phase_times.restype = C.c_int
    lib.ganon_fastq_edit.argtypes = [C.c_int64, C.c_char_p, _i64p, _u8p, _i32p, _i64p, _i64p, C.c_char_p, _i64p,
                                     _p, C.c_int64, _i64p, _i64p]
    lib.ganon_objects_last_error.restype = C.c_char_p
    lib.ganon_resolver_mark_written.argtypes = [_p, C.c_int64, _p, _i64p, _i32p]
    lib.ganon_resolver_mark_written.restype = C.c_int64
    lib.ganon_resolver_take_log.argtypes = [_p, _i64p, C.c_int64]
    lib.ganon_resolver_take_log.restype = C.c_int64
    lib.ganon_resolver_pending.argtypes = [_p, _i64p, C.c_int64]
    lib.ganon_resolver_pending.restype = C.c_int64
    lib.ganon_resolver_finish.argtypes = [_p, C.c_int64, _i64p, _p, _i64p, _i32p, _i64p, _i64p, _i64p, _i64p,
                                          _i64p, _i32p]
    lib.ganon_io_replay.restype = C.c_int64
    _host = lib
    return lib
