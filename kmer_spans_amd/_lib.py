"""ctypes binding of libkmerspans.so (the C ABI in include/kmer_spans.h).

The shared library is built in-tree by ``__graft_entry__.build()``
(kmer_spans_amd/csrc/Makefile).  There is no fallback: importing this module
without the library raises, so a missing build can never silently turn into
a CPU path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# KS_LIB_PATH: an alternative build of the same library (kernel-variant
# experiments); the in-tree build is the default.
LIB_PATH = os.environ.get("KS_LIB_PATH") or os.path.join(_HERE, "libkmerspans.so")

KS_OK = 0
KS_MAX_K = 15


class KmerSpansError(RuntimeError):
    """An error reported by libkmerspans (the reference's error() strings)."""


class Regions(C.Structure):
    _fields_ = [("n", C.c_int64), ("seq_id", C.POINTER(C.c_int32)), ("beg", C.POINTER(C.c_int32)),
                ("end", C.POINTER(C.c_int32)), ("score", C.POINTER(C.c_double))]


class DevSeqs(C.Structure):
    _fields_ = [("seq", C.c_void_p), ("offsets_host", C.c_void_p), ("offsets_dev", C.c_void_p),
                ("nseq", C.c_int32)]


class ScanStats(C.Structure):
    _fields_ = [("ms_total", C.c_double), ("ms_runs", C.c_double), ("ms_scan", C.c_double),
                ("ms_rescan", C.c_double), ("ms_finish", C.c_double), ("n_bases", C.c_int64),
                ("n_scored", C.c_int64), ("n_runs", C.c_int64), ("n_regions", C.c_int64),
                ("n_rescan", C.c_int64), ("scan_algo", C.c_int32),
                ("n_replay", C.c_int64), ("ms_layout", C.c_double), ("ms_predict", C.c_double),
                ("ms_carry", C.c_double), ("ms_stitch", C.c_double)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class TableInfo(C.Structure):
    _fields_ = [("k", C.c_int32), ("compressed", C.c_int32), ("positions_per_read", C.c_int32),
                ("code_bits", C.c_int32), ("distinct", C.c_int64), ("ext_bytes", C.c_int64),
                ("escape_fraction", C.c_double), ("ms_upload", C.c_double), ("ms_compress", C.c_double),
                ("ms_codes12", C.c_double), ("ms_ext_alloc", C.c_double), ("ms_ext_build", C.c_double),
                ("ms_total", C.c_double), ("line_kind", C.c_int32), ("line_own", C.c_int32)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class Fasta(C.Structure):
    _fields_ = [("seqs", DevSeqs), ("names", C.POINTER(C.c_char_p)), ("n_records", C.c_int64),
                ("bases_all", C.c_int64), ("bases_kept", C.c_int64), ("device", C.c_int32),
                ("ms_upload", C.c_double), ("ms_parse", C.c_double)]


class CountFile(C.Structure):
    _fields_ = [("valid", C.c_int32), ("nk", C.c_int32), ("k", C.POINTER(C.c_int32)),
                ("lens", C.POINTER(C.c_int64)), ("counts", C.POINTER(C.POINTER(C.c_int32)))]


class KmerFileInfo(C.Structure):
    _fields_ = [("written", C.c_int32), ("seq_size", C.c_double), ("seq_fsize", C.c_double),
                ("seq_fl", C.c_double), ("out_path", C.c_char * 4096), ("message", C.c_char * 512)]


# Every symbol include/kmer_spans.h declares (tests check they are exported).
EXPORTS = [
    "ks_last_error", "ks_version", "ks_regions_free", "ks_ctx_create", "ks_ctx_destroy",
    "ks_ctx_set_stream", "ks_default_ctx", "ks_kmer_counts", "ks_kmer_regions",
    "ks_low_comp_regions", "ks_kmer_seq", "ks_rank_table", "ks_log2_table", "ks_pm1_table",
    "ks_table_create", "ks_table_destroy", "ks_table_is_compressed", "ks_table_distinct",
    "ks_table_positions_per_read", "ks_table_create_hint", "ks_table_code_bits", "ks_table_escape_fraction",
    "ks_table_get_info",
    "ks_scan_dev", "ks_count_dev", "ks_ctx_set_scan_algo", "ks_tr_lr_regions", "ks_tr_lr_dev",
    "ks_fasta_load", "ks_fasta_parse", "ks_fasta_copy_seqs", "ks_fasta_free", "ks_count_multi_dev",
    "ks_count_file_write", "ks_count_file_read", "ks_count_file_free", "ks_kmers_to_file",
    "ks_windowed_dist", "ks_windowed_dev", "ks_table_from_counts",
    "ks_release_cache", "ks_set_fork_broker", "ks_set_host_cache",
    "ks_set_devices", "ks_get_devices", "ks_shard_plan", "ks_merge_parts", "ks_set_host_cache_idle",
    "ks_multi_last_stats",
]

SCORES = {"log2": 1, "pm1": 2, "rank": 3}  # KS_SCORE_* of ks_table_from_counts

_lib = None


def load():
    """Load and type the library (raises if it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
    L = C.CDLL(LIB_PATH)
    P, I32, I64, D = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    sigs = {
        "ks_last_error": ([], C.c_char_p),
        "ks_version": ([], C.c_char_p),
        "ks_regions_free": ([P], None),
        "ks_ctx_create": ([I32, P], I32),
        "ks_ctx_destroy": ([P], None),
        "ks_ctx_set_stream": ([P, P], I32),
        "ks_default_ctx": ([], P),
        "ks_ctx_set_scan_algo": ([P, I32], I32),
        "ks_kmer_counts": ([P, P, P, I32, I32, P, P], I32),
        "ks_kmer_regions": ([P, P, P, I32, I32, P, I64, I32, D, P, P, P], I32),
        "ks_low_comp_regions": ([P, P, P, I32, I32, I32, D, D, P, P, P, P], I32),
        "ks_kmer_seq": ([I32, P, C.c_size_t], I32),
        "ks_rank_table": ([P, I32, D, P], I32),
        "ks_log2_table": ([P, I32, P], I32),
        "ks_pm1_table": ([P, I32, P], I32),
        "ks_table_create": ([P, P, I32, D, I32, P], I32),
        "ks_table_destroy": ([P], None),
        "ks_table_is_compressed": ([P], I32),
        "ks_table_distinct": ([P], I64),
        "ks_table_positions_per_read": ([P], I32),
        "ks_table_create_hint": ([P, P, I32, D, I32, P, P], I32),
        "ks_table_code_bits": ([P], I32),
        "ks_table_escape_fraction": ([P], D),
        "ks_table_get_info": ([P, P], I32),
        "ks_scan_dev": ([P, P, I32, P, I32, D, P, P, P], I32),
        "ks_count_dev": ([P, P, I32, P, P], I32),
        "ks_tr_lr_regions": ([P, P, P, I32, I32, I32, P, P, P, I64, P, P], I32),
        "ks_tr_lr_dev": ([P, P, I32, P, P, I32, P, P], I32),
        "ks_fasta_load": ([P, C.c_char_p, I64, P], I32),
        "ks_fasta_parse": ([P, C.c_char_p, I64, I64, P], I32),
        "ks_fasta_copy_seqs": ([P, P], I32),
        "ks_fasta_free": ([P], None),
        "ks_count_multi_dev": ([P, P, P, I32, P, P], I32),
        "ks_count_file_write": ([C.c_char_p, I32, I32, P, P], I32),
        "ks_count_file_read": ([C.c_char_p, I32, P], I32),
        "ks_count_file_free": ([P], None),
        "ks_kmers_to_file": ([P, C.c_char_p, C.c_char_p, P, I32, D, I32, P], I32),
        "ks_windowed_dist": ([P, P, P, I32, P, I32, I32, I32, I32, P, P, P], I32),
        "ks_windowed_dev": ([P, P, P, I32, I32, I32, P, P, P], I32),
        "ks_table_from_counts": ([P, P, I32, I32, D, D, I32, I64, P, P], I32),
        "ks_release_cache": ([], None),
        "ks_set_fork_broker": ([I32], I32),
        "ks_set_host_cache": ([I32], I32),
        "ks_set_devices": ([P, I32], I32),
        "ks_set_host_cache_idle": ([D], I32),
        "ks_get_devices": ([P, I32], I32),
        "ks_shard_plan": ([P, P, I32, I32, P, I64], I64),
        "ks_merge_parts": ([P, I64, I32, P, P], I32),
        "ks_multi_last_stats": ([P, I32], I32),
    }
    for name, (args, res) in sigs.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def version() -> str:
    return load().ks_version().decode()


def build_id() -> str:
    """Hash of the library's sources and build flags (csrc/Makefile)."""
    v = version()
    return v.rsplit("build ", 1)[1] if "build " in v else "unknown"


def check(rc: int) -> None:
    if rc != KS_OK:
        msg = load().ks_last_error().decode(errors="replace")
        raise KmerSpansError(msg or f"libkmerspans error {rc}")


class _RegionBlock:
    """Owns a ks_regions block; freed when the last numpy view of it dies."""

    def __init__(self, r: Regions):
        self.r = r

    def __del__(self):
        if _lib is not None:
            _lib.ks_regions_free(C.byref(self.r))


def regions_to_numpy(r: Regions):
    """(pos int32[3, n], score float64[2, n]) as views of the library's output
    block (seq_id|beg|end contiguous, score followed by zeros: include/
    kmer_spans.h), which is freed with the last view -- no host copy."""
    n = int(r.n)
    if n == 0:
        load().ks_regions_free(C.byref(r))
        return np.empty((3, 0), dtype=np.int32), np.empty((2, 0), dtype=np.float64)
    holder = _RegionBlock(r)
    ib = (C.c_char * (3 * n * 4)).from_address(C.cast(r.seq_id, C.c_void_p).value)
    sb = (C.c_char * (2 * n * 8)).from_address(C.cast(r.score, C.c_void_p).value)
    ib._holder = holder
    sb._holder = holder
    pos = np.frombuffer(ib, dtype=np.int32).reshape(3, n)
    score = np.frombuffer(sb, dtype=np.float64).reshape(2, n)
    return pos, score


def shard_plan(seqs, nparts: int):
    """ks_shard_plan (csrc/ks_multi.cpp): the pieces nparts devices take, as
    (part, sequence, lo, hi) rows -- whole sequences by LPT on length, cut in
    the middle of N gaps of >= 1000 bases when whole sequences leave a part
    more than 0.5 % above the fair share.  seqs: uint8 numpy arrays or bytes
    (host memory; the gap scan runs on the host, no device is touched)."""
    arrs = [np.ascontiguousarray(np.frombuffer(s, dtype=np.uint8) if isinstance(s, (bytes, bytearray)) else s,
                                 dtype=np.uint8) for s in seqs]
    ptrs = (C.c_void_p * len(arrs))(*[a.ctypes.data if a.size else None for a in arrs])
    lens = np.array([a.size for a in arrs], dtype=np.int64)
    L = load()
    n = L.ks_shard_plan(ptrs, lens.ctypes.data, len(arrs), int(nparts), None, 0)
    if n < 0:
        raise KmerSpansError("ks_shard_plan: bad argument")
    out = np.zeros((max(n, 1), 4), dtype=np.int64)
    L.ks_shard_plan(ptrs, lens.ctypes.data, len(arrs), int(nparts), out.ctypes.data, n)
    return [tuple(int(x) for x in row) for row in out[:n]]


def multi_last_stats():
    """Phases of the last multi-device host call (ks_multi_last_stats, ms)."""
    L = load()
    n = L.ks_multi_last_stats(None, 0)
    v = (C.c_double * n)()
    L.ks_multi_last_stats(v, n)
    v = list(v)
    parts = int(v[5])
    return {"total_ms": v[0], "phase1_ms": v[1], "host_sum_ms": v[2], "phase2_ms": v[3], "merge_ms": v[4],
            "parts": [{"body_ms": v[6 + 4 * p], "stage_count_ms": v[7 + 4 * p], "table_upload_ms": v[8 + 4 * p],
                       "scan_ms": v[9 + 4 * p]} for p in range(parts)]}


class Context:
    """One GPU + HIP stream + device workspace (ks_ctx).  Created lazily, so a
    process that only forks workers never touches HIP in the parent."""

    def __init__(self, device: int = 0):
        self.device = device
        self.stream = -1  # -1: the ctx's own non-blocking stream
        self._h = C.c_void_p()
        check(load().ks_ctx_create(device, C.byref(self._h)))

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_ptr: int | None):
        """hipStream_t as an int; 0/None = HIP's default (null) stream."""
        check(load().ks_ctx_set_stream(self._h, C.c_void_p(stream_ptr) if stream_ptr else None))
        self.stream = int(stream_ptr or 0)

    def set_scan_algo(self, algo: int):
        check(load().ks_ctx_set_scan_algo(self._h, int(algo)))

    def close(self):
        if self._h:
            load().ks_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_contexts: dict[int, Context] = {}


def context(device: int = 0) -> Context:
    ctx = _contexts.get(device)
    if ctx is None:
        ctx = _contexts[device] = Context(device)
    return ctx
