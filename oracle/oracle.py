"""ctypes wrapper of the CPU oracle (oracle/libksoracle.so).

TEST INFRASTRUCTURE ONLY -- the parity checker for the HIP product path and
the "port" CPU baseline of bench.py.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.  The C restatement it
loads follows /root/reference/src/kmer_spans.c line by line (see
oracle/ks_oracle.c for the per-function citations); parity is pinned by the
fixtures in tests/golden/ ("Oracle").

Outputs mirror the reference's .Call return values:
  kmer_counts      -> (n, counts)                                   kmer_spans.c:453-487
  kmer_regions     -> dict(n, counts, pos[3,R] int32, score[2,R])   kmer_spans.c:490-546
  low_comp_regions -> dict(n[2], counts, w_rank, pos, score)        kmer_spans.c:548-621
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libksoracle.so")
_lib = None


class _Regions(C.Structure):
    _fields_ = [("n", C.c_int64), ("cap", C.c_int64),
                ("seq_id", C.POINTER(C.c_int32)), ("beg", C.POINTER(C.c_int32)),
                ("end", C.POINTER(C.c_int32)), ("score", C.POINTER(C.c_double))]


def build() -> str:
    """Compile the oracle (gcc) in place; returns the .so path."""
    subprocess.check_call(["make", "-s", "-C", _HERE, "libksoracle.so"])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        L.orc_kmer_counts.argtypes = [P, P, C.c_int32, C.c_int32, P, P]
        L.orc_kmer_regions.argtypes = [P, P, C.c_int32, C.c_int32, P, C.c_int32, C.c_double, P, P, P]
        L.orc_scan.argtypes = [P, P, C.c_int32, C.c_int32, P, C.c_double, C.c_int32, C.c_double, P, P]
        L.orc_low_comp.argtypes = [P, P, C.c_int32, C.c_int32, C.c_int32, C.c_double, C.c_double, P, P, P, P]
        L.orc_rank_table.argtypes = [P, C.c_int32, C.c_double, P]
        L.orc_log2_table.argtypes = [P, C.c_int32, P]
        L.orc_pm1_table.argtypes = [P, C.c_int32, P]
        L.orc_kmer_seq.argtypes = [C.c_int32, P]
        L.orc_regions_free.argtypes = [P]
        L.orc_trlr_remap.argtypes = [P, C.c_int32, P, P, P, P]
        L.orc_tr_lr_regions.argtypes = [P, P, C.c_int32, C.c_int32, C.c_int32, P, P, P]
        L.orc_fasta_parse.argtypes = [P, C.c_int64, C.c_int64, P]
        L.orc_windowed_dist.argtypes = [P, P, C.c_int32, P, C.c_int32, C.c_int32, C.c_int32, P, P, P]
        L.orc_fasta_free.argtypes = [P]
        _lib = L
    return _lib


class OracleError(RuntimeError):
    pass


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise OracleError(f"{what}: oracle error {rc}")


def _as_bytes(s) -> bytes:
    return s.encode("latin-1") if isinstance(s, str) else bytes(s)


class _SeqArgs:
    """Keeps the byte buffers alive while their pointers are passed."""

    def __init__(self, seqs):
        if isinstance(seqs, (str, bytes, bytearray, memoryview, np.ndarray)):
            seqs = [seqs]
        self.bufs = []
        for s in seqs:
            if isinstance(s, np.ndarray):
                self.bufs.append(np.ascontiguousarray(s, dtype=np.uint8))
            else:
                self.bufs.append(np.frombuffer(_as_bytes(s), dtype=np.uint8))
        self.n = len(self.bufs)
        self.ptrs = (C.c_void_p * max(self.n, 1))(*[b.ctypes.data if b.size else 0 for b in self.bufs])
        self.lens = np.array([b.size for b in self.bufs] or [0], dtype=np.int64)
        # empty buffers: give a valid non-null pointer
        self._empty = np.zeros(1, dtype=np.uint8)
        for i, b in enumerate(self.bufs):
            if b.size == 0:
                self.ptrs[i] = self._empty.ctypes.data


def _regions_to_numpy(r: _Regions):
    n = r.n
    pos = np.zeros((3, n), dtype=np.int32)
    score = np.zeros((2, n), dtype=np.float64)
    if n:
        pos[0] = np.ctypeslib.as_array(r.seq_id, shape=(n,))
        pos[1] = np.ctypeslib.as_array(r.beg, shape=(n,))
        pos[2] = np.ctypeslib.as_array(r.end, shape=(n,))
        score[0] = np.ctypeslib.as_array(r.score, shape=(n,))
    lib().orc_regions_free(C.byref(r))
    return pos, score


def kmer_counts(seqs, k: int):
    a = _SeqArgs(seqs)
    counts = np.zeros(4 ** k if 1 <= k <= 15 else 1, dtype=np.int32)
    n = C.c_double(0)
    _check(lib().orc_kmer_counts(a.ptrs, a.lens.ctypes.data, a.n, k, counts.ctypes.data, C.byref(n)),
           "kmer_counts")
    return n.value, counts


def kmer_regions(seqs, k: int, w, min_width: int, min_score: float, visits: bool = True):
    a = _SeqArgs(seqs)
    w = np.ascontiguousarray(w, dtype=np.float64)
    if w.size != 4 ** k:
        raise OracleError("kmer_w must have 4^k elements")
    vis = np.zeros(4 ** k, dtype=np.int32) if visits else None
    n = C.c_double(0)
    r = _Regions()
    _check(lib().orc_kmer_regions(a.ptrs, a.lens.ctypes.data, a.n, k, w.ctypes.data, int(min_width),
                                  float(min_score), vis.ctypes.data if vis is not None else None,
                                  C.byref(n), C.byref(r)), "kmer_regions")
    pos, score = _regions_to_numpy(r)
    return {"n": n.value, "counts": vis, "pos": pos, "score": score}


def scan(seqs, k: int, w, thr: float, min_width: int, min_score: float, visits: bool = False):
    """The bare kmer_regions loop (threshold thr) over every sequence with len >= k."""
    a = _SeqArgs(seqs)
    w = np.ascontiguousarray(w, dtype=np.float64)
    vis = np.zeros(4 ** k, dtype=np.int32) if visits else None
    r = _Regions()
    _check(lib().orc_scan(a.ptrs, a.lens.ctypes.data, a.n, k, w.ctypes.data, float(thr), int(min_width),
                          float(min_score), vis.ctypes.data if vis is not None else None, C.byref(r)), "scan")
    pos, score = _regions_to_numpy(r)
    return {"counts": vis, "pos": pos, "score": score}


def low_comp_regions(seqs, k: int, min_width: int, min_score: float, thr: float = 0.75):
    a = _SeqArgs(seqs)
    counts = np.zeros(4 ** k, dtype=np.int32)
    ranks = np.zeros(4 ** k, dtype=np.float64)
    n = np.zeros(2, dtype=np.float64)
    r = _Regions()
    _check(lib().orc_low_comp(a.ptrs, a.lens.ctypes.data, a.n, k, int(min_width), float(min_score),
                              float(thr), counts.ctypes.data, ranks.ctypes.data, n.ctypes.data,
                              C.byref(r)), "low_comp_regions")
    pos, score = _regions_to_numpy(r)
    return {"n": n, "counts": counts, "w_rank": ranks, "pos": pos, "score": score}


def rank_table(counts, k: int, total: float):
    counts = np.ascontiguousarray(counts, dtype=np.int32)
    out = np.zeros(4 ** k, dtype=np.float64)
    _check(lib().orc_rank_table(counts.ctypes.data, k, float(total), out.ctypes.data), "rank_table")
    return out


def log2_table(counts, k: int):
    counts = np.ascontiguousarray(counts, dtype=np.int32)
    out = np.zeros(4 ** k, dtype=np.float64)
    _check(lib().orc_log2_table(counts.ctypes.data, k, out.ctypes.data), "log2_table")
    return out


def pm1_table(counts, k: int):
    counts = np.ascontiguousarray(counts, dtype=np.int32)
    out = np.zeros(4 ** k, dtype=np.float64)
    _check(lib().orc_pm1_table(counts.ctypes.data, k, out.ctypes.data), "pm1_table")
    return out


def kmer_seq(k: int):
    buf = C.create_string_buffer((4 ** k) * (k + 1))
    _check(lib().orc_kmer_seq(k, buf), "kmer_seq")
    raw = buf.raw
    return [raw[i * (k + 1):i * (k + 1) + k].decode() for i in range(4 ** k)]


def trlr_remap(kmers, k: int, kmer_scores, trans_scores):
    """tr_lr_regions_r's remap of user-ordered tables to 2-bit code order:
    returns (ks, tr, n_bad)."""
    n = 4 ** k
    bufs = [C.create_string_buffer(_as_bytes(x)) for x in kmers]
    ptrs = (C.c_char_p * n)(*[C.cast(b, C.c_char_p) for b in bufs])
    ks_in = np.ascontiguousarray(kmer_scores, dtype=np.float64)
    tr_in = np.ascontiguousarray(trans_scores, dtype=np.float64)
    ks = np.zeros(n, dtype=np.float64)
    tr = np.zeros(n, dtype=np.float64)
    bad = lib().orc_trlr_remap(ptrs, k, ks_in.ctypes.data, tr_in.ctypes.data, ks.ctypes.data, tr.ctypes.data)
    return ks, tr, bad


def tr_lr_regions(seqs, k: int, min_len: int, ks, tr):
    """find_kmer_tr_lr_regions over every sequence with 2-bit-ordered tables;
    1-based (seq_id, beg, end) and the region maximum."""
    a = _SeqArgs(seqs)
    ks = np.ascontiguousarray(ks, dtype=np.float64)
    tr = np.ascontiguousarray(tr, dtype=np.float64)
    r = _Regions()
    _check(lib().orc_tr_lr_regions(a.ptrs, a.lens.ctypes.data, a.n, k, int(min_len), ks.ctypes.data,
                                   tr.ctypes.data, C.byref(r)), "tr_lr_regions")
    pos, score = _regions_to_numpy(r)
    return {"pos": pos, "score": score}


class _Fasta(C.Structure):
    _fields_ = [("n_records", C.c_int64), ("nseq", C.c_int64), ("bases_all", C.c_int64), ("err_pos", C.c_int64),
                ("seq", C.POINTER(C.c_uint8)), ("offs", C.POINTER(C.c_int64)), ("names", C.POINTER(C.c_char_p))]


def fasta_parse(text, min_len: int = 0) -> dict:
    """FASTA text -> {'names', 'seqs' (bytes, upper-cased), 'n_records',
    'bases_all'} (orc_fasta_parse); raises OracleError with the failing byte
    position on invalid input."""
    b = _as_bytes(text)
    buf = np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, dtype=np.uint8)
    f = _Fasta()
    rc = lib().orc_fasta_parse(buf.ctypes.data, len(b), int(min_len), C.byref(f))
    if rc != 0:
        pos = int(f.err_pos)
        lib().orc_fasta_free(C.byref(f))
        raise OracleError(("invalid byte" if rc == -1 else "sequence before description") + f" at {pos}")
    try:
        n = int(f.nseq)
        offs = np.ctypeslib.as_array(f.offs, shape=(n + 1,)).copy()
        data = np.ctypeslib.as_array(f.seq, shape=(max(int(offs[-1]), 1),))[:int(offs[-1])].tobytes()
        return {"names": [f.names[q].decode("latin-1") for q in range(n)],
                "seqs": [data[offs[q]:offs[q + 1]] for q in range(n)],
                "n_records": int(f.n_records), "bases_all": int(f.bases_all)}
    finally:
        lib().orc_fasta_free(C.byref(f))


def count_file_bytes(magic: int, ks, counts) -> bytes:
    """kmers.to.file's file image (kmer_spans.R:152-159): R writeBin of
    as.integer values, little-endian int32: magic, n, n x 4^k, counts."""
    parts = [np.array([magic, len(ks)], dtype="<i4"), np.array([4 ** int(k) for k in ks], dtype="<i4")]
    parts += [np.asarray(c, dtype="<i4") for c in counts]
    return b"".join(p.tobytes() for p in parts)


def read_count_file(data: bytes, magic: int):
    """read.kmers (kmer_spans.R:162-186) on a file image: False on a wrong
    magic or n < 1, else {'k', 'counts'}; readBin stops short at EOF."""
    a = np.frombuffer(data[:len(data) // 4 * 4], dtype="<i4")
    if a.size < 1 or a[0] != magic or a.size < 2 or a[1] < 1:
        return False
    kn = int(a[1])
    lens = a[2:2 + kn]
    pos = 2 + lens.size
    counts = []
    for n in lens:
        counts.append(a[pos:pos + int(n)].astype(np.int32))
        pos += int(n)
    ks = np.array([int(np.log2(float(n)) / 2) if n > 0 else -1 for n in lens], dtype=np.int32)
    return {"k": ks, "counts": counts}


def windowed_dist(seqs, kmers, k: int, window: int, ret_flag: int = 0) -> dict:
    """windowed_kmer_count_distributions_r (kmer_spans.c:717-793):
    {'dist': int32[window + 1, kmer_n], 'seq_i': int32[nseq],
    'scores': None or per sequence int32[len, kmer_n] (None where excluded)}."""
    sa = _SeqArgs(seqs)
    kb = [_as_bytes(x) for x in kmers]
    kp = (C.c_char_p * max(len(kb), 1))(*kb)
    n = len(kb)
    dist = np.zeros((n, window + 1), dtype=np.int32)  # column-major [window+1, n]
    inc = np.zeros(max(sa.n, 1), dtype=np.int32)
    pos = None
    pp = None
    if ret_flag & 1:
        pos = [np.zeros((n, int(L)), dtype=np.int32) for L in sa.lens[:sa.n]]
        pp = (C.c_void_p * max(sa.n, 1))(*[p.ctypes.data for p in pos])
    rc = lib().orc_windowed_dist(sa.ptrs, sa.lens.ctypes.data, sa.n, kp, n, int(k), int(window),
                                 dist.ctypes.data, inc.ctypes.data, pp)
    _check(rc, "windowed_dist")
    scores = None
    if pos is not None:
        scores = [p.T.copy() if inc[i] else None for i, p in enumerate(pos)]
    return {"dist": dist.T.copy(), "seq_i": inc[:sa.n].copy(), "scores": scores}
