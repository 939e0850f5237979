"""The reference's user API (kmer_spans.R) on top of the C ABI.

Same function names (dots become underscores), argument meaning, return
layout and error behaviour as /root/reference/kmer_spans.R:

  kmer_counts(seq, k, with_f=True)               kmer_spans.R:18-27
  kmer_regions(seq, k, kmer_scores, min_width, min_score)   :41-52
  kmer_low_comp_regions(seq, k, min_w, min_score, thr=0.75) :72-79
  kmer_seq(k)                                     :84-86
  lr_regions(seq, params, kmers, kmer_scores, trans_scores)  :88-99
  kmers_to_file(seq_f, out_prefix, k, min_l=1e5, magic)      :127-160
  read_kmers(fname, magic)                        :162-186
  read_fasta(path, min_len=0)   (readDNAStringSet + as.character, :136-144)
  window_kmer_dist(seq, kmers, window, freq=True, ret_flag=0)  :103-118

Sequences are a str/bytes or a list of them (R character vectors).  Results
come from libkmerspans.so on the GPU; nothing here computes a result on the
CPU.  Table builders for the README score functions are exposed as
``log2_table`` / ``pm1_table`` / ``rank_table``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import KmerSpansError, Regions, check, load, regions_to_numpy


class _HostSeqs:
    """(char* const*, int64 lens) view of a list of byte strings."""

    def __init__(self, seq):
        if isinstance(seq, (str, bytes, bytearray, memoryview, np.ndarray)):
            seq = [seq]
        self.bufs = []
        for s in seq:
            if isinstance(s, np.ndarray):
                b = np.ascontiguousarray(s, dtype=np.uint8)
            elif isinstance(s, str):
                b = np.frombuffer(s.encode("latin-1"), dtype=np.uint8)
            else:
                b = np.frombuffer(bytes(s), dtype=np.uint8)
            self.bufs.append(b)
        self.n = len(self.bufs)
        self._empty = np.zeros(1, dtype=np.uint8)
        self.ptrs = (C.c_void_p * max(self.n, 1))()
        for i, b in enumerate(self.bufs):
            self.ptrs[i] = b.ctypes.data if b.size else self._empty.ctypes.data
        self.lens = np.array([b.size for b in self.bufs] or [0], dtype=np.int64)


def set_devices(devices) -> None:
    """Devices the host entry points (kmer_counts, kmer_regions,
    kmer_low_comp_regions on device 0, i.e. the library's default) spread a
    call over (ks_set_devices: LPT shards, one context and host thread per
    entry, counts added, regions merged into the caller's order).  [] or one
    device: device 0 alone.  The list may repeat a device."""
    d = np.ascontiguousarray(np.asarray(list(devices), dtype=np.int32))
    check(load().ks_set_devices(d.ctypes.data if d.size else None, int(d.size)))


def get_devices() -> list:
    n = int(load().ks_get_devices(None, 0))
    d = np.zeros(max(n, 1), dtype=np.int32)
    load().ks_get_devices(d.ctypes.data, n)
    return d[:n].tolist()


def _ctx(device):
    """Device 0 uses the library's lazily created default context, so that
    argument errors surface before any HIP call (kmer_spans.c validates before
    allocating); other devices get an explicit context."""
    return None if int(device) == 0 else _lib.context(device).handle


def kmer_seq(k: int) -> list[str]:
    """k-mer strings in the internal A,C,T,G code order (kmer_seq_r)."""
    k = int(k)
    if k < 1 or k > _lib.KS_MAX_K:
        check(load().ks_kmer_seq(k, None, 0))
    n = 4 ** k
    buf = C.create_string_buffer(n * (k + 1))
    check(load().ks_kmer_seq(k, buf, n * (k + 1)))
    raw = buf.raw
    return [raw[i * (k + 1):i * (k + 1) + k].decode() for i in range(n)]


def kmer_counts(seq, k: int, with_f: bool = True, device: int = 0) -> dict:
    """kmer.counts: {'n': {'k': k, 'n': words}, 'counts': int32[4^k], 'f': ...}."""
    k = int(k)
    hs = _HostSeqs(seq)
    counts = np.zeros(4 ** k if 1 <= k <= _lib.KS_MAX_K else 1, dtype=np.int32)
    n = C.c_double(0)
    check(load().ks_kmer_counts(_ctx(device), hs.ptrs, hs.lens.ctypes.data, hs.n, k,
                                counts.ctypes.data, C.byref(n)))
    out = {"n": {"k": k, "n": n.value}, "counts": counts}
    if with_f:
        with np.errstate(invalid="ignore", divide="ignore"):
            out["f"] = counts / float(counts.astype(np.int64).sum())
    return out


def _ordered_scores(k: int, kmer_scores):
    """kmer.regions reorders a named score vector by kmer.seq(k)
    (kmer_spans.R:42-47); an unnamed array is taken as internal order."""
    if isinstance(kmer_scores, dict):
        if len(kmer_scores) != 4 ** k:
            raise KmerSpansError("There should be a total of 4^k scores")
        names = kmer_seq(k)
        if any(nm not in kmer_scores for nm in names):
            raise KmerSpansError("all kmers not defined")
        return np.array([kmer_scores[nm] for nm in names], dtype=np.float64)
    if hasattr(kmer_scores, "index") and hasattr(kmer_scores, "values"):  # pandas Series
        return _ordered_scores(k, dict(zip(kmer_scores.index, kmer_scores.values)))
    w = np.ascontiguousarray(kmer_scores, dtype=np.float64).ravel()
    if w.size != 4 ** k:
        raise KmerSpansError("There should be a total of 4^k scores")
    return w


def kmer_regions(seq, k: int, kmer_scores, min_width: int, min_score: float, visits: bool = True,
                 device: int = 0) -> dict:
    """kmer.regions: {'n', 'counts' (visit histogram), 'pos' int32[3, R]
    (seq_id, beg, end), 'score' float64[2, R] (score, 0)} -- not transposed,
    exactly as kmer_spans.R:48-51 returns it."""
    k = int(k)
    w = _ordered_scores(k, kmer_scores)
    hs = _HostSeqs(seq)
    vis = np.zeros(4 ** k, dtype=np.int32) if visits else None
    n = C.c_double(0)
    r = Regions()
    check(load().ks_kmer_regions(_ctx(device), hs.ptrs, hs.lens.ctypes.data, hs.n, k, w.ctypes.data,
                                 w.size, int(min_width), float(min_score),
                                 vis.ctypes.data if vis is not None else None, C.byref(n), C.byref(r)))
    pos, score = regions_to_numpy(r)
    return {"n": n.value, "counts": vis, "pos": pos, "score": score}


def kmer_low_comp_regions(seq, k: int, min_w: int, min_score: float, thr: float = 0.75,
                          device: int = 0) -> dict:
    """kmer.low.comp.regions: {'n' [#words, 0], 'counts', 'w_rank',
    'pos' int32[R, 3], 'score' float64[R, 2]} (pos/score transposed as
    kmer_spans.R:76-77 does)."""
    k = int(k)
    hs = _HostSeqs(seq)
    nk = 4 ** k if 1 <= k <= _lib.KS_MAX_K else 1
    counts = np.zeros(nk, dtype=np.int32)
    ranks = np.zeros(nk, dtype=np.float64)
    n = np.zeros(2, dtype=np.float64)
    r = Regions()
    check(load().ks_low_comp_regions(_ctx(device), hs.ptrs, hs.lens.ctypes.data, hs.n, k, int(min_w),
                                     float(min_score), float(thr), counts.ctypes.data,
                                     ranks.ctypes.data, n.ctypes.data, C.byref(r)))
    pos, score = regions_to_numpy(r)
    return {"n": n, "counts": counts, "w_rank": ranks, "pos": pos.T.copy(), "score": score.T.copy()}


def lr_regions(seq, params, kmers, kmer_scores, trans_scores, device: int = 0) -> dict:
    """lr.regions (kmer_spans.R:88-99) -> tr_lr_regions_r (kmer_spans.c:649-713):
    {'kmer_scores': float64[4^k, 2] (the scores remapped to 2-bit code order,
    rows named by kmer_seq(k)), 'reg': {'seq_i', 'beg', 'end', 'score', 'null'}}
    with 1-based sequence indices and positions, as the reference returns them.
    params = (k, min_length); kmers[i] spells entry i of both score vectors."""
    if len(params) != 2:
        raise KmerSpansError("params_r should have two integers (k, and min_length)")
    k, min_length = int(params[0]), int(params[1])
    hs = _HostSeqs(seq)
    ks_in = np.ascontiguousarray(kmer_scores, dtype=np.float64).ravel()
    tr_in = np.ascontiguousarray(trans_scores, dtype=np.float64).ravel()
    n = len(kmers)
    if ks_in.size != n or tr_in.size != n:
        raise KmerSpansError("kmers_r, freq_a, freq_b should all be 4^k long")
    bufs = [C.create_string_buffer(x.encode("latin-1") if isinstance(x, str) else bytes(x)) for x in kmers]
    kptrs = (C.c_char_p * max(n, 1))(*[C.cast(b, C.c_char_p) for b in bufs])
    nk = 4 ** k if 1 <= k <= _lib.KS_MAX_K else 1
    spectra = np.zeros(2 * nk, dtype=np.float64)
    r = Regions()
    check(load().ks_tr_lr_regions(_ctx(device), hs.ptrs, hs.lens.ctypes.data, hs.n, k, min_length, kptrs,
                                  ks_in.ctypes.data, tr_in.ctypes.data, n, spectra.ctypes.data, C.byref(r)))
    pos, score = regions_to_numpy(r)
    reg = {"seq_i": pos[0], "beg": pos[1], "end": pos[2], "score": score[0], "null": score[1]}
    return {"kmer_scores": spectra.reshape(2, nk).T.copy(), "reg": reg, "pos": pos, "score": score}


# ------------------------------------------------------------ table builders

def _table(fn, counts, k):
    counts = np.ascontiguousarray(counts, dtype=np.int32)
    out = np.zeros(4 ** int(k), dtype=np.float64)
    check(fn(counts.ctypes.data, int(k), out.ctypes.data))
    return out


def log2_table(counts, k: int) -> np.ndarray:
    """log2(f / f_med) with f = counts / sum(counts) (README.md:27-29)."""
    return _table(load().ks_log2_table, counts, k)


def pm1_table(counts, k: int) -> np.ndarray:
    """ifelse(f >= f_med, 1, -1) (README.md:37-42)."""
    return _table(load().ks_pm1_table, counts, k)


def rank_table(counts, k: int, total: float) -> np.ndarray:
    """Weighted rank (rank_kmers_w, kmer_spans.c:189-202)."""
    counts = np.ascontiguousarray(counts, dtype=np.int32)
    out = np.zeros(4 ** int(k), dtype=np.float64)
    check(load().ks_rank_table(counts.ctypes.data, int(k), float(total), out.ctypes.data))
    return out


KMER_MAGIC = 310572  # kmer.magic(), kmer_spans.R:5


def kmer_magic() -> int:
    return KMER_MAGIC


def read_fasta(path, min_len: int = 0, device: int = 0):
    """Read a (plain or gzip) FASTA file, parsed on the GPU: returns
    (names, sequences) with the sequences upper-cased, records shorter than
    min_len dropped."""
    from . import device as D
    fa = D.load_fasta(None if int(device) == 0 else _lib.context(device), path, min_len)
    try:
        return fa.names, [b.decode("latin-1") for b in fa.host_seqs()]
    finally:
        fa.close()


def kmers_to_file(seq_f, out_prefix, k, min_l=1e5, magic: int = KMER_MAGIC, device: int = 0) -> list:
    """kmers.to.file: count every k of seq_f's records of length >= min_l into
    <out_prefix>counts_<k...>.bin.  Returns [seq_f, out_f or None (R's NA),
    seq.size, seq.fsize, seq.fl] like the reference's list."""
    ks = np.atleast_1d(np.asarray(k)).astype(np.int32)
    info = _lib.KmerFileInfo()
    check(load().ks_kmers_to_file(_ctx(device), str(seq_f).encode(), str(out_prefix).encode(), ks.ctypes.data,
                                  int(ks.size), float(min_l), int(magic), C.byref(info)))
    out_f = info.out_path.decode() if info.written else None
    return [seq_f, out_f, info.seq_size, info.seq_fsize, info.seq_fl]


def read_kmers(fname, magic: int = KMER_MAGIC):
    """read.kmers: {'k': int array, 'counts': [int32 arrays]} or False."""
    cf = _lib.CountFile()
    check(load().ks_count_file_read(str(fname).encode(), int(magic), C.byref(cf)))
    try:
        if not cf.valid:
            return False
        nk = int(cf.nk)
        ks = np.array([cf.k[i] for i in range(nk)], dtype=np.int32)
        counts = [np.ctypeslib.as_array(cf.counts[i], shape=(int(cf.lens[i]),)).copy() if cf.lens[i] else
                  np.zeros(0, dtype=np.int32) for i in range(nk)]
        return {"k": ks, "counts": counts}
    finally:
        load().ks_count_file_free(C.byref(cf))


def write_kmers(fname, ks, counts, magic: int = KMER_MAGIC) -> None:
    """Write a count file in kmers.to.file's format from host count vectors."""
    ks = np.atleast_1d(np.asarray(ks)).astype(np.int32)
    arrs = [np.ascontiguousarray(c, dtype=np.int32) for c in counts]
    for kk, a in zip(ks, arrs):
        if a.size != 4 ** int(kk):
            raise KmerSpansError(f"counts for k={int(kk)} must have 4^k entries")
    ptrs = (C.c_void_p * max(len(arrs), 1))(*[a.ctypes.data for a in arrs])
    check(load().ks_count_file_write(str(fname).encode(), int(magic), int(ks.size), ks.ctypes.data, ptrs))


def r_recycled_freq(dist: np.ndarray) -> np.ndarray:
    """window.kmer.dist's `dist / colSums(dist)` (kmer_spans.R:116) with R's
    recycling: the column-major elements are divided by colSums repeated
    along them, so element [r, c] of an (n x m) matrix is divided by
    colSums[(r + c * n) % m] -- per-column normalisation only when n % m == 0
    happens to align, as R computes it."""
    dist = np.asarray(dist, dtype=np.float64)
    flat = dist.flatten(order="F")
    cs = dist.sum(axis=0)
    return (flat / np.resize(cs, flat.size)).reshape(dist.shape, order="F")


def window_kmer_dist(seq, kmers, window: int, freq: bool = True, ret_flag: int = 0, device: int = 0) -> dict:
    """window.kmer.dist: {'dist': (window + 1) x kmer_n (counts, or R's
    recycled ratios when freq), 'seq_i': int per sequence, 'scores': None or
    per sequence an int32 [len x kmer_n] matrix (None where excluded)}.
    Column j corresponds to kmers[j]."""
    kmers = [kmers] if isinstance(kmers, (str, bytes)) else list(kmers)
    kb = [x.encode() if isinstance(x, str) else bytes(x) for x in kmers]
    if len(set(len(x) for x in kb)) != 1:
        raise KmerSpansError("All kmers must be of the same size")
    k = len(kb[0])
    hs = _HostSeqs(seq)
    n = len(kb)
    window = int(window)
    if window < 0:
        raise KmerSpansError("The window size must be at least two times k")
    dist = np.zeros((n, window + 1), dtype=np.int32)
    inc = np.zeros(max(hs.n, 1), dtype=np.int32)
    kp = (C.c_char_p * n)(*kb)
    scores = None
    sp = None
    if ret_flag & 1:
        scores = [np.zeros((n, int(L)), dtype=np.int32) if L > window else None for L in hs.lens[:hs.n]]
        sp = (C.c_void_p * max(hs.n, 1))(*[s.ctypes.data if s is not None else None for s in scores])
    check(load().ks_windowed_dist(_ctx(device), hs.ptrs, hs.lens.ctypes.data, hs.n, kp, n, k, window,
                                  int(ret_flag), dist.ctypes.data, inc.ctypes.data, sp))
    d = dist.T.copy()
    if freq:
        d = r_recycled_freq(d)
    return {"dist": d, "seq_i": inc[:hs.n].copy(),
            "scores": [s.T.copy() if s is not None else None for s in scores] if scores is not None else None}
