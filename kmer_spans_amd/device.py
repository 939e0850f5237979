"""Device-resident sequences and tables (the hot path with inputs in HBM).

PyTorch is used only as the device allocator and stream provider: a genome is
one ``torch.uint8`` CUDA tensor holding the concatenated sequences plus an
int64 offsets array (host and device copies).  All compute goes through
libkmerspans.so (ks_scan_dev / ks_count_dev / ks_table_create).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import DevSeqs, Fasta, Regions, ScanStats, check, load, regions_to_numpy


@dataclass
class DeviceSeqs:
    seq: torch.Tensor          # uint8 [total + pad] on cuda
    offsets: np.ndarray        # int64 [nseq + 1] host
    offsets_dev: torch.Tensor  # int64 [nseq + 1] on cuda

    @property
    def nseq(self) -> int:
        return int(self.offsets.size - 1)

    @property
    def total(self) -> int:
        return int(self.offsets[-1])

    def struct(self) -> DevSeqs:
        s = DevSeqs()
        s.seq = self.seq.data_ptr()
        s.offsets_host = self.offsets.ctypes.data
        s.offsets_dev = self.offsets_dev.data_ptr()
        s.nseq = self.nseq
        return s

    def host_seq(self, q: int) -> bytes:
        a, b = int(self.offsets[q]), int(self.offsets[q + 1])
        return self.seq[a:b].cpu().numpy().tobytes()

    def subset(self, ids) -> "DeviceSeqs":
        """A new DeviceSeqs holding the given sequences (device copy)."""
        parts = [self.seq[int(self.offsets[q]):int(self.offsets[q + 1])] for q in ids]
        lens = [int(self.offsets[q + 1] - self.offsets[q]) for q in ids]
        return from_parts(parts, lens, self.seq.device)


def _pad16(n: int) -> int:
    return (n + 16 + 15) // 16 * 16


def from_parts(parts, lens, device) -> DeviceSeqs:
    offs = np.zeros(len(lens) + 1, dtype=np.int64)
    offs[1:] = np.cumsum(np.asarray(lens, dtype=np.int64))
    buf = torch.empty(_pad16(int(offs[-1])), dtype=torch.uint8, device=device)
    buf[int(offs[-1]):] = ord("N")
    for p, a, b in zip(parts, offs[:-1], offs[1:]):
        if b > a:
            buf[int(a):int(b)].copy_(p)
    return DeviceSeqs(buf, offs, torch.from_numpy(offs).to(device))


def from_host(seqs, device="cuda") -> DeviceSeqs:
    """Upload a list of str/bytes sequences."""
    bs = [s.encode("latin-1") if isinstance(s, str) else bytes(s) for s in seqs]
    lens = [len(b) for b in bs]
    parts = [torch.frombuffer(bytearray(b), dtype=torch.uint8) if b else torch.empty(0, dtype=torch.uint8)
             for b in bs]
    return from_parts(parts, lens, device)


class DeviceTable:
    """A score table s = w - thr on the device (ks_table)."""

    def __init__(self, ctx: _lib.Context, w, k: int, thr: float = 0.0, compress: bool = True,
                 expand: bool = False, freq: torch.Tensor | None = None):
        """freq: optional k-mer counts (int32[4^k], cuda) of the sequences to be
        scanned -- a hint for the expanded table's short codes, never the results."""
        w = np.ascontiguousarray(w, dtype=np.float64)
        if w.size != 4 ** k:
            raise _lib.KmerSpansError(f"kmer_w contains {w.size} elements but should have {4 ** k}")
        if freq is not None and (freq.dtype != torch.int32 or freq.numel() != 4 ** k or not freq.is_cuda):
            raise _lib.KmerSpansError("freq must be an int32 cuda tensor of 4^k counts")
        self.k = k
        self._h = C.c_void_p()
        flags = (1 if compress else 0) | (2 if expand else 0)
        if freq is not None:
            _order(ctx)
        check(load().ks_table_create_hint(ctx.handle, w.ctypes.data, k, float(thr), flags,
                                          C.c_void_p(freq.data_ptr()) if freq is not None else None,
                                          C.byref(self._h)))

    @classmethod
    def from_counts(cls, ctx: _lib.Context, counts: torch.Tensor, k: int, score: str, total: float = 0.0,
                    thr: float = 0.0, compress: bool = True, expand: bool = False, max_ext_bytes: int = 0,
                    w_out: torch.Tensor | None = None) -> "DeviceTable":
        """ks_table_from_counts: the log2 / pm1 / rank table of device counts
        (int32[4^k] cuda) built on the device; w_out (float64[4^k] cuda, optional)
        receives w.  total: the word count (rank only)."""
        if counts.dtype != torch.int32 or counts.numel() != 4 ** k or not counts.is_cuda:
            raise _lib.KmerSpansError("counts must be an int32 cuda tensor of 4^k counts")
        if w_out is not None and (w_out.dtype != torch.float64 or w_out.numel() != 4 ** k or not w_out.is_cuda):
            raise _lib.KmerSpansError("w_out must be a float64 cuda tensor of 4^k values")
        self = cls.__new__(cls)
        self.k = k
        self._h = C.c_void_p()
        flags = (1 if compress else 0) | (2 if expand else 0)
        _order(ctx)
        check(load().ks_table_from_counts(ctx.handle, C.c_void_p(counts.data_ptr()), int(k), _lib.SCORES[score],
                                          float(total), float(thr), flags, int(max_ext_bytes),
                                          C.c_void_p(w_out.data_ptr()) if w_out is not None else None,
                                          C.byref(self._h)))
        return self

    def info(self) -> dict:
        """ks_table_get_info: shape and setup cost (ms) of the table."""
        inf = _lib.TableInfo()
        check(load().ks_table_get_info(self._h, C.byref(inf)))
        return inf.as_dict()

    def setup_ms(self) -> dict:
        """Setup time of this table by phase (ms; host wall clock around the
        synchronised device work)."""
        inf = self.info()
        return {key[3:]: round(v, 3) for key, v in inf.items() if key.startswith("ms_")}

    @property
    def code_bits(self) -> int:
        return int(load().ks_table_code_bits(self._h))

    @property
    def escape_fraction(self) -> float:
        return float(load().ks_table_escape_fraction(self._h))

    @property
    def compressed(self) -> bool:
        return bool(load().ks_table_is_compressed(self._h))

    @property
    def positions_per_read(self) -> int:
        return int(load().ks_table_positions_per_read(self._h))

    @property
    def line_kind(self) -> int:
        """0: no line table; 1: uint16 64-B lines (k_pass1l); 2: FP64 64-B lines
        (k_pass1l); 3: 128-B lines (k_pass1w); 4: weighted-rank 128-B code lines
        for pass 1 (k_pass1r) beside FP64 64-B lines for the later passes."""
        return int(self.info()["line_kind"])

    @property
    def pass1_kernel(self) -> str:
        """The pass-1 kernel the chunked scan runs on this table."""
        lk = self.line_kind
        if self.k <= 7 and not os.environ.get("KS_NO_LDS_TABLE"):  # (scan_chunked: the table staged in LDS first)
            return "k_pass1_lds"
        if lk == 3:
            return "k_pass1w"
        if lk == 4:
            return "k_pass1r"
        if lk:
            return "k_pass1l"
        if self.positions_per_read > 1:
            return "k_pass1p" if self.compressed else "k_pass1pf"
        return "k_pass1"

    @property
    def distinct(self) -> int:
        return int(load().ks_table_distinct(self._h))

    def close(self):
        if self._h:
            load().ks_table_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def bind_torch_stream(ctx: _lib.Context) -> None:
    """Run library work on torch's current stream (ordering with torch ops)."""
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)


def _order(ctx) -> None:
    """Make torch's pending work on the buffers we are handed visible to the
    ctx's stream: a no-op when the ctx runs on torch's current stream (see
    bind_torch_stream), otherwise a wait for torch's stream.  Every library
    call synchronises its own stream before returning, so results are ready
    for torch afterwards."""
    if ctx is None or getattr(ctx, "stream", -1) != torch.cuda.current_stream().cuda_stream:
        torch.cuda.current_stream().synchronize()


def scan(ctx: _lib.Context, ds: DeviceSeqs, k: int, table: DeviceTable, min_width: int, min_score: float,
         visits: torch.Tensor | None = None):
    """ks_scan_dev: returns (pos int32[3, R], score float64[2, R], stats dict)."""
    st = ScanStats()
    r = Regions()
    s = ds.struct()
    _order(ctx)
    check(load().ks_scan_dev(ctx.handle, C.byref(s), int(k), table._h, int(min_width), float(min_score),
                             C.c_void_p(visits.data_ptr()) if visits is not None else None, C.byref(r),
                             C.byref(st)))
    pos, score = regions_to_numpy(r)
    return pos, score, st.as_dict()


def tr_lr(ctx: _lib.Context, ds: DeviceSeqs, k: int, trans: DeviceTable, init: DeviceTable, min_length: int):
    """ks_tr_lr_dev: tr_lr regions (1-based, as tr_lr_regions_r) of
    device-resident sequences; trans / init tables with threshold 0 (init
    built with compress=False).  Returns (pos int32[3, R], score float64[2, R], stats)."""
    st = ScanStats()
    r = Regions()
    s = ds.struct()
    _order(ctx)
    check(load().ks_tr_lr_dev(ctx.handle, C.byref(s), int(k), trans._h, init._h, int(min_length), C.byref(r),
                              C.byref(st)))
    pos, score = regions_to_numpy(r)
    return pos, score, st.as_dict()


def count(ctx: _lib.Context, ds: DeviceSeqs, k: int, counts: torch.Tensor) -> float:
    """ks_count_dev: accumulates into counts (int32[4^k] cuda); returns #words."""
    n = C.c_double(0)
    s = ds.struct()
    _order(ctx)
    check(load().ks_count_dev(ctx.handle, C.byref(s), int(k), C.c_void_p(counts.data_ptr()), C.byref(n)))
    return n.value


class FastaSeqs:
    """Records of a FASTA file parsed on the device (ks_fasta_load /
    ks_fasta_parse): usable wherever a DeviceSeqs is (scan, tr_lr, count).
    The device buffers belong to the library and are freed by close()."""

    def __init__(self, f: Fasta):
        self._f = f
        n = int(f.seqs.nseq)
        self.offsets = (np.ctypeslib.as_array(C.cast(f.seqs.offsets_host, C.POINTER(C.c_int64)), shape=(n + 1,)).copy()
                        if n else np.zeros(1, dtype=np.int64))
        self.names = [f.names[q].decode("latin-1") for q in range(n)]
        self.n_records = int(f.n_records)
        self.bases_all = int(f.bases_all)
        self.bases_kept = int(f.bases_kept)
        self.ms_upload = float(f.ms_upload)
        self.ms_parse = float(f.ms_parse)

    @property
    def nseq(self) -> int:
        return int(self.offsets.size - 1)

    @property
    def total(self) -> int:
        return int(self.offsets[-1])

    def struct(self) -> DevSeqs:
        if self._f is None:
            raise ValueError("FastaSeqs is closed")
        return self._f.seqs

    def host_bytes(self) -> bytes:
        """All kept records' bytes, concatenated (device -> host copy)."""
        buf = np.empty(max(self.total, 1), dtype=np.uint8)
        check(load().ks_fasta_copy_seqs(C.byref(self._f), buf.ctypes.data))
        return buf[:self.total].tobytes()

    def host_seqs(self) -> list[bytes]:
        b = self.host_bytes()
        return [b[int(a):int(e)] for a, e in zip(self.offsets[:-1], self.offsets[1:])]

    def close(self):
        if self._f is not None:
            load().ks_fasta_free(C.byref(self._f))
            self._f = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_fasta(ctx: _lib.Context | None, path: str, min_len: int = 0) -> FastaSeqs:
    """ks_fasta_load: plain or gzip FASTA -> device-resident records."""
    f = Fasta()
    check(load().ks_fasta_load(ctx.handle if ctx is not None else None, str(path).encode(), int(min_len),
                               C.byref(f)))
    return FastaSeqs(f)


def parse_fasta(ctx: _lib.Context | None, text, min_len: int = 0) -> FastaSeqs:
    """ks_fasta_parse: FASTA text (str/bytes) -> device-resident records."""
    b = text.encode("latin-1") if isinstance(text, str) else bytes(text)
    f = Fasta()
    check(load().ks_fasta_parse(ctx.handle if ctx is not None else None, b, len(b), int(min_len), C.byref(f)))
    return FastaSeqs(f)


def count_multi(ctx: _lib.Context, ds, ks, counts) -> list[float]:
    """ks_count_multi_dev: one pass for several k; counts[i] int32[4^ks[i]]
    cuda tensors (accumulated).  Returns the words counted per k."""
    ks = np.ascontiguousarray(ks, dtype=np.int32)
    ptrs = (C.c_void_p * max(len(ks), 1))(*[c.data_ptr() for c in counts])
    words = np.zeros(max(len(ks), 1), dtype=np.float64)
    s = ds.struct()
    _order(ctx)
    check(load().ks_count_multi_dev(ctx.handle, C.byref(s), ks.ctypes.data, len(ks), ptrs, words.ctypes.data))
    return [float(w) for w in words[:len(ks)]]


def windowed(ctx: _lib.Context, ds, kmer_codes, k: int, window: int, dist: torch.Tensor,
             included: torch.Tensor | None = None, scores: torch.Tensor | None = None) -> None:
    """ks_windowed_dev: dist int32 [kmer_n, window + 1] cuda (accumulated; row
    i = query i), included int32 [nseq] cuda or None, scores int32 cuda
    [kmer_n * total] (zeroed; per sequence q the [kmer_n][len_q] block at
    kmer_n * offsets[q]) or None."""
    codes = np.ascontiguousarray(kmer_codes, dtype=np.uint32)
    if dist.dtype != torch.int32 or dist.numel() != codes.size * (int(window) + 1) or not dist.is_cuda:
        raise _lib.KmerSpansError("dist must be an int32 cuda tensor of kmer_n * (window + 1)")
    if scores is not None and (scores.dtype != torch.int32 or scores.numel() < codes.size * ds.total):
        raise _lib.KmerSpansError("scores must be an int32 cuda tensor of kmer_n * total")
    if included is not None and (included.dtype != torch.int32 or included.numel() < ds.nseq):
        raise _lib.KmerSpansError("included must be an int32 cuda tensor of nseq")
    s = ds.struct()
    _order(ctx)
    check(load().ks_windowed_dev(ctx.handle, C.byref(s), codes.ctypes.data, int(codes.size), int(k), int(window),
                                 C.c_void_p(dist.data_ptr()),
                                 C.c_void_p(included.data_ptr()) if included is not None else None,
                                 C.c_void_p(scores.data_ptr()) if scores is not None else None))
