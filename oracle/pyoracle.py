"""Pure-Python second restatement of the span scan -- TEST INFRASTRUCTURE ONLY.

Where oracle/ks_oracle.c follows the reference's restart loop literally
(kmer_regions, /root/reference/src/kmer_spans.c:243-307), this module uses the
excursion decomposition the HIP path is built on (SURVEY.md 8(a) row a5'):

  per N-free run, scored indices i in [a+k, b-1] (the k-mer ending at i-1);
  a range scan S_i = max(S_{i-1} + s_i, 0) yields excursions
  (beg, first argmax, max, end) where end is the reset index (S back to 0) or
  the last index of the range; an excursion passing the emit test produces a
  region and a fresh rescan of (argmax, end]; every scanned index counts one
  visit for its k-mer.

Agreement of the two restatements on random inputs (tests/test_oracle.py) is
what licenses the decomposition.  Pure-Python loops: small inputs only.
"""
from __future__ import annotations

import numpy as np


def _is_n(c: int) -> bool:
    return (c | 0x20) == 0x6E


def runs(s: bytes, k: int):
    """Maximal N-free runs [a, b) with at least one scored index (b - a > k)."""
    out, i, L = [], 0, len(s)
    while i < L:
        while i < L and _is_n(s[i]):
            i += 1
        a = i
        while i < L and not _is_n(s[i]):
            i += 1
        if i - a > k:
            out.append((a, i))
    return out


def kmer_codes(s: bytes, a: int, b: int, k: int):
    """code[i] for i in [a+k, b-1]: 2-bit code of bases [i-k, i-1]."""
    mask = (1 << (2 * k)) - 1
    codes = {}
    c = 0
    for j in range(a, b - 1):
        c = ((c << 2) | ((s[j] >> 1) & 3)) & mask
        if j - a + 1 >= k:
            codes[j + 1] = c
    return codes


def scan_range(vals, lo: int, hi: int):
    """Clamp scan over indices lo..hi (inclusive) with fresh state.
    Returns excursions [(beg, arg, best, end)], end = reset index or hi."""
    exc = []
    S = 0.0
    open_ = None
    for i in range(lo, hi + 1):
        prev = S
        t = prev + vals[i]
        S = t if t > 0 else 0.0
        if prev == 0 and S > 0:
            open_ = [i, i, S]
        elif open_ is not None:
            if S == 0:
                exc.append((open_[0], open_[1], open_[2], i))
                open_ = None
            elif S > open_[2]:
                open_[1], open_[2] = i, S
    if open_ is not None:
        exc.append((open_[0], open_[1], open_[2], hi))
    return exc


def regions(seqs, k: int, w, thr: float, min_width: int, min_score: float):
    """Regions (list of (seq_id, beg, end, score)) and the visit histogram."""
    w = np.asarray(w, dtype=np.float64)
    visits = np.zeros(4 ** k, dtype=np.int64)
    mw = min_width if min_width >= 0 else (1 << 64) + min_width  # size_t compare
    out = []
    for q, s in enumerate(seqs):
        s = s.encode("latin-1") if isinstance(s, str) else bytes(s)
        if len(s) < k:
            continue
        regs = []
        for a, b in runs(s, k):
            codes = kmer_codes(s, a, b, k)
            vals = {i: float(np.float64(w[c]) - np.float64(thr)) for i, c in codes.items()}
            work = [(a + k, b - 1)]
            while work:
                lo, hi = work.pop()
                for i in range(lo, hi + 1):
                    visits[codes[i]] += 1
                for beg, arg, best, end in scan_range(vals, lo, hi):
                    if (arg - beg) >= mw and best >= min_score:
                        regs.append((q, beg, arg, best))
                        if arg + 1 <= end:
                            work.append((arg + 1, end))
        regs.sort(key=lambda r: r[1])
        out.extend(regs)
    return out, visits.astype(np.uint32).view(np.int32)


# ----------------------------------------------------------- tr_lr regions
#
# find_kmer_tr_lr_regions (kmer_spans.c:329-395) in decomposition form, the
# form the HIP path implements.  Per N-free run [a, b) the steps are: the first
# k-mer's kmer score at position a+k, then the transition score of the k-mer
# ending at each position a+k .. b-1.  A clamp scan over those steps gives
# excursions (beg, first argmax, max, end); every excursion passing
# (pos(argmax) - pos(beg)) >= min_len is a region, and every CLOSED excursion
# (emitted or not) spawns a fresh rescan of positions (pos(argmax), pos(end)]
# with transition scores only; an excursion still open at the run end spawns
# nothing.  A run whose first k-mer ends within the last two bytes of the
# string is skipped (:341).  Finite tables only (NaN persists in the
# reference and is exercised against the literal oracle instead).

def _scan_steps(vals):
    """Clamp scan; excursions [(beg, arg, best, end|None)] over step indices."""
    exc = []
    S = 0.0
    open_ = None
    for i, v in enumerate(vals):
        prev = S
        t = prev + v
        S = t if t > 0 else 0.0
        if prev == 0 and S > 0:
            open_ = [i, i, S]
        elif open_ is not None:
            if S == 0:
                exc.append((open_[0], open_[1], open_[2], i))
                open_ = None
            elif S > open_[2]:
                open_[1], open_[2] = i, S
    if open_ is not None:
        exc.append((open_[0], open_[1], open_[2], None))
    return exc


def trlr_regions(seqs, k: int, min_len: int, ks, tr):
    """1-based regions [(seq_id, beg, end, score)] of tr_lr_regions_r."""
    ks = np.asarray(ks, dtype=np.float64)
    tr = np.asarray(tr, dtype=np.float64)
    mask = (1 << (2 * k)) - 1
    out = []
    for q, s in enumerate(seqs):
        s = s.encode("latin-1") if isinstance(s, str) else bytes(s)
        L = len(s)

        def kmer_end(p):  # code of bases [p-k+1, p]
            c = 0
            for j in range(p - k + 1, p + 1):
                c = (c << 2) | ((s[j] >> 1) & 3)
            return c & mask

        regs = []
        i = 0
        while i < L:
            while i < L and _is_n(s[i]):
                i += 1
            a = i
            while i < L and not _is_n(s[i]):
                i += 1
            b = i
            if b - a < k or a + k + 1 >= L:  # :341, the string ends within a base of the k-mer
                continue
            pos = [a + k] + list(range(a + k, b))
            vals = [float(ks[kmer_end(a + k - 1)])] + [float(tr[kmer_end(p)]) for p in range(a + k, b)]
            work = [(pos, vals, True)]
            while work:
                ps, vs, top = work.pop()
                for beg, arg, best, end in _scan_steps(vs):
                    pb, pa = ps[beg], ps[arg]
                    if pa - pb >= min_len:
                        regs.append((q + 1, pb + 1, pa + 1, best))
                    if end is None:
                        assert top, "a rescan ends at 0 (coalescence)"
                        continue
                    pe = ps[end]
                    if pa + 1 <= pe:
                        rp = list(range(pa + 1, pe + 1))
                        work.append((rp, [float(tr[kmer_end(p)]) for p in rp], False))
        regs.sort(key=lambda r: r[1])
        out.extend(regs)
    return out
