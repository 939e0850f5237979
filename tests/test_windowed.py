"""Windowed k-mer count distributions:
windowed_kmer_count_distributions(_r) (kmer_spans.c:413-449, 717-793) and
window.kmer.dist (kmer_spans.R:103-118).

Pinning: tests/golden/windowed_kats.json holds the two known answers the
reference's own test.R records in comments (:373-439); the C oracle
(oracle/ks_oracle.c orc_windowed_dist, a restatement of the reference loop)
reproduces both, and an independent brute-force restatement below agrees
with it on random inputs.  GPU tests compare the HIP path with the oracle
bit-exactly (integer histograms and per-position counts).
"""
import json
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def kats():
    with open(os.path.join(ROOT, "tests", "golden", "windowed_kats.json")) as f:
        return json.load(f)


def _code(s, k):
    """init_kmer (kmer_spans.c:119-132) on a k-character query: the first k
    non-N bytes after skipping N runs; a short tail leaves the partial code."""
    c, j, i = 0, 0, 0
    b = s.encode() if isinstance(s, str) else s
    while i < len(b):
        c, j = 0, 0
        while j < k and i + j < len(b) and (b[i + j] | 0x20) != ord("n"):
            c = (c << 2) | ((b[i + j] >> 1) & 3)
            j += 1
        if i + j >= len(b) or j == k:
            break
        i += j
        while i < len(b) and (b[i] | 0x20) == ord("n"):
            i += 1
    return c


def brute_windowed(seqs, kmers, k, window):
    """Independent restatement: every N-free run [a, b), every window start
    s in [a, b - window], count the query's k-mers ending in
    [s + k - 1, s + window - 1]."""
    codes = [_code(q, k) for q in kmers]
    dist = np.zeros((window + 1, len(kmers)), dtype=np.int64)
    scores = []
    mask = (1 << (2 * k)) - 1
    for s in seqs:
        b = s.encode() if isinstance(s, str) else s
        L = len(b)
        sc = np.zeros((L, len(kmers)), dtype=np.int64) if L > window else None
        scores.append(sc)
        if L <= window:
            continue
        # k-mer code ending at each position (None where the k bases are not N-free)
        ends = [None] * L
        run = 0
        c = 0
        for p in range(L):
            if (b[p] | 0x20) == ord("n"):
                run, c = 0, 0
                continue
            c = ((c << 2) | ((b[p] >> 1) & 3)) & mask
            run += 1
            if run >= k:
                ends[p] = c
        p = 0
        while p < L:
            if (b[p] | 0x20) == ord("n"):
                p += 1
                continue
            a = p
            while p < L and (b[p] | 0x20) != ord("n"):
                p += 1
            for st in range(a, p - window + 1):
                for i, q in enumerate(codes):
                    n = sum(1 for e in range(st + k - 1, st + window) if ends[e] == q)
                    dist[n, i] += 1
                    sc[st, i] = n
    return dist, scores


# ------------------------------------------------------------------- CPU

def test_oracle_reproduces_test_r_kats(oracle, kats):
    for case in kats["cases"]:
        km = list(case["expect"])
        r = oracle.windowed_dist(case["seq"], km, case["k"], case["window"], 1)
        for i, m in enumerate(km):
            assert r["dist"][:case["window"], i].tolist() == case["expect"][m], m
        assert r["seq_i"].tolist() == [1]


def test_oracle_matches_brute_force(oracle):
    rng = random.Random(13)
    for _ in range(40):
        k = rng.randint(1, 4)
        window = rng.randint(2 * k, 2 * k + 12)
        seqs = ["".join(rng.choice("ACGTacgtN" if rng.random() < 0.3 else "ACGT") for _ in range(rng.randint(0, 60)))
                for _ in range(rng.randint(1, 3))]
        kmers = ["".join(rng.choice("ACGTN") for _ in range(k)) for _ in range(rng.randint(1, 5))]
        o = oracle.windowed_dist(seqs, kmers, k, window, 1)
        d, sc = brute_windowed(seqs, kmers, k, window)
        assert np.array_equal(o["dist"], d), (seqs, kmers, k, window)
        for a, b in zip(o["scores"], sc):
            assert (a is None and b is None) or np.array_equal(a, b)


def test_oracle_errors(oracle):
    with pytest.raises(oracle.OracleError):
        oracle.windowed_dist(["ACGT"], ["AC"], 2, 3)      # window < 2k
    with pytest.raises(oracle.OracleError):
        oracle.windowed_dist(["ACGT"], ["AC", "A"], 2, 6)  # k-mer of another length
    with pytest.raises(oracle.OracleError):
        oracle.windowed_dist(["ACGT"], ["A" * 16], 16, 40)  # k >= MAX_K


def test_r_recycled_freq():
    """window.kmer.dist(freq=TRUE) divides by colSums with R's recycling."""
    from kmer_spans_amd.api import r_recycled_freq
    d = np.array([[1, 4], [2, 5], [3, 6]], dtype=np.int32)  # 3 x 2, colSums (6, 15)
    # column-major elements 1,2,3,4,5,6 / 6,15,6,15,6,15
    want = np.array([[1 / 6, 4 / 15], [2 / 15, 5 / 6], [3 / 6, 6 / 15]])
    assert np.allclose(r_recycled_freq(d), want, rtol=0, atol=0)


# ------------------------------------------------------------------- GPU

@pytest.mark.gpu
def test_gpu_reproduces_test_r_kats(kats):
    import kmer_spans_amd as K
    for case in kats["cases"]:
        km = list(case["expect"])
        r = K.window_kmer_dist(case["seq"], km, case["window"], freq=False, ret_flag=1)
        for i, m in enumerate(km):
            assert r["dist"][:case["window"], i].tolist() == case["expect"][m], m
        assert r["seq_i"].tolist() == [1]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_windowed_vs_oracle(oracle, seed):
    import kmer_spans_amd as K
    rng = random.Random(100 + seed)
    k = rng.choice([1, 2, 3, 5, 8, 11])
    window = rng.choice([2 * k, 2 * k + 1, 50, 333, 1024, 1500])
    window = max(window, 2 * k)
    seqs = []
    for _ in range(rng.randint(1, 6)):
        L = rng.choice([0, window, window + 1, rng.randint(0, 6000), rng.randint(0, 30000)])
        seqs.append("".join(rng.choice("ACGTacgtNR") if rng.random() < 0.05 else rng.choice("ACGT")
                            for _ in range(L)))
    alphabet = "ACGT"
    kmers = ["".join(rng.choice(alphabet) for _ in range(k)) for _ in range(rng.choice([1, 5, 16, 17, 40]))]
    kmers[0] = "A" * k
    if len(kmers) > 2:
        kmers[2] = kmers[1]           # duplicate query
        kmers[-1] = "N" * (k - 1) + "A"  # N in a query (init_kmer semantics)
    ret = rng.choice([0, 1])
    o = oracle.windowed_dist(seqs, kmers, k, window, ret)
    g = K.window_kmer_dist(seqs, kmers, window, freq=False, ret_flag=ret)
    assert np.array_equal(g["dist"], o["dist"]), (k, window)
    assert np.array_equal(g["seq_i"], o["seq_i"])
    if ret:
        for a, b in zip(g["scores"], o["scores"]):
            assert (a is None and b is None) or np.array_equal(a, b)
    else:
        assert g["scores"] is None


@pytest.mark.gpu
def test_gpu_windowed_device_entry(oracle):
    import torch
    from kmer_spans_amd import _lib, device as D
    ctx = _lib.context(0)
    rng = random.Random(7)
    seqs = ["".join(rng.choice("ACGT") if rng.random() > 0.002 else "N" for _ in range(rng.randint(5000, 40000)))
            for _ in range(4)]
    k, window = 4, 200
    kmers = ["ACGT", "AAAA", "CGCG", "TTTT", "GATC"]
    o = oracle.windowed_dist(seqs, kmers, k, window, 1)
    ds = D.from_host(seqs)
    dist = torch.zeros((len(kmers), window + 1), dtype=torch.int32, device="cuda")
    inc = torch.zeros(len(seqs), dtype=torch.int32, device="cuda")
    scores = torch.zeros(len(kmers) * ds.total, dtype=torch.int32, device="cuda")
    codes = [_code(x, k) for x in kmers]
    D.windowed(ctx, ds, codes, k, window, dist, inc, scores)
    assert np.array_equal(dist.cpu().numpy().T, o["dist"])
    assert inc.cpu().tolist() == o["seq_i"].tolist()
    sc = scores.cpu().numpy()
    for q, want in enumerate(o["scores"]):
        a, L = int(ds.offsets[q]), int(ds.offsets[q + 1] - ds.offsets[q])
        got = sc[len(kmers) * a: len(kmers) * a + len(kmers) * L].reshape(len(kmers), L).T
        assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_windowed_errors():
    import kmer_spans_amd as K
    with pytest.raises(K.KmerSpansError, match="at least two times k"):
        K.window_kmer_dist(["ACGTACGT"], ["AC"], 3)
    with pytest.raises(K.KmerSpansError, match="same size"):
        K.window_kmer_dist(["ACGTACGT"], ["AC", "A"], 6)
    with pytest.raises(K.KmerSpansError, match="larger than or equal to 16"):
        K.window_kmer_dist(["ACGT" * 20], ["A" * 16], 40)
