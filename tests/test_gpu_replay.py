"""Replays of the exact call sequences behind the round-4 intermittent
host-entry failures, on the default context,
under the memory policy those runs had (0: every host call allocates its
workspace afresh and returns it at the end) and under the default (2).

1. The random kmer_regions corpus: 300 cases of the lane-per-run scan
   (seed 11), then the chunked scan (seed 12) through case 268 -- the case that
   returned four regions where the oracle has none (a k = 4 table with NaN and
   +-Inf values, 24 chunks).
2. Config 1 (1 Mbp uniform, k = 7, +-1 table from its own counts) after the
   random count and low-complexity corpora -- the call whose 1 Mbp excursion
   restarted at index 208,714.

Every call is checked against the oracle, region by region and bit for bit
(reference: kmer_regions_r / kmer_low_comp_regions, kmer_spans.c:490-546,
548-621)."""
import random

import numpy as np
import pytest

from tests.test_gpu_parity import _assert_same_regions, _random_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[0, 2], ids=["policy0", "policy2"])
def policy(request):
    from kmer_spans_amd import _lib
    L = _lib.load()
    assert L.ks_set_host_cache(request.param) == 0
    try:
        yield request.param
    finally:
        L.ks_set_host_cache(2)


@pytest.fixture(scope="module")
def K():
    import kmer_spans_amd as K
    return K


def _algo(a):
    from kmer_spans_amd import _lib
    L = _lib.load()
    _lib.check(L.ks_ctx_set_scan_algo(L.ks_default_ctx(), a))


def test_replay_random_corpus_through_case_268(K, oracle, policy):
    try:
        for algo, seed, n in ((0, 11, 300), (1, 12, 269)):
            _algo(algo)
            rng = random.Random(seed)
            for case in range(n):
                k, seqs, w, mw, ms = _random_inputs(rng)
                g = K.kmer_regions(seqs, k, w, mw, ms)
                o = oracle.kmer_regions(seqs, k, w, mw, ms)
                _assert_same_regions(g["pos"], g["score"], o["pos"], o["score"], (algo, case, k, mw, ms))
                assert np.array_equal(g["counts"], o["counts"]), (algo, case)
        # case 268 of the chunked scan: the oracle's answer is no region
        assert g["pos"].shape == (3, 0)
    finally:
        _algo(-1)


def test_replay_config1_after_low_comp_corpus(K, oracle, policy):
    from kmer_spans_amd import genome
    rng = random.Random(5)
    for _ in range(200):
        k = rng.randint(1, 9)
        seqs = ["".join(rng.choice(rng.choice(["ACGT", "ACGTNacgtn", "NNNNA"])) for _ in range(rng.randint(0, 300)))
                for _ in range(rng.randint(1, 4))]
        g = K.kmer_counts(seqs, k)
        n, c = oracle.kmer_counts(seqs, k)
        assert g["n"]["n"] == n and np.array_equal(g["counts"], c), (seqs, k)
    rng = random.Random(9)
    for _ in range(120):
        k = rng.randint(1, 6)
        seqs = ["".join(rng.choice("ACGTN" if rng.random() < 0.3 else "ACGT") for _ in range(rng.randint(0, 400)))
                for _ in range(rng.randint(1, 3))]
        thr = rng.choice([0.5, 0.75, 0.9])
        mw, ms = rng.randint(0, 20), rng.choice([0.0, 2.0, 5.0])
        g = K.kmer_low_comp_regions(seqs, k, mw, ms, thr)
        o = oracle.low_comp_regions(seqs, k, mw, ms, thr)
        assert np.array_equal(g["counts"], o["counts"])
        _assert_same_regions(g["pos"].T, g["score"].T, o["pos"], o["score"], (seqs, k, thr))
    s = genome.uniform_xorshift(1_000_000, 1)
    c = K.kmer_counts(s, 7)
    w = K.pm1_table(c["counts"], 7)
    g = K.kmer_regions(s, 7, w, 100, 20)
    o = oracle.kmer_regions(s, 7, w, 100, 20)
    _assert_same_regions(g["pos"], g["score"], o["pos"], o["score"], "config1 after the corpora")
    assert np.array_equal(g["counts"], o["counts"])
    # the excursion from index 27 to the end (the one that restarted at 208,714)
    assert g["pos"][:, 0].tolist() == o["pos"][:, 0].tolist()
