"""Pin the CPU oracle (oracle/) against the reference's recorded outputs and
known answers (tests/golden/reference_kats.json), and cross-check its two
independent restatements (restart loop in C vs excursion decomposition in
Python) on random inputs.  CPU only."""
import random

import numpy as np
import pytest


def _regions(r):
    return [[int(r["pos"][0][i]), int(r["pos"][1][i]), int(r["pos"][2][i]), float(r["score"][0][i])]
            for i in range(r["pos"].shape[1])]


def test_golden_counts(oracle, golden):
    for case in golden["kmer_counts"]:
        n, counts = oracle.kmer_counts(case["seq"], case["k"])
        assert n == case["n"], case
        if "counts" in case:
            assert counts.tolist() == case["counts"], case


def test_golden_regions(oracle, golden):
    for case in golden["kmer_regions_r"]:
        r = oracle.kmer_regions(case["seq"], case["k"], case["w"], case["min_width"], case["min_score"])
        assert _regions(r) == case["regions"], case
        assert int(r["counts"].sum()) == case["visits_total"], case
        assert r["n"] == sum(len(s) for s in case["seq"] if len(s) >= case["k"])


def test_golden_low_comp(oracle, golden):
    for case in golden["kmer_low_comp_regions"]:
        r = oracle.low_comp_regions(case["seq"], case["k"], case["min_width"], case["min_score"], case["thr"])
        assert r["w_rank"].tolist() == case["w_rank"]
        assert r["n"].tolist() == case["n"]
        assert _regions(r) == case["regions"]


def test_n_gap_property(oracle):
    """test.R:66-76: counts(seq ++ N*36 ++ seq) == 2 * counts(seq) ('## TRUE')."""
    rng = random.Random(7)
    seqs = ["".join(rng.choice("ACGT") for _ in range(100)) for _ in range(2)]
    seqs.append("AG" * 50 + seqs[0] + seqs[1] + seqs[0])
    ns = "N" * 36
    _, c2 = oracle.kmer_counts(seqs, 2)
    _, c3 = oracle.kmer_counts([s + ns + s for s in seqs], 2)
    assert np.array_equal(c2 * 2, c3)


def test_kmer_seq_order(oracle):
    assert oracle.kmer_seq(1) == ["A", "C", "T", "G"]
    assert oracle.kmer_seq(2)[:5] == ["AA", "AC", "AT", "AG", "CA"]


def test_rank_table_small(oracle):
    # counts A=10, C=3, T=0, G=1 over 14 words (zeroed-allocation reference result)
    r = oracle.rank_table(np.array([10, 3, 0, 1], dtype=np.int32), 1, 14.0)
    order = np.lexsort((np.arange(4), [10, 3, 0, 1]))
    assert order.tolist() == [2, 3, 1, 0]
    assert r[2] == 0.0 and r[3] == 0.0 and r[1] == 1 / 14 and r[0] == 1 / 14 + 3 / 14


def _random_case(rng):
    k = rng.randint(1, 4)
    seqs = []
    for _ in range(rng.randint(1, 3)):
        L = rng.randint(0, 60)
        alpha = rng.choice(["ACGT", "ACGTN", "ACGTNacgtn", "AC", "ACGTNNNN", "ACGTRY"])
        seqs.append("".join(rng.choice(alpha) for _ in range(L)))
    if rng.random() < 0.5:
        w = np.array([rng.randint(-3, 3) for _ in range(4 ** k)], dtype=float)
    else:
        w = np.array([rng.uniform(-2, 1.5) for _ in range(4 ** k)])
    thr = rng.choice([0.0, 0.25, 0.5])
    return k, seqs, w, thr, rng.randint(-1, 5), rng.choice([0.0, 1.0, 2.5, 5.0])


def test_restatements_agree(oracle):
    from oracle import pyoracle as P
    rng = random.Random(1)
    for _ in range(1500):
        k, seqs, w, thr, mw, ms = _random_case(rng)
        r = oracle.scan(seqs, k, w, thr, mw, ms, visits=True)
        regs, vis = P.regions(seqs, k, w, thr, mw, ms)
        assert _regions(r) == [list(x) for x in regs], (seqs, k, thr, mw, ms)
        assert np.array_equal(r["counts"], vis)


def test_counts_match_python(oracle):
    """sequence_kmer_count incl. Q1, against a direct Python enumeration."""
    rng = random.Random(3)
    for _ in range(400):
        k = rng.randint(1, 5)
        seqs = ["".join(rng.choice("ACGTNacgtnX") for _ in range(rng.randint(0, 40))) for _ in range(2)]
        n, c = oracle.kmer_counts(seqs, k)
        ref = np.zeros(4 ** k, dtype=np.int64)
        words = 0
        for s in seqs:
            if len(s) < k:
                continue
            b = s.encode()
            runs = []
            i = 0
            while i < len(b):
                while i < len(b) and (b[i] | 0x20) == 0x6E:
                    i += 1
                a = i
                while i < len(b) and (b[i] | 0x20) != 0x6E:
                    i += 1
                if i - a >= k:
                    runs.append((a, i))
            for a, e in runs:
                if e - a == k and e == len(b):
                    continue  # Q1
                for st in range(a, e - k + 1):
                    code = 0
                    for c_ in b[st:st + k]:
                        code = (code << 2) | ((c_ >> 1) & 3)
                    ref[code] += 1
                    words += 1
        assert n == words and np.array_equal(c, ref)


def test_min_width_negative_never_emits(oracle):
    r = oracle.kmer_regions("CAAAC", 1, [1, -1, -3, 2], -1, 0)
    assert r["pos"].shape[1] == 0  # (size_t)-1 is huge (kmer_spans.c:279)


@pytest.mark.parametrize("k", [2, 5])
def test_log2_pm1_tables(oracle, k):
    rng = np.random.default_rng(k)
    c = rng.integers(0, 20, 4 ** k).astype(np.int32)
    w = oracle.log2_table(c, k)
    f = c / c.sum()
    srt = np.sort(f)
    fmed = (srt[len(f) // 2 - 1] + srt[len(f) // 2]) / 2
    with np.errstate(divide="ignore"):
        assert np.allclose(w, np.log2(f / fmed), equal_nan=True)
    p = oracle.pm1_table(c, k)
    assert np.array_equal(p, np.where(f >= fmed, 1.0, -1.0))


# ------------------------------------------------------------------ tr_lr

def _trlr_case(rng):
    k = rng.randint(1, 4)
    n = 4 ** k
    if rng.random() < 0.5:
        ks = np.array([rng.randint(-3, 3) for _ in range(n)], float)
        tr = np.array([rng.randint(-3, 2) for _ in range(n)], float)
    else:
        ks = np.array([rng.gauss(0, 1) for _ in range(n)])
        tr = np.array([rng.gauss(-0.2, 1) for _ in range(n)])
    seqs = ["".join(rng.choice("ACGTACGTACGTNacgt") for _ in range(rng.randint(0, 80)))
            for _ in range(rng.randint(1, 3))]
    return k, seqs, rng.choice([0, 0, 1, 2, 5]), ks, tr


def test_trlr_known_answers(oracle):
    """find_kmer_tr_lr_regions traced by hand (k=1, scores A,C,T,G = 1,-1,-3,2
    for both tables): 1-based records, the first k-mer's score at the position
    after it, a region ending at the run end without a restart, the :341 skip."""
    ks = tr = np.array([1.0, -1.0, -3.0, 2.0])
    def regs(s, ml=0):
        r = oracle.tr_lr_regions([s], 1, ml, ks, tr)
        return [tuple(int(x) for x in p) + (float(sc),) for p, sc in zip(r["pos"].T, r["score"][0])]
    assert regs("CAAAC") == [(1, 2, 4, 3.0)]
    assert regs("GGNGGG") == [(1, 2, 2, 4.0), (1, 5, 6, 6.0)]
    assert regs("GGNGGG", ml=1) == [(1, 5, 6, 6.0)]
    assert regs("GN") == []             # the first k-mer ends two bytes before the end: skipped
    assert regs("GGN") == [(1, 2, 2, 4.0)]
    assert regs("GG") == [] and regs("G") == []


def test_trlr_decomposition_agrees(oracle):
    """The decomposition the HIP path implements (every closed excursion
    rescans its tail, open ones at the run end do not) against the literal
    restart loop, 3,000 random cases."""
    from oracle import pyoracle as P
    rng = random.Random(3)
    for _ in range(3000):
        k, seqs, ml, ks, tr = _trlr_case(rng)
        o = oracle.tr_lr_regions(seqs, k, ml, ks, tr)
        got = [(int(a), int(b), int(c), float(d)) for (a, b, c), d in zip(o["pos"].T.tolist(), o["score"][0].tolist())]
        assert got == P.trlr_regions(seqs, k, ml, ks, tr), (k, ml, seqs)


def test_trlr_remap(oracle):
    """tr_lr_regions_r's remap: entry i goes to the code of kmers[i]."""
    k = 3
    names = oracle.kmer_seq(k)
    rng = np.random.default_rng(0)
    perm = rng.permutation(4 ** k)
    ks_in = np.arange(4 ** k, dtype=float)[perm]
    tr_in = -ks_in
    ks, tr, bad = oracle.trlr_remap([names[p] for p in perm], k, ks_in, tr_in)
    assert bad == 0
    assert np.array_equal(ks, np.arange(4 ** k, dtype=float)) and np.array_equal(tr, -ks)
    _, _, bad = oracle.trlr_remap(["AN"] + names[1:], k, ks_in, tr_in)
    assert bad == 1
