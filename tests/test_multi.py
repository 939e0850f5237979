"""Multi-device host entries (ks_multi.cpp): the shard plan and the merge of
the parts' regions, on the CPU (host-only library functions, the oracle as
the per-part scanner), and -- marked gpu -- the three host entry points over
the device list [0, 0] (two contexts on one card) against the oracle.
Reference: kmer_counts / kmer_regions_r / kmer_low_comp_regions
(kmer_spans.c:452-487, 490-546, 548-621); the shards replace the
mclapply-over-sequences pattern of test.R:550-567."""
import ctypes as C
import random

import numpy as np
import pytest


def _seqs_with_gaps(rng, n_long=2, n_short=5):
    seqs = []
    for _ in range(n_long):
        parts = []
        for _ in range(rng.randint(2, 5)):
            parts.append("".join(rng.choice("ACGTacgt") for _ in range(rng.randint(500, 3000))))
            parts.append("N" * rng.choice([3, 999, 1000, 1500, 2500]))
        parts.append("".join(rng.choice("ACGT") for _ in range(rng.randint(1, 800))))
        seqs.append("".join(parts))
    for _ in range(n_short):
        seqs.append("".join(rng.choice("ACGTN") for _ in range(rng.randint(0, 400))))
    rng.shuffle(seqs)
    return seqs


def _plan(seqs, nparts):
    from kmer_spans_amd import _lib
    L = _lib.load()
    bufs = [s.encode("latin-1") for s in seqs]
    ptrs = (C.c_char_p * len(bufs))(*bufs)
    lens = np.array([len(b) for b in bufs], dtype=np.int64)
    n = L.ks_shard_plan(ptrs, lens.ctypes.data, len(bufs), nparts, None, 0)
    assert n >= 0
    out = np.zeros((max(n, 1), 4), dtype=np.int64)
    assert L.ks_shard_plan(ptrs, lens.ctypes.data, len(bufs), nparts, out.ctypes.data, n) == n
    return out[:n]


def _part_seqs(seqs, plan, p):
    return [seqs[int(q)][int(lo):int(hi)] for part, q, lo, hi in plan if part == p]


@pytest.mark.parametrize("nparts", [1, 2, 3, 8])
def test_shard_plan_covers_and_cuts_in_gaps(nparts):
    rng = random.Random(nparts)
    for _ in range(6):
        seqs = _seqs_with_gaps(rng)
        plan = _plan(seqs, nparts)
        assert set(plan[:, 0].tolist()) <= set(range(nparts))
        # every non-empty sequence covered exactly once, in order
        for q, s in enumerate(seqs):
            rows = sorted((int(lo), int(hi)) for part, qq, lo, hi in plan if qq == q)
            if not s:
                assert rows == []
                continue
            assert rows[0][0] == 0 and rows[-1][1] == len(s)
            for (a, b), (c, d) in zip(rows, rows[1:]):
                assert b == c
                # a cut: N on both sides, inside a gap of >= 1000 N
                assert s[c - 1] in "Nn" and s[c] in "Nn"
                lo, hi = c, c
                while lo > 0 and s[lo - 1] in "Nn":
                    lo -= 1
                while hi < len(s) and s[hi] in "Nn":
                    hi += 1
                assert hi - lo >= 1000 and c == (lo + hi) // 2
        # each part's rows in (sequence, lo) order
        for p in range(nparts):
            rows = [(int(q), int(lo)) for part, q, lo, hi in plan if part == p]
            assert rows == sorted(rows)


def test_shard_plan_balances_one_long_sequence():
    rng = random.Random(3)
    body = []
    for _ in range(40):
        body.append("".join(rng.choice("ACGT") for _ in range(2000)))
        body.append("N" * 1200)
    seqs = ["".join(body)]
    plan = _plan(seqs, 4)
    load = np.zeros(4, dtype=np.int64)
    for part, q, lo, hi in plan:
        load[part] += hi - lo
    assert load.max() <= 1.15 * load.sum() / 4


def _regions_struct(pos, score):
    from kmer_spans_amd import _lib
    n = pos.shape[1]
    keep = [np.ascontiguousarray(pos[i].astype(np.int32)) for i in range(3)]
    sc = np.ascontiguousarray(score[0].astype(np.float64)) if n else np.zeros(1)
    r = _lib.Regions()
    r.n = n
    r.seq_id = keep[0].ctypes.data_as(C.POINTER(C.c_int32))
    r.beg = keep[1].ctypes.data_as(C.POINTER(C.c_int32))
    r.end = keep[2].ctypes.data_as(C.POINTER(C.c_int32))
    r.score = sc.ctypes.data_as(C.POINTER(C.c_double))
    return r, keep + [sc]


@pytest.mark.parametrize("nparts", [2, 3, 5])
def test_merge_of_parts_equals_whole(oracle, nparts):
    """Each part's pieces scanned as sequences of their own (the oracle), the
    regions merged by ks_merge_parts, the counts and visits added: equal to
    the whole input's, for kmer_counts, kmer_regions and the low-complexity
    scan with the weighted-rank table of the summed counts."""
    from kmer_spans_amd import _lib
    L = _lib.load()
    rng = random.Random(40 + nparts)
    for trial in range(4):
        seqs = _seqs_with_gaps(rng, n_long=2, n_short=3)
        k = rng.choice([3, 4, 5])
        plan = _plan(seqs, nparts)
        # counts
        n_all, c_all = oracle.kmer_counts(seqs, k)
        c_sum = np.zeros_like(c_all)
        n_sum = 0
        for p in range(nparts):
            ps = _part_seqs(seqs, plan, p)
            if ps:
                n_p, c_p = oracle.kmer_counts(ps, k)
                c_sum += c_p
                n_sum += n_p
        assert np.array_equal(c_sum, c_all) and n_sum == n_all
        # regions + visits, and the rank scan from the summed counts
        w = np.array([rng.uniform(-2, 1.5) for _ in range(4 ** k)])
        ranks = oracle.rank_table(c_all, k, float(n_all))
        for w_scan, mw, ms in [(w, 4, 1.0), (ranks - 0.75, 10, 2.0)]:
            whole = oracle.kmer_regions(seqs, k, w_scan, mw, ms)
            structs, keep, vis = [], [], np.zeros_like(whole["counts"])
            for p in range(nparts):
                ps = _part_seqs(seqs, plan, p)
                if ps:
                    r = oracle.kmer_regions(ps, k, w_scan, mw, ms)
                    vis += r["counts"]
                    s, kp = _regions_struct(r["pos"], r["score"])
                else:
                    s, kp = _regions_struct(np.zeros((3, 0), np.int32), np.zeros((2, 0)))
                structs.append(s)
                keep.append(kp)
            arr = (_lib.Regions * nparts)(*structs)
            out = _lib.Regions()
            flat = np.ascontiguousarray(plan.reshape(-1))
            _lib.check(L.ks_merge_parts(flat.ctypes.data, len(plan), nparts, arr, C.byref(out)))
            pos, score = _lib.regions_to_numpy(out)
            assert np.array_equal(pos, whole["pos"]), (trial, k)
            assert np.array_equal(score[0].view(np.uint64), whole["score"][0].view(np.uint64))
            assert np.array_equal(vis, whole["counts"])


# ------------------------------------------------------------------ GPU


@pytest.fixture
def two_contexts():
    from kmer_spans_amd import api
    api.set_devices([0, 0])
    try:
        yield
    finally:
        api.set_devices([])


@pytest.mark.gpu
def test_device_list_host_entries_vs_oracle(K, oracle, two_contexts):
    """ks_kmer_counts / ks_kmer_regions / ks_low_comp_regions over the device
    list [0, 0] (two contexts on one card, the input dealt by the shard plan;
    a long sequence cut in its N gaps) against the oracle, bit for bit."""
    rng = random.Random(77)
    cases = [_seqs_with_gaps(rng, n_long=2, n_short=4) for _ in range(3)]
    big = np.frombuffer(b"ACGTacgt", dtype=np.uint8)[np.random.default_rng(5).integers(0, 8, size=3_000_000)].copy()
    for a in range(200_000, 3_000_000, 450_000):
        big[a:a + 1500] = ord("N")
    cases.append([big.tobytes().decode(), "ACGTTGCA" * 50, ""])
    for seqs in cases:
        for k in (5, 9):
            c = K.kmer_counts(seqs, k)
            n, oc = oracle.kmer_counts(seqs, k)
            assert c["n"]["n"] == n and np.array_equal(c["counts"], oc)
            w = np.round(np.random.default_rng(k).normal(size=4 ** k) * 4) / 4 + 0.1
            g = K.kmer_regions(seqs, k, w, 20, 3.0)
            o = oracle.kmer_regions(seqs, k, w, 20, 3.0)
            assert np.array_equal(g["pos"], o["pos"])
            assert np.array_equal(g["score"].view(np.uint64), o["score"].view(np.uint64))
            assert np.array_equal(g["counts"], o["counts"]) and g["n"] == o["n"]
            lc = K.kmer_low_comp_regions(seqs, k, 20, 5.0, 0.75)
            ol = oracle.low_comp_regions(seqs, k, 20, 5.0, 0.75)
            assert np.array_equal(lc["counts"], ol["counts"])
            assert np.array_equal(lc["w_rank"].view(np.uint64), ol["w_rank"].view(np.uint64))
            assert np.array_equal(lc["n"], ol["n"])
            assert np.array_equal(lc["pos"].T, ol["pos"])
            assert np.array_equal(lc["score"].T[0].view(np.uint64), ol["score"][0].view(np.uint64))


@pytest.fixture(scope="module")
def K():
    import kmer_spans_amd as K
    return K
