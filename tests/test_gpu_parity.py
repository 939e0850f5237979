"""GPU parity: the HIP path (libkmerspans.so through the C ABI) against the
CPU oracle and the reference's recorded outputs.  Bit-exact everywhere:
region triples and order, FP64 scores (0 ulp), counts, visit histograms.
Runs on an MI355X (pytest -m gpu); skipped where no HIP device exists."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _regions_from(pos, score):
    return [(int(pos[0][i]), int(pos[1][i]), int(pos[2][i]), float(score[0][i])) for i in range(pos.shape[1])]


def _diff(a_pos, a_score, b_pos, b_score):
    """Records only in a / only in b (for the failure message)."""
    ra = {tuple(c) + (float(s),) for c, s in zip(a_pos.T.tolist(), a_score[0].tolist())}
    rb = {tuple(c) + (float(s),) for c, s in zip(b_pos.T.tolist(), b_score[0].tolist())}
    return {"only_gpu": sorted(ra - rb)[:6], "only_ref": sorted(rb - ra)[:6]}


def _assert_same_regions(a_pos, a_score, b_pos, b_score, what=""):
    assert a_pos.shape == b_pos.shape, (what, a_pos.shape, b_pos.shape, _diff(a_pos, a_score, b_pos, b_score))
    assert np.array_equal(a_pos, b_pos), (what, a_pos.T.tolist()[:8], b_pos.T.tolist()[:8],
                                          _diff(a_pos, a_score, b_pos, b_score))
    # bitwise FP64 equality of the scores
    assert np.array_equal(a_score.view(np.uint64), b_score.view(np.uint64)), what


@pytest.fixture(scope="module")
def K():
    import kmer_spans_amd as K
    return K


@pytest.fixture(scope="module")
def ctx():
    from kmer_spans_amd import _lib
    return _lib.context(0)


# ------------------------------------------------------------- known answers

def test_golden_through_gpu(K, golden):
    for case in golden["kmer_counts"]:
        r = K.kmer_counts(case["seq"], case["k"])
        assert r["n"]["n"] == case["n"], case
        if "counts" in case:
            assert r["counts"].tolist() == case["counts"]
    for case in golden["kmer_regions_r"]:
        r = K.kmer_regions(case["seq"], case["k"], case["w"], case["min_width"], case["min_score"])
        got = [[a, b, c, d] for a, b, c, d in _regions_from(r["pos"], r["score"])]
        assert got == case["regions"], case
        assert int(r["counts"].sum()) == case["visits_total"]
    for case in golden["kmer_low_comp_regions"]:
        r = K.kmer_low_comp_regions(case["seq"], case["k"], case["min_width"], case["min_score"], case["thr"])
        assert r["w_rank"].tolist() == case["w_rank"] and r["n"].tolist() == case["n"]
        assert r["pos"].shape[0] == len(case["regions"])


def test_n_gap_property_gpu(K):
    rng = random.Random(7)
    seqs = ["".join(rng.choice("ACGT") for _ in range(100)) for _ in range(2)]
    seqs.append("AG" * 50 + seqs[0] + seqs[1] + seqs[0])
    c2 = K.kmer_counts(seqs, 2)["counts"]
    c3 = K.kmer_counts([s + "N" * 36 + s for s in seqs], 2)["counts"]
    assert np.array_equal(2 * c2, c3)


# ----------------------------------------------------------- random corpus

def _random_inputs(rng, kmax=5, lmax=200):
    k = rng.randint(1, kmax)
    seqs = []
    for _ in range(rng.randint(1, 4)):
        L = rng.randint(0, lmax)
        alpha = rng.choice(["ACGT", "ACGTN", "ACGTNacgtn", "AC", "ACGTNNNN", "ACGTRY", "A"])
        seqs.append("".join(rng.choice(alpha) for _ in range(L)))
    kind = rng.random()
    if kind < 0.4:
        w = np.array([rng.randint(-3, 3) for _ in range(4 ** k)], dtype=float)
    elif kind < 0.8:
        w = np.array([rng.uniform(-2, 1.5) for _ in range(4 ** k)])
    else:  # specials flow through the clamp (NaN -> 0, +-Inf)
        w = np.array([rng.choice([1.0, -1.0, np.inf, -np.inf, np.nan, 0.0, 2.5]) for _ in range(4 ** k)])
    return k, seqs, w, rng.randint(-1, 6), rng.choice([0.0, 1.0, 2.5, 5.0, -1.0])


ALGOS = [0, 1]  # scan algorithms exercised (0 lane-per-run, 1 chunked carry scan)


@pytest.mark.parametrize("algo", ALGOS)
def test_random_regions_vs_oracle(K, oracle, ctx, algo):
    from kmer_spans_amd import _lib
    dctx = _lib.load().ks_default_ctx()
    _lib.check(_lib.load().ks_ctx_set_scan_algo(dctx, algo))
    try:
        rng = random.Random(11 + algo)
        for _ in range(300):
            k, seqs, w, mw, ms = _random_inputs(rng)
            g = K.kmer_regions(seqs, k, w, mw, ms)
            o = oracle.kmer_regions(seqs, k, w, mw, ms)
            if g["pos"].shape != o["pos"].shape or not np.array_equal(g["pos"], o["pos"]):
                # a failure that does not repeat: the same call again, 3 times
                again = [K.kmer_regions(seqs, k, w, mw, ms)["pos"] for _ in range(3)]
                print("random case mismatch", (k, mw, ms, [len(s) for s in seqs]), "again",
                      [(a.shape, bool(np.array_equal(a, o["pos"]))) for a in again],
                      "first", g["pos"].T.tolist()[:8], "oracle", o["pos"].T.tolist()[:8])
            _assert_same_regions(g["pos"], g["score"], o["pos"], o["score"], (seqs, k, mw, ms))
            assert np.array_equal(g["counts"], o["counts"])
            assert g["n"] == o["n"]
    finally:
        _lib.check(_lib.load().ks_ctx_set_scan_algo(dctx, -1))


def test_random_counts_vs_oracle(K, oracle):
    rng = random.Random(5)
    for _ in range(200):
        k = rng.randint(1, 9)
        seqs = ["".join(rng.choice(rng.choice(["ACGT", "ACGTNacgtn", "NNNNA"])) for _ in range(rng.randint(0, 300)))
                for _ in range(rng.randint(1, 4))]
        g = K.kmer_counts(seqs, k)
        n, c = oracle.kmer_counts(seqs, k)
        assert g["n"]["n"] == n and np.array_equal(g["counts"], c), (seqs, k)


def test_random_low_comp_vs_oracle(K, oracle):
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
        assert np.array_equal(g["w_rank"].view(np.uint64), o["w_rank"].view(np.uint64))
        assert np.array_equal(g["n"], o["n"])
        _assert_same_regions(g["pos"].T, g["score"].T, o["pos"], o["score"], (seqs, k, thr))


# ---------------------------------------------------- configuration shapes

def test_config1_uniform_pm1_k7(K, oracle):
    """Config 1: 1 Mbp uniform xorshift64 (seed 1), k=7, +-1 from its own
    counts, min_width 100, min_score 20."""
    from kmer_spans_amd import genome
    s = genome.uniform_xorshift(1_000_000, 1)
    c = K.kmer_counts(s, 7)
    n, oc = oracle.kmer_counts(s, 7)
    assert np.array_equal(c["counts"], oc) and c["n"]["n"] == n
    w = K.pm1_table(c["counts"], 7)
    assert np.array_equal(w, oracle.pm1_table(oc, 7))
    g = K.kmer_regions(s, 7, w, 100, 20)
    o = oracle.kmer_regions(s, 7, w, 100, 20)
    _assert_same_regions(g["pos"], g["score"], o["pos"], o["score"], "config1")
    assert np.array_equal(g["counts"], o["counts"])


@pytest.mark.parametrize("alpha,env", [(b"ACGTACGTACGTacgtNnRYx", None),  # dense Ns: 4-bit chunks
                                       (b"ACGT" * 400 + b"acgtRYxn", None),  # sparse Ns: 2-bit codes + N runs
                                       (b"ACGT" * 400 + b"acgtRYxn", "KS_STAGE_NIB"),
                                       (b"ACGT" * 400 + b"acgtRYxn", "KS_STAGE_BYTES")])
def test_host_entry_compact_staging(K, oracle, monkeypatch, alpha, env):
    """Host entry at >= 1 MiB stages each base as its class (N or
    (c >> 1) & 3): 2-bit codes + N runs, or 4-bit classes where a chunk has
    too many N runs.  Odd-length sequences (bytes shared by sequences, starts
    at every offset mod 4), lower case, N runs and non-ACGT letters, against
    the oracle."""
    if env:
        monkeypatch.setenv(env, "1")
    rng = np.random.default_rng(21)
    alpha = np.frombuffer(alpha, dtype=np.uint8)
    seqs = []
    for ln in [1, 3, 700_001, 2, 5, 1_200_003, 0, 999_999, 1, 17]:
        b = alpha[rng.integers(0, len(alpha), size=ln)].copy()
        if ln > 1000:
            b[ln // 3: ln // 3 + 500] = ord("N")
        seqs.append(b.tobytes().decode())
    k = 7
    w = rng.normal(size=4 ** k) * 0.5 + 0.05
    g = K.kmer_regions(seqs, k, w, 20, 3.0)
    o = oracle.kmer_regions(seqs, k, w, 20, 3.0)
    assert o["n"] > 100
    _assert_same_regions(g["pos"], g["score"], o["pos"], o["score"], "nibble staging")
    assert np.array_equal(g["counts"], o["counts"])


@pytest.mark.parametrize("tail", [1, 17, 29, 31, 33, 61])
def test_host_entry_short_last_chunk(K, oracle, tail):
    """A last staging chunk of a few bases (total = 16 Mi + tail) that
    alternates N and non-N: a 2-bit chunk shorter than its 16-B code payload
    has no room for N runs and must go as 4-bit classes (no write past the
    pinned / device staging buffers), against the oracle."""
    rng = np.random.default_rng(tail)
    head = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=(1 << 24) - 5)].tobytes().decode()
    last = ("NA" * tail)[:tail + 5]  # the first sequence's last 5 bases + the tail chunk, alternating
    seqs = [head, last]
    k = 5
    w = rng.normal(size=4 ** k) * 0.5 + 0.05
    g = K.kmer_regions(seqs, k, w, 20, 3.0)
    o = oracle.kmer_regions(seqs, k, w, 20, 3.0)
    _assert_same_regions(g["pos"], g["score"], o["pos"], o["score"], ("short tail", tail))
    assert np.array_equal(g["counts"], o["counts"])


@pytest.mark.parametrize("piecewise,alpha", [(True, b"ACGTACGTACGTACGTacgN"), (False, b"ACGTACGTACGTACGTacgN"),
                                             (True, b"ACGT" * 300 + b"acgN")])
def test_host_entry_counted_in_pieces(K, oracle, monkeypatch, piecewise, alpha):
    """Host entry at k >= 11 over ~150 Mbp: the staged bases are counted in
    64 Mi-base pieces on a side stream while later pieces cross PCIe (k-mers
    straddling a piece boundary belong to the later piece); the count is the
    visit histogram and the table's frequency hint.  Against the oracle,
    and the same with the count after staging (KS_HOST_COUNT_AFTER)."""
    if not piecewise:
        monkeypatch.setenv("KS_HOST_COUNT_AFTER", "1")
    rng = np.random.default_rng(5)
    alpha = np.frombuffer(alpha, dtype=np.uint8)
    seqs = []
    for ln in [67_108_863, 3, 50_000_001, 33_554_435]:
        b = alpha[rng.integers(0, len(alpha), size=ln)]
        b[(ln // 7) * np.arange(1, 7)] = ord("N")
        b[ln // 2: ln // 2 + 3_000_017] = ord("n")  # a gap over chunk boundaries
        seqs.append(b.tobytes().decode())
    k = 11
    w = np.round(rng.normal(size=4 ** k) * 4) / 4 + 0.3
    g = K.kmer_regions(seqs, k, w, 40, 8.0)
    o = oracle.kmer_regions(seqs, k, w, 40, 8.0)
    assert o["n"] > 1000
    _assert_same_regions(g["pos"], g["score"], o["pos"], o["score"], ("pieces", piecewise))
    assert np.array_equal(g["counts"], o["counts"])


@pytest.mark.parametrize("k,score", [(9, "log2"), (11, "log2"), (9, "pm1"), (8, "rank")])
def test_human_like_device_path(K, oracle, ctx, k, score):
    """Scaled config-3 genome (~6 Mbp, repeats + N gaps), device-resident
    entry points, both scan algorithms, against the oracle."""
    import torch
    from kmer_spans_amd import device as D, genome
    parts, lens = genome.human_like(scale=0.002, seed=3, device="cuda")
    ds = D.from_parts(parts, lens, "cuda")
    D.bind_torch_stream(ctx)
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    host = [ds.host_seq(q) for q in range(ds.nseq)]
    n, oc = oracle.kmer_counts(host, k)
    assert words == n and np.array_equal(counts.cpu().numpy(), oc)
    thr = 0.0
    if score == "log2":
        w = K.log2_table(oc, k)
    elif score == "pm1":
        w = K.pm1_table(oc, k)
    else:
        w, thr = K.rank_table(oc, k, n), 0.75
    o = oracle.scan(host, k, w, thr, 100, 20.0, visits=True)
    for expand in (False, True):
        tab = D.DeviceTable(ctx, w, k, thr, compress=True, expand=expand)
        assert (tab.positions_per_read > 1) == expand
        for algo in ALGOS:
            ctx.set_scan_algo(algo)
            vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
            pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0, vis)
            _assert_same_regions(pos, sc, o["pos"], o["score"], (k, score, algo, expand))
            assert np.array_equal(vis.cpu().numpy(), o["counts"]), (k, score, algo, expand)
        tab.close()
    ctx.set_scan_algo(-1)
    D.bind_torch_stream(ctx)


@pytest.mark.parametrize("mode", ["concurrent", "KS_VISITS_ATOMIC"])
def test_visit_histogram_modes(K, oracle, ctx, monkeypatch, mode):
    """The visit histogram of kmer_regions_r (kmer_spans.c:266-267) by each
    route: the top-level count on the sub-context concurrently with the scan
    (default), one atomic per scanned index -- both
    equal to the oracle's, with the same regions; twice in a row (the
    sub-context's workspace is reused)."""
    import torch
    from kmer_spans_amd import device as D, genome
    if mode != "concurrent":
        monkeypatch.setenv(mode, "1")
    k = 11
    parts, lens = genome.human_like(scale=0.002, seed=5, device="cuda")
    ds = D.from_parts(parts, lens, "cuda")
    D.bind_torch_stream(ctx)
    host = [ds.host_seq(q) for q in range(ds.nseq)]
    n, oc = oracle.kmer_counts(host, k)
    w = K.log2_table(oc, k)
    o = oracle.scan(host, k, w, 0.0, 100, 20.0, visits=True)
    tab = D.DeviceTable(ctx, w, k, 0.0, compress=True, expand=True)
    ctx.set_scan_algo(1)
    try:
        for rep in range(2):
            vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
            pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0, vis)
            _assert_same_regions(pos, sc, o["pos"], o["score"], (mode, rep))
            assert np.array_equal(vis.cpu().numpy(), o["counts"]), (mode, rep)
    finally:
        ctx.set_scan_algo(-1)
        tab.close()


@pytest.mark.parametrize("k,expand", [(11, True), (11, False), (13, True)])
def test_rank_carried_replays(K, oracle, ctx, k, expand):
    """Weighted-rank scores (config 3 shape): excursions at small S cross
    binades inside chunks, so the carry replays them (wave-parallel replay
    with parity-pair increments, binade crossings, ties) -- bit-exact
    regions and scores against the oracle, and the replay path was taken."""
    import torch
    from kmer_spans_amd import device as D, genome
    parts, lens = genome.human_like(scale=0.004, seed=11, device="cuda")
    ds = D.from_parts(parts, lens, "cuda")
    D.bind_torch_stream(ctx)
    host = [ds.host_seq(q) for q in range(ds.nseq)]
    n, oc = oracle.kmer_counts(host, k)
    w = K.rank_table(oc, k, n)
    o = oracle.scan(host, k, w, 0.75, 100, 20.0)
    tab = D.DeviceTable(ctx, w, k, 0.75, compress=True, expand=expand)
    ctx.set_scan_algo(1)
    pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0)
    ctx.set_scan_algo(-1)
    _assert_same_regions(pos, sc, o["pos"], o["score"], ("rank", k, expand))
    assert st["n_replay"] > 0 and pos.shape[1] > 100, (st["n_replay"], pos.shape)
    tab.close()


def test_edge_inputs(K, oracle):
    w = np.array([1.0, -1.0, -3.0, 2.0])
    cases = [[""], ["N" * 50], ["A"], ["ACGT" * 3, "", "NNN", "G"], ["n" * 3 + "acgt" + "N"],
             ["A" * 5000], ["AC" * 3000 + "N" + "GT" * 3000]]
    for seqs in cases:
        for k in (1, 2, 3):
            ww = np.resize(w, 4 ** k)
            g = K.kmer_regions(seqs, k, ww, 0, 0.0)
            o = oracle.kmer_regions(seqs, k, ww, 0, 0.0)
            _assert_same_regions(g["pos"], g["score"], o["pos"], o["score"], (seqs, k))
            assert np.array_equal(g["counts"], o["counts"])
            gc = K.kmer_counts(seqs, k)
            n, c = oracle.kmer_counts(seqs, k)
            assert gc["n"]["n"] == n and np.array_equal(gc["counts"], c)


def test_compressed_table_matches_full(K, ctx):
    import torch
    from kmer_spans_amd import device as D
    rng = np.random.default_rng(4)
    k = 10
    vals = rng.normal(size=300)
    w = vals[rng.integers(0, 300, 4 ** k)]
    seq = "".join(rng.choice(list("ACGT"), 200000))
    ds = D.from_host([seq, seq[:5000]], "cuda")
    D.bind_torch_stream(ctx)
    t1 = D.DeviceTable(ctx, w, k, 0.1, compress=True)
    t2 = D.DeviceTable(ctx, w, k, 0.1, compress=False)
    assert t1.compressed and not t2.compressed and t1.distinct == len(np.unique(w))
    p1, s1, _ = D.scan(ctx, ds, k, t1, 5, 1.0)
    p2, s2, _ = D.scan(ctx, ds, k, t2, 5, 1.0)
    _assert_same_regions(p1, s1, p2, s2, "compressed vs full")


@pytest.mark.parametrize("expand", [False, True])
@pytest.mark.parametrize("big", [1.5 * 2.0 ** 50, 3.0 * 2.0 ** 20])
def test_binade_summary_ties(K, oracle, ctx, big, expand):
    """Long runs where S sits deep inside one binade and steps are dyadic, so
    fl(S + s) rounds with exact ties (decided by the accumulator's parity):
    the chunked scan's binade-integer summaries must reproduce the sequential
    FP64 chain bit for bit."""
    import torch
    from kmer_spans_amd import device as D
    rng = np.random.default_rng(8)
    k = 4
    steps = np.array([0.125, -0.125, 0.375, -0.375, 0.625, -0.875, 1.125, 0.0])
    w = rng.choice(steps, 4 ** k)
    w[rng.integers(0, 4 ** k, 3)] = big
    w[rng.integers(0, 4 ** k, 2)] = -2.0 * big
    seqs = ["".join(rng.choice(list("ACGT"), 400_000)), "".join(rng.choice(list("ACGT"), 70_000))]
    ds = D.from_host(seqs, "cuda")
    D.bind_torch_stream(ctx)
    tab = D.DeviceTable(ctx, w, k, 0.0, expand=expand)
    o = oracle.scan(seqs, k, w, 0.0, 0, 0.0, visits=True)
    for algo in ALGOS:
        ctx.set_scan_algo(algo)
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, 0, 0.0, vis)
        _assert_same_regions(pos, sc, o["pos"], o["score"], ("ties", algo))
        assert np.array_equal(vis.cpu().numpy(), o["counts"])
    ctx.set_scan_algo(-1)


@pytest.mark.parametrize("k", [6, 12])
def test_long_drift_run(K, oracle, ctx, k):
    """One 3 Mbp run with positive drift (a giant excursion, the log-ratio
    shape): exercised through the chunked carry (summaries + replays)."""
    import torch
    from kmer_spans_amd import device as D, genome
    s = genome.contig(3_000_000, 21, device="cuda", repeats=True)
    s[s == ord("N")] = ord("A")
    ds = D.from_parts([s], [s.numel()], "cuda")
    host = [ds.host_seq(0)]
    n, oc = oracle.kmer_counts(host, k)
    w = K.log2_table(oc, k)
    w[~np.isfinite(w)] = -5.0
    D.bind_torch_stream(ctx)
    tab = D.DeviceTable(ctx, w, k, 0.0, expand=True)
    o = oracle.scan(host, k, w, 0.0, 100, 20.0, visits=True)
    for algo in ALGOS:
        ctx.set_scan_algo(algo)
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0, vis)
        _assert_same_regions(pos, sc, o["pos"], o["score"], ("drift", k, algo))
        assert np.array_equal(vis.cpu().numpy(), o["counts"])
        assert st["scan_algo"] == algo
    ctx.set_scan_algo(-1)


@pytest.mark.parametrize("k,compress,jmax", [(3, False, 5), (7, False, 5), (7, False, 3), (7, False, 2),
                                             (5, True, 5), (10, True, 5), (10, True, 4), (6, True, 3),
                                             (11, True, 2)])
def test_expanded_table_edges(K, oracle, ctx, monkeypatch, k, compress, jmax):
    """Expanded tables (FP64 and uint16/12-bit entries, every J) on ragged
    inputs: runs shorter than J, N runs, sequence ends inside a read group."""
    import torch
    from kmer_spans_amd import device as D
    monkeypatch.setenv("KS_EXT_MAX_J", str(jmax))
    rng = np.random.default_rng(k)
    w = rng.normal(size=4 ** k) - 0.1
    if compress:
        w = np.round(w * 8) / 8
    seqs = []
    for L in (0, k, k + 1, k + 2, k + 3, 17, 255, 256, 257, 1000, 5003):
        seqs.append("".join(rng.choice(list("ACGTN"), L, p=[0.24, 0.24, 0.24, 0.24, 0.04])))
    seqs.append("".join(rng.choice(list("ACGT"), 200000)))
    ds = D.from_host(seqs, "cuda")
    D.bind_torch_stream(ctx)
    tab = D.DeviceTable(ctx, w, k, 0.05, compress=compress, expand=True)
    assert tab.positions_per_read == (jmax if compress else min(jmax, 4))
    o = oracle.scan(seqs, k, w, 0.05, 0, 0.5, visits=True)
    for algo in ALGOS:
        ctx.set_scan_algo(algo)
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, 0, 0.5, vis)
        _assert_same_regions(pos, sc, o["pos"], o["score"], ("ext", k, algo))
        assert np.array_equal(vis.cpu().numpy(), o["counts"])
    ctx.set_scan_algo(-1)


def test_many_regions_retry(K, oracle):
    """More regions (and rescans) than the initial region buffer holds: the
    chunked path grows the buffer and reruns with visits counted once; one
    long run so that the carry is cut into many segments."""
    import torch
    from kmer_spans_amd import _lib, device as D
    ctx = _lib.Context(0)  # fresh workspace: the initial region buffer is the minimum
    k = 6
    rng = np.random.default_rng(5)
    seq = "".join(rng.choice(list("ACGT"), 4_000_000))
    w = rng.normal(size=4 ** k) - 0.05
    ds = D.from_host([seq], "cuda")
    D.bind_torch_stream(ctx)
    tab = D.DeviceTable(ctx, w, k, 0.0, expand=True)
    o = oracle.scan([seq], k, w, 0.0, 0, 0.5, visits=True)
    assert o["pos"].shape[1] > 150_000
    for algo in ALGOS:
        ctx.set_scan_algo(algo)
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, 0, 0.5, vis)
        _assert_same_regions(pos, sc, o["pos"], o["score"], ("many", algo))
        assert np.array_equal(vis.cpu().numpy(), o["counts"])
        assert st["scan_algo"] == algo  # no fallback: buffers grew instead
    del tab
    ctx.close()


def test_carry_segment_fallback(K, oracle, ctx, monkeypatch):
    """The per-run carry that replaces a failed segment assumption gives the
    same results (KS_TEST_SEG_FALLBACK forces that path)."""
    import torch
    from kmer_spans_amd import device as D, genome
    s = genome.contig(2_000_000, 33, device="cuda", repeats=True)
    ds = D.from_parts([s], [s.numel()], "cuda")
    host = [ds.host_seq(0)]
    k = 9
    n, oc = oracle.kmer_counts(host, k)
    w = K.rank_table(oc, k, n)
    D.bind_torch_stream(ctx)
    tab = D.DeviceTable(ctx, w, k, 0.75, expand=True)
    o = oracle.scan(host, k, w, 0.75, 20, 5.0, visits=True)
    ctx.set_scan_algo(1)
    for forced in (False, True):
        if forced:
            monkeypatch.setenv("KS_TEST_SEG_FALLBACK", "1")
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, 20, 5.0, vis)
        _assert_same_regions(pos, sc, o["pos"], o["score"], ("segfb", forced))
        assert np.array_equal(vis.cpu().numpy(), o["counts"])
    monkeypatch.delenv("KS_TEST_SEG_FALLBACK")
    ctx.set_scan_algo(-1)


def test_torch_stream_ordering(K, oracle, ctx):
    """A ctx bound to torch's current (default, null) stream is ordered after
    pending torch work: a zero-fill queued behind a long sleep must land
    before the count kernel adds into the tensor."""
    import torch
    from kmer_spans_amd import device as D, genome
    s = genome.contig(2_000_000, 3, device="cuda", repeats=True)
    ds = D.from_parts([s], [s.numel()], "cuda")
    D.bind_torch_stream(ctx)
    k = 12
    counts = torch.full((4 ** k,), 7, dtype=torch.int32, device="cuda")
    torch.cuda._sleep(200_000_000)  # keep the stream busy
    counts.zero_()
    words = D.count(ctx, ds, k, counts)
    assert int(counts.sum(dtype=torch.int64)) == int(words)
    n, oc = oracle.kmer_counts([ds.host_seq(0)], k)
    assert np.array_equal(counts.cpu().numpy(), oc) and n == words


@pytest.mark.parametrize("k,ndist,force", [(9, 6000, True), (13, 3000, False), (7, 5000, True)])
def test_code12_tables(K, oracle, ctx, monkeypatch, k, ndist, force):
    """J = 5 expanded tables with 12-bit codes: escapes to the base table
    (forced on with KS_EXT_ESCAPE_MAX=1 when more than 4095 values), and
    (k+4)-mer indices beyond 32 bits at k=13."""
    import torch
    from kmer_spans_amd import device as D, genome
    monkeypatch.setenv("KS_NO_LINES", "1")  # the (k+4)-mer form, not a line table
    if force:
        monkeypatch.setenv("KS_EXT_ESCAPE_MAX", "1.0")
    torch.cuda.empty_cache()  # the 128 GiB J = 5 table at k = 13 must fit beside torch's cache
    rng = np.random.default_rng(k + ndist)
    vals = np.round(rng.normal(size=ndist) * 64) / 64 + rng.normal(size=ndist) * 1e-3
    w = vals[rng.integers(0, ndist, size=4 ** k)]
    s = genome.contig(1_500_000, k, device="cuda", repeats=True)
    ds = D.from_parts([s], [s.numel()], "cuda")
    host = [ds.host_seq(0)]
    D.bind_torch_stream(ctx)
    tab = D.DeviceTable(ctx, w, k, 0.02, compress=True, expand=True)
    assert tab.positions_per_read == 5 and tab.code_bits == 12, (tab.positions_per_read, tab.code_bits)
    if ndist > 4095:
        assert tab.escape_fraction > 0
    o = oracle.scan(host, k, w, 0.02, 30, 3.0, visits=True)
    for algo in ALGOS:
        ctx.set_scan_algo(algo)
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, 30, 3.0, vis)
        _assert_same_regions(pos, sc, o["pos"], o["score"], ("c12", k, algo))
        hv = vis.cpu().numpy()
        bad = np.nonzero(hv != o["counts"])[0]
        assert bad.size == 0, ("c12 visits", k, algo, bad.size, bad[:5], hv[bad[:5]], o["counts"][bad[:5]])
    ctx.set_scan_algo(-1)
    tab.close()


# ------------------------------------------------------------------ tr_lr

def _trlr_expect(oracle, seqs, k, ml, ks, tr):
    o = oracle.tr_lr_regions(seqs, k, ml, ks, tr)
    return o["pos"], o["score"]


def test_trlr_random_vs_oracle(K, oracle):
    """lr.regions through the host entry point (k-mer strings remapped on
    the host) against the literal oracle: random sequences with N runs,
    short runs at the string ends, integer and real scores."""
    rng = random.Random(11)
    for case in range(150):
        k = rng.randint(1, 5)
        n = 4 ** k
        if case % 2:
            ks = np.array([rng.randint(-3, 3) for _ in range(n)], float)
            tr = np.array([rng.randint(-3, 2) for _ in range(n)], float)
        else:
            ks = np.array([rng.gauss(0, 1) for _ in range(n)])
            tr = np.array([rng.gauss(-0.1, 1) for _ in range(n)])
        seqs = ["".join(rng.choice("ACGTACGTACGTNacgt") for _ in range(rng.randint(0, 400)))
                for _ in range(rng.randint(1, 4))]
        ml = rng.choice([0, 1, 3, 10])
        names = oracle.kmer_seq(k)
        perm = np.random.default_rng(case).permutation(n)
        r = K.lr_regions(seqs, (k, ml), [names[p] for p in perm], ks[perm], tr[perm])
        pos, score = _trlr_expect(oracle, seqs, k, ml, ks, tr)
        _assert_same_regions(r["pos"], r["score"], pos, score, ("trlr", case))
        assert np.array_equal(r["kmer_scores"][:, 0], ks) and np.array_equal(r["kmer_scores"][:, 1], tr)


@pytest.mark.parametrize("k", [7, 11])
def test_trlr_device_chunked(K, oracle, ctx, k):
    """tr_lr on a human-shaped contig through the device path, the chunked
    scan (giant and small excursions, rescans) and the lane kernel."""
    import torch
    from kmer_spans_amd import device as D, genome
    s = genome.contig(3_000_000, 40 + k, device="cuda", repeats=True)
    ds = D.from_parts([s, s[:100_000].clone()], [s.numel(), 100_000], "cuda")
    host = [ds.host_seq(0), ds.host_seq(1)]
    n, oc = oracle.kmer_counts(host, k)
    tr = np.log2(oc + 1.0) - np.log2(np.median(oc) + 1.0) - 0.4  # repeats score positive
    ks = np.random.default_rng(k).normal(size=4 ** k)
    D.bind_torch_stream(ctx)
    ttr = D.DeviceTable(ctx, tr, k, 0.0, expand=True)
    tks = D.DeviceTable(ctx, ks, k, 0.0, compress=False)
    pos_o, score_o = _trlr_expect(oracle, host, k, 5, ks, tr)
    assert pos_o.shape[1] >= 1
    for algo in ALGOS:
        ctx.set_scan_algo(algo)
        pos, sc, st = D.tr_lr(ctx, ds, k, ttr, tks, 5)
        _assert_same_regions(pos, sc, pos_o, score_o, ("trlr-dev", k, algo))
        assert st["scan_algo"] == algo
    ctx.set_scan_algo(-1)


@pytest.mark.parametrize("nan", [True, False])
def test_trlr_nonfinite_tables(K, oracle, ctx, nan):
    """NaN / +Inf scores: the reference's clamp keeps NaN, so these tables
    take the literal kernel whatever the algorithm setting; -Inf alone only
    ever clamps to 0 and stays on the chunked scan."""
    import torch
    from kmer_spans_amd import device as D, genome
    k = 6
    rng = np.random.default_rng(2)
    tr = rng.normal(size=4 ** k) - 0.1
    if nan:
        tr[rng.integers(0, 4 ** k, 20)] = np.nan
        tr[rng.integers(0, 4 ** k, 5)] = np.inf
    tr[rng.integers(0, 4 ** k, 9)] = -np.inf
    ks = rng.normal(size=4 ** k)
    ks[:7] = -np.inf
    s = genome.contig(200_000, 5, device="cuda", repeats=True)
    ds = D.from_parts([s], [s.numel()], "cuda")
    D.bind_torch_stream(ctx)
    ttr = D.DeviceTable(ctx, tr, k, 0.0, expand=True)
    tks = D.DeviceTable(ctx, ks, k, 0.0, compress=False)
    pos_o, score_o = _trlr_expect(oracle, [ds.host_seq(0)], k, 0, ks, tr)
    ctx.set_scan_algo(1)
    pos, sc, st = D.tr_lr(ctx, ds, k, ttr, tks, 0)
    _assert_same_regions(pos, sc, pos_o, score_o, ("trlr-nonfinite", nan))
    assert st["scan_algo"] == (0 if nan else 1)
    ctx.set_scan_algo(-1)


def test_host_entry_memory_policy(K, oracle):
    """The host entries' device memory (ks_set_host_cache): policy 0 returns it
    when the call ends (VRAM back at its pre-call level), 1 keeps it until
    ks_release_cache, 2 (the default) keeps it while calls keep coming and
    returns it once the context has been idle for the idle time.  Results are
    the same under every policy."""
    import time
    import torch
    from kmer_spans_amd import _lib
    rng = np.random.default_rng(8)
    seqs = [np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=n)].tobytes().decode()
            for n in (20_000_000, 3_000_001)]
    k = 11
    w = np.round(rng.normal(size=4 ** k) * 4) / 4 + 0.2
    L = _lib.load()
    free = lambda: torch.cuda.mem_get_info()[0]  # noqa: E731
    res = []
    try:
        assert L.ks_set_host_cache(0) == 0
        res.append(K.kmer_regions(seqs, k, w, 40, 8.0))  # warm: contexts, pinned staging
        torch.cuda.synchronize()
        free0 = free()
        res.append(K.kmer_regions(seqs, k, w, 40, 8.0))
        assert free() >= free0 - (16 << 20), (free0, free())
        assert L.ks_set_host_cache(1) == 0
        res.append(K.kmer_regions(seqs, k, w, 40, 8.0))
        assert free() < free0 - (64 << 20), (free0, free())  # the workspace stayed
        L.ks_release_cache()
        assert free() >= free0 - (16 << 20), (free0, free())
        assert L.ks_set_host_cache(2) == 0 and L.ks_set_host_cache_idle(1.0) == 0
        res.append(K.kmer_regions(seqs, k, w, 40, 8.0))
        assert free() < free0 - (64 << 20), (free0, free())  # kept while idle < 1 s
        time.sleep(3.0)
        assert free() >= free0 - (16 << 20), (free0, free())  # returned by the library's thread
        res.append(K.kmer_regions(seqs, k, w, 40, 8.0))
    finally:
        L.ks_set_host_cache(2)
        L.ks_set_host_cache_idle(20.0)
    o = oracle.kmer_regions(seqs, k, w, 40, 8.0)
    for r in res:
        _assert_same_regions(r["pos"], r["score"], o["pos"], o["score"], "host cache policy")
        assert np.array_equal(r["counts"], o["counts"])


def test_many_regions_pinned_output_block(oracle, ctx):
    """A scan with > 100 K regions: the output block (>= 1 MiB) is kept and
    pinned by the library, and the regions are copied into it by DMA with no
    staging copy (ks_abi.cpp regions_pin, ks_scan.hip).  Three calls: the
    first pins a fresh block, the second reuses the kept pinned block, the
    third follows ks_release_cache (a fresh block again); every result equal
    to the oracle bit for bit, and equal to each other."""
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    D.bind_torch_stream(ctx)
    k = 9
    s = genome.contig(12_000_000, 77, device="cuda", repeats=True)
    ds = D.from_parts([s], [s.numel()], "cuda")
    host = [ds.host_seq(0)]
    rng = np.random.default_rng(5)
    w = rng.normal(0.0, 1.0, 4 ** k)  # low thresholds below: many short regions
    o = oracle.scan(host, k, w, 0.0, 3, 1.0)
    assert o["pos"].shape[1] > 100_000, o["pos"].shape
    tab = D.DeviceTable(ctx, w, k, 0.0, compress=False, expand=True)
    try:
        for call in range(3):
            if call == 2:
                _lib.load().ks_release_cache()
            pos, sc, _ = D.scan(ctx, ds, k, tab, 3, 1.0)
            _assert_same_regions(pos, sc, o["pos"], o["score"], f"many regions, call {call}")
            assert np.all(sc[1] == 0.0)
            del pos, sc  # (the block goes back to the library's keep list)
    finally:
        tab.close()
