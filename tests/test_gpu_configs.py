"""GPU parity at the BASELINE configurations that are hardest for the
chunked exact-carry scan (VERDICT r1 "what's weak" #1):

  * config 2 shape: ONE N-gapped chr1-like contig of 50 Mbp, k = 11,
    log2(f/f_med) from its own counts: one giant excursion per N-free run,
    i.e. carry chains through hundreds of 256-index chunks and many carry
    segments (kmer_spans.c:261-306);
  * config 4 shape: k = 15 (the reference's largest k, kmer_spans.c:504-505):
    a 4^15-entry table, compressed (uint16 codes, J = 3 expanded 17-mer
    table of 128 GiB) and uncompressed (FP64, J = 2 16-mer table), with the
    visit histogram.

Everything is compared with the CPU oracle bit for bit: region triples and
order, FP64 scores (0 ulp), visit histograms."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(pos, sc, o, what):
    assert pos.shape == o["pos"].shape, (what, pos.shape, o["pos"].shape)
    assert np.array_equal(pos, o["pos"]), what
    assert np.array_equal(np.ascontiguousarray(sc).view(np.uint64), o["score"].view(np.uint64)), what


@pytest.mark.parametrize("split_min", ["0", None])  # the two-part scan forced, and the default (one part here)
def test_chr1_like_50mbp_k11_log2(oracle, monkeypatch, split_min):
    if split_min is not None:
        monkeypatch.setenv("KS_SPLIT_MIN_CHUNKS", split_min)
    import torch
    from kmer_spans_amd import _lib, api, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    k = 11
    s = genome.contig(50_000_000, 101, device="cuda", repeats=True)
    ds = D.from_parts([s], [s.numel()], "cuda")
    host = [ds.host_seq(0)]
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    n, oc = oracle.kmer_counts(host, k)
    hc = counts.cpu().numpy()
    assert words == n and np.array_equal(hc, oc)
    w = api.log2_table(hc, k)
    o = oracle.scan(host, k, w, 0.0, 100, 20.0, visits=True)
    tab = D.DeviceTable(ctx, w, k, 0.0, compress=True, expand=True, freq=counts)
    ctx.set_scan_algo(1)
    vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0, vis)
    ctx.set_scan_algo(-1)
    _same(pos, sc, o, "chr1-like 50 Mbp")
    assert np.array_equal(vis.cpu().numpy(), o["counts"])
    # the giant-excursion regime: few regions, each spanning most of a run
    assert 0 < pos.shape[1] < 200
    assert st["scan_algo"] == 1 and st["n_scored"] > 49_000_000
    tab.close()


def _k15_table(ndist, seed, k=15):
    """A 4^k-entry table with ndist distinct values, built on the GPU."""
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    vals = torch.randn(ndist, generator=g, device="cuda", dtype=torch.float64) * 0.5 - 0.05
    idx = torch.randint(0, ndist, (4 ** k,), generator=g, device="cuda")
    w = vals[idx].cpu().numpy()
    del idx
    return w


@pytest.mark.parametrize("k,compress,ndist,J", [(15, True, 3000, 3), (15, True, 2000, 4), (14, True, 2000, 5),
                                                (15, False, None, 2)])
def test_k15_scan(oracle, k, compress, ndist, J):
    """k = 15 / 14 tables in every form the builder picks: wide 128-B lines
    indexed by the 15-mer (own 1 / 2 + 4 L1 + 16 L2 13-bit codes, 64 L3 11-bit
    codes: J = 4 / 5) when at most 2047 values carry the positions; the
    17-mer expanded table (J = 3) when the L3 codes would escape too often
    (3000 uniform values); FP64 J = 2."""
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts = [genome.contig(L, 151 + i, device="cuda", repeats=True) for i, L in enumerate((2_000_000, 700_000, 15))]
    ds = D.from_parts(parts, [p.numel() for p in parts], "cuda")
    host = [ds.host_seq(q) for q in range(ds.nseq)]
    # compressed: ndist distinct values (uint16 codes); uncompressed: every
    # entry its own value (FP64)
    if compress:
        w = _k15_table(ndist, 15, k)
    else:
        import torch as T
        g = T.Generator(device="cuda")
        g.manual_seed(16)
        w = (T.randn(4 ** k, generator=g, device="cuda", dtype=T.float64) * 0.5 - 0.05).cpu().numpy()
    thr = 0.0
    o = oracle.scan(host, k, w, thr, 30, 3.0, visits=True)
    tab = D.DeviceTable(ctx, w, k, thr, compress=compress, expand=True)
    assert tab.compressed == compress
    assert tab.positions_per_read == J, tab.positions_per_read
    if J >= 4:
        assert tab.line_kind == 3 and tab.pass1_kernel == "k_pass1w"
    for algo in (0, 1):
        ctx.set_scan_algo(algo)
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, 30, 3.0, vis)
        _same(pos, sc, o, ("k15", compress, algo))
        assert np.array_equal(vis.cpu().numpy(), o["counts"]), ("k15 visits", compress, algo)
        del vis
    ctx.set_scan_algo(-1)
    tab.close()
    assert o["pos"].shape[1] > 0


def test_rank_k15(oracle):
    """Config 4 as surveyed (weighted rank at k = 15, kmer_spans.c:189-202,
    :548-621 with no k limit): device count of a ~3 Mbp genome, the device
    (count, index) sort of 4^15 pairs and closed-form FP64 rank table (equal
    to the host builder, itself pinned to the oracle's sequential prefix in
    tests/test_lib.py), its expanded FP64 table, and the chunked scan (thr
    0.75) against the oracle."""
    import torch
    from kmer_spans_amd import _lib, api, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    k = 15
    torch.cuda.empty_cache()
    s = genome.contig(3_000_000, 515, device="cuda", repeats=True)
    ds = D.from_parts([s], [s.numel()], "cuda")
    host = [ds.host_seq(0)]
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    w = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
    tab = D.DeviceTable.from_counts(ctx, counts, k, "rank", total=words, thr=0.75, expand=True, w_out=w)
    assert not tab.compressed and tab.positions_per_read >= 2
    wh = w.cpu().numpy()
    hc = counts.cpu().numpy()
    ref = np.asarray(api.rank_table(hc, k, words), dtype=np.float64)
    assert np.array_equal(wh.view(np.uint64), ref.view(np.uint64)), "device rank table vs host builder"
    del ref, hc
    o = oracle.scan(host, k, wh, 0.75, 100, 20.0, visits=True)
    ctx.set_scan_algo(1)
    vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0, vis)
    ctx.set_scan_algo(-1)
    _same(pos, sc, o, "rank k=15")
    assert np.array_equal(vis.cpu().numpy(), o["counts"]), "rank k=15 visits"
    assert pos.shape[1] > 0
    tab.close()


@pytest.mark.parametrize("k,sizes", [(13, (9_000_000, 4_000_000, 700_000, 30_000)), (15, (3_000_000, 900_000, 20_000))])
def test_rank_code_lines(oracle, monkeypatch, k, sizes):
    """Configs 3 and 4's table form (weighted rank at k = 13 / 15,
    kmer_spans.c:189-202): the 32-bit rank codes (piece, offset) of the
    closed-form prefix -- verified on the device against the FP64 ranks when
    built -- in 128-B code lines of 15-mers that pass 1 reads 5 / 3 positions
    at a time (k_pass1r), beside the FP64 form of the later passes (64-B lines
    at k = 13, the expanded table at k = 15); regions, FP64 scores and visits
    against the oracle, and equal to the FP64 scan (KS_NO_RANK_CODES=1) on a
    multi-contig genome with repeats."""
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    torch.cuda.empty_cache()
    parts = [genome.contig(L, 80 + i, device="cuda", repeats=True) for i, L in enumerate(sizes)]
    ds = D.from_parts(parts, [p.numel() for p in parts], "cuda")
    host = [ds.host_seq(i) for i in range(len(parts))]
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    w = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
    tab = D.DeviceTable.from_counts(ctx, counts, k, "rank", total=words, thr=0.75, expand=True, w_out=w)
    assert tab.line_kind == 4 and tab.pass1_kernel == "k_pass1r" and tab.positions_per_read == 18 - k
    wh = w.cpu().numpy()
    o = oracle.scan(host, k, wh, 0.75, 100, 20.0, visits=True)
    assert o["pos"].shape[1] > 10
    ctx.set_scan_algo(1)
    try:
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0, vis)
        _same(pos, sc, o, "rank code lines")
        assert np.array_equal(vis.cpu().numpy(), o["counts"]), "rank code lines: visits"
        tab.close()
        monkeypatch.setenv("KS_NO_RANK_CODES", "1")
        tab = D.DeviceTable.from_counts(ctx, counts, k, "rank", total=words, thr=0.75, expand=True)
        assert tab.line_kind == (2 if k == 13 else 0)
        pos2, sc2, _ = D.scan(ctx, ds, k, tab, 100, 20.0)
        _same(pos2, sc2, o, "rank FP64 lines")
    finally:
        ctx.set_scan_algo(-1)
        tab.close()


@pytest.mark.parametrize("k,jmax", [(10, 2), (11, 3), (9, 4)])
def test_rank_expanded_pass1_summaries(oracle, monkeypatch, k, jmax):
    """The FP64 expanded form of the k = 14 / 15 weighted-rank tables
    (k_pass1pf, forced at small k by KS_EXT_MAX_J) with its pass-1 binade
    summaries and halves, with k_summaries after an unexpanded-summary pass
    (KS_F64_P1SUMM=0), and with no summaries (the default): regions, scores
    and visits equal to the oracle on a multi-contig genome."""
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    monkeypatch.setenv("KS_EXT_MAX_J", str(jmax))
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts = [genome.contig(L, 40 + i, device="cuda", repeats=True)
             for i, L in enumerate((1_500_000, 1_100_000, 800_000, 60_000))]
    ds = D.from_parts(parts, [p.numel() for p in parts], "cuda")
    host = [ds.host_seq(i) for i in range(len(parts))]
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    w = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
    tab = D.DeviceTable.from_counts(ctx, counts, k, "rank", total=words, thr=0.6, expand=True, w_out=w)
    assert not tab.compressed and tab.positions_per_read == jmax
    o = oracle.scan(host, k, w.cpu().numpy(), 0.6, 50, 5.0, visits=True)
    ctx.set_scan_algo(1)
    # two parts forced; the default one part; no summaries (one part)
    for summ, split_min in (("1", "0"), ("0", "0"), ("1", str(2 << 20)), (None, "0")):
        if summ is None:
            monkeypatch.delenv("KS_F64_P1SUMM", raising=False)
        else:
            monkeypatch.setenv("KS_F64_P1SUMM", summ)
        monkeypatch.setenv("KS_SPLIT_MIN_CHUNKS", split_min)
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, 50, 5.0, vis)
        _same(pos, sc, o, ("rank expanded", k, jmax, summ, split_min))
        assert np.array_equal(vis.cpu().numpy(), o["counts"]), ("rank expanded visits", k, jmax, summ, split_min)
    ctx.set_scan_algo(-1)
    assert o["pos"].shape[1] > 0
    tab.close()


def test_genomes_mode(oracle):
    """Config 5 logic (bench.py --mode genomes, test.R:550-567's per-scaffold
    pattern at genome scale): several genomes scanned one after another on
    one context, each with its own device count -> device log2 table (a
    32 GiB cap, as the mode builds it per genome) -> scan with the visit
    histogram; every genome's regions, scores and visits against the
    oracle with that genome's table."""
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    k = 13
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    for g in range(3):
        parts, lens = genome.human_like(scale=0.002, seed=1 + 1000 * g, device="cuda", ncontigs=24)
        ds = D.from_parts(parts, lens, "cuda")
        host = [ds.host_seq(q) for q in range(ds.nseq)]
        counts.zero_()
        words = D.count(ctx, ds, k, counts)
        w = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
        tab = D.DeviceTable.from_counts(ctx, counts, k, "log2", total=words, expand=True,
                                        max_ext_bytes=32 << 30, w_out=w)
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0, vis)
        o = oracle.scan(host, k, w.cpu().numpy(), 0.0, 100, 20.0, visits=True)
        _same(pos, sc, o, ("genome", g))
        assert np.array_equal(vis.cpu().numpy(), o["counts"]), ("genome visits", g)
        assert st["n_bases"] == sum(lens)
        tab.close()


@pytest.mark.parametrize("k", [11, 13, 14])
def test_count_hot_buckets(oracle, k):
    """The partitioned counter's hard cases (sequence_kmer_count,
    kmer_spans.c:135-155): a few buckets holding most of the k-mers (long
    homopolymer and dinucleotide runs -> the k_bins work list cuts them into
    shares that add with atomics, and runs of equal items are added once per
    lane), sequence starts inside tiles (many short sequences, the Q1 quirk at
    sequence ends), N runs, and the staged scatter's padded regions; counts
    and the k-mer total equal the oracle's.  k = 14 takes the two-level
    counter."""
    import torch
    from kmer_spans_amd import _lib, device as D
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    rng = np.random.default_rng(k)
    parts = [b"A" * 3_000_000, b"CA" * 1_000_000, b"T" * 500_000 + b"N" * 77 + b"T" * 700_001]
    parts.append(rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=2_000_000).tobytes())
    for _ in range(300):  # short sequences: starts inside the count's tiles
        L = int(rng.integers(0, 40))
        parts.append(rng.choice(np.frombuffer(b"ACGTN", dtype=np.uint8), size=L).tobytes())
    mixed = bytearray(rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=1_500_000).tobytes())
    for at in rng.integers(0, len(mixed) - 5000, size=200):
        mixed[at:at + 4000] = b"A" * 4000
    parts.append(bytes(mixed))
    ds = D.from_host(parts, "cuda")
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    n, oc = oracle.kmer_counts(parts, k)
    assert words == n
    assert np.array_equal(counts.cpu().numpy(), oc)


@pytest.mark.parametrize("score,k", [("rank", 11), ("log2", 9)])
def test_carry_and_rescan_forms(oracle, monkeypatch, score, k):
    """The round-5 carry / heads / rescan forms and their A/B alternatives on
    one multi-contig genome (k = 11 rank, k = 9 log2), each against the oracle (regions,
    FP64 scores bit for bit, visits): the default forms (clean / certain-clamp
    runs in one wave step, certain-clamp heads packed densely, wide rescan
    batches), no summaries for any table (KS_NO_SUMMARIES), the two-part path
    on a small genome (KS_SPLIT_MIN_CHUNKS=0), FP64 tables with k_summaries
    (KS_F64_P1SUMM=0).
    (kmer_spans.c:261-306, 298-305: the carried state, the restart.)"""
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts = [genome.contig(L, 60 + i, device="cuda", repeats=True)
             for i, L in enumerate((1_800_000, 900_000, 300_000, 40_000))]
    ds = D.from_parts(parts, [p.numel() for p in parts], "cuda")
    host = [ds.host_seq(i) for i in range(len(parts))]
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    w = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
    thr = 0.6 if score == "rank" else 0.0
    tab = D.DeviceTable.from_counts(ctx, counts, k, score, total=words, thr=thr, expand=True, w_out=w)
    mw, ms = (50, 5.0) if score == "rank" else (20, 5.0)
    o = oracle.scan(host, k, w.cpu().numpy(), thr, mw, ms, visits=True)
    assert o["pos"].shape[1] > 0
    ctx.set_scan_algo(1)
    forms = [{}, {"KS_NO_SUMMARIES": "1"}, {"KS_SPLIT_MIN_CHUNKS": "0"}]
    if score == "rank":
        forms.append({"KS_F64_P1SUMM": "0"})
    try:
        for env in forms:
            for key, val in env.items():
                monkeypatch.setenv(key, val)
            vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
            pos, sc, st = D.scan(ctx, ds, k, tab, mw, ms, vis)
            assert st["scan_algo"] == 1
            _same(pos, sc, o, (score, env))
            assert np.array_equal(vis.cpu().numpy(), o["counts"]), (score, env, "visits")
            for key in env:
                monkeypatch.delenv(key)
    finally:
        ctx.set_scan_algo(-1)
        tab.close()
