"""The exact carry of integer tables (ks_table::int_exact, k_carry_exact):
with every s a small integer the FP64 partial sums are exact, so the
max-plus prescan is the carry itself.  Regions, FP64 scores and visits
against the oracle (kmer_spans.c:243-307) and against the general path
(KS_NO_EXACT=1: binade summaries and replays) on the same inputs: +-1 tables
(README.md:40-42), random small-integer tables, and a giant positive
excursion that carries through every chunk of a 3 Mbp run."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(pos, sc, opos, osc, what):
    assert pos.shape == opos.shape, (what, pos.shape, opos.shape)
    assert np.array_equal(pos, opos), what
    assert np.array_equal(np.ascontiguousarray(sc).view(np.uint64), osc.view(np.uint64)), what


def _run_both(ctx, ds, k, tab, mw, ms, o, what, monkeypatch):
    import torch
    from kmer_spans_amd import device as D
    ctx.set_scan_algo(1)
    for exact in (True, False):
        if not exact:
            monkeypatch.setenv("KS_NO_EXACT", "1")
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, mw, ms, vis)
        _same(pos, sc, o["pos"], o["score"], (what, exact))
        assert np.array_equal(vis.cpu().numpy(), o["counts"]), (what, exact, "visits")
        monkeypatch.delenv("KS_NO_EXACT", raising=False)
    ctx.set_scan_algo(-1)


@pytest.mark.parametrize("k", [7, 9, 13])
def test_pm1_exact(oracle, monkeypatch, k):
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=0.002, seed=5 + k, device="cuda", ncontigs=5)
    ds = D.from_parts(parts, lens, "cuda")
    host = [ds.host_seq(q) for q in range(ds.nseq)]
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    w = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
    tab = D.DeviceTable.from_counts(ctx, counts, k, "pm1", total=words, expand=True, w_out=w)
    o = oracle.scan(host, k, w.cpu().numpy(), 0.0, 20, 5.0, visits=True)
    assert o["pos"].shape[1] > 0
    _run_both(ctx, ds, k, tab, 20, 5.0, o, ("pm1", k), monkeypatch)
    tab.close()


@pytest.mark.parametrize("k,compress", [(6, False), (8, False), (11, True)])
def test_small_integer_tables(oracle, monkeypatch, k, compress):
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=0.0015, seed=31 + k, device="cuda", ncontigs=4)
    ds = D.from_parts(parts, lens, "cuda")
    host = [ds.host_seq(q) for q in range(ds.nseq)]
    rng = np.random.default_rng(k)
    w = rng.integers(-3, 3, size=4 ** k).astype(np.float64)  # drift -0.5 per base: many short excursions
    tab = D.DeviceTable(ctx, w, k, 0.0, compress=compress, expand=True)
    o = oracle.scan(host, k, w, 0.0, 10, 6.0, visits=True)
    assert o["pos"].shape[1] > 0
    _run_both(ctx, ds, k, tab, 10, 6.0, o, ("int", k), monkeypatch)
    tab.close()


def test_giant_integer_excursion(oracle, monkeypatch):
    """+2 / -1 values with a positive drift: one excursion carried through
    every chunk of an N-free 3 Mbp run (x up to ~10^6), the last region
    emitted at the run's end."""
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    k = 8
    s = genome.contig(3_000_000, 77, device="cuda", repeats=True)
    s[s == ord("N")] = ord("C")
    ds = D.from_parts([s], [s.numel()], "cuda")
    host = [ds.host_seq(0)]
    rng = np.random.default_rng(3)
    w = np.where(rng.random(4 ** k) < 0.45, 2.0, -1.0)
    tab = D.DeviceTable(ctx, w, k, 0.0, compress=True, expand=True)
    o = oracle.scan(host, k, w, 0.0, 100, 20.0, visits=True)
    assert o["pos"].shape[1] >= 1
    _run_both(ctx, ds, k, tab, 100, 20.0, o, "giant", monkeypatch)
    tab.close()
