"""GPU parity of pass 1 on line tables (k_pass1l): every line form -- uint16
codes with own = 2..5 k-mers per line (J = own + 2 scan indices per 64-B
line) and FP64 values with own = 2..4 (J = own + 1) -- forced by the
expanded-table byte cap, for kmer_regions (log2 / +-1 / weighted rank,
with the visit histogram through both the count-derived and the atomic
route) and tr_lr, against the oracle (kmer_spans.c:243-307, :329-395)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _two_parts(monkeypatch):
    """The two-part scan (the default above ~2 M chunks, ks_scan_chunked.hip)
    on these small genomes too, as before round 5."""
    monkeypatch.setenv("KS_SPLIT_MIN_CHUNKS", "0")

GiB = 1 << 30


def _same(pos, sc, opos, osc, what):
    assert pos.shape == opos.shape, (what, pos.shape, opos.shape)
    assert np.array_equal(pos, opos), what
    assert np.array_equal(sc.view(np.uint64), osc.view(np.uint64)), what


@pytest.fixture(scope="module")
def setup():
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=0.0015, seed=77, device="cuda", ncontigs=6)
    ds = D.from_parts(parts, lens, "cuda")
    host = [ds.host_seq(q) for q in range(ds.nseq)]
    return ctx, ds, host, torch


# (k, cap GiB) -> own of the uint16 line (m = k + own - 1, 4^m x 64 B <= cap)
@pytest.mark.parametrize("k,cap,own_u16,own_f64", [(11, 80, 5, 4), (11, 20, 4, 4), (11, 5, 3, 3), (11, 1.5, 2, 2),
                                                   (13, 80, 3, 3), (12, 20, 3, 3), (9, 1.0, 4, 4)])
@pytest.mark.parametrize("score", ["log2", "pm1", "rank"])
def test_line_forms(oracle, setup, monkeypatch, k, cap, own_u16, own_f64, score):
    ctx, ds, host, torch = setup
    from kmer_spans_amd import device as D
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    thr = 0.75 if score == "rank" else 0.0
    w = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
    tab = D.DeviceTable.from_counts(ctx, counts, k, score, total=words, thr=thr, expand=True,
                                    max_ext_bytes=int(cap * GiB), w_out=w)
    own = own_f64 if score == "rank" else own_u16
    J = own + (1 if score == "rank" else 2)
    assert tab.positions_per_read == J, (score, k, cap, tab.positions_per_read)
    wh = w.cpu().numpy()
    o = oracle.scan(host, k, wh, thr, 100 if score != "pm1" else 20, 20.0 if score != "pm1" else 5.0, visits=True)
    mw, ms = (100, 20.0) if score != "pm1" else (20, 5.0)
    for route in ("count", "atomic", "f64summ", "f64ksumm"):
        if route == "atomic":
            monkeypatch.setenv("KS_VISITS_ATOMIC", "1")
        if route.startswith("f64"):  # FP64 lines with pass-1 summaries / k_summaries (no summaries by default)
            if score != "rank":
                continue
            monkeypatch.setenv("KS_F64_P1SUMM", "1" if route == "f64summ" else "0")
        ctx.set_scan_algo(1)
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, mw, ms, vis)
        assert st["scan_algo"] == 1
        _same(pos, sc, o["pos"], o["score"], (score, k, cap, route))
        assert np.array_equal(vis.cpu().numpy(), o["counts"]), (score, k, cap, route, "visits")
        monkeypatch.delenv("KS_VISITS_ATOMIC", raising=False)
        monkeypatch.delenv("KS_F64_P1SUMM", raising=False)
    ctx.set_scan_algo(-1)
    tab.close()


@pytest.mark.parametrize("k,cap", [(13, 80), (11, 5)])
def test_line_trlr(oracle, setup, k, cap):
    """tr_lr regions through the line pass (the first k-mer's own score at
    each run start, 1-based records), log2 table as both tables."""
    ctx, ds, host, torch = setup
    from kmer_spans_amd import device as D
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    w = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
    tab = D.DeviceTable.from_counts(ctx, counts, k, "log2", total=words, expand=True, max_ext_bytes=int(cap * GiB),
                                    w_out=w)
    assert tab.positions_per_read >= 4
    wh = w.cpu().numpy()
    init = D.DeviceTable(ctx, wh, k, 0.0, compress=False)
    o = oracle.tr_lr_regions(host, k, 50, wh, wh)
    ctx.set_scan_algo(1)
    pos, sc, st = D.tr_lr(ctx, ds, k, tab, init, 50)
    ctx.set_scan_algo(-1)
    _same(pos, sc, o["pos"], o["score"], ("trlr", k, cap))
    tab.close()
    init.close()


def test_line_vs_expanded_same_regions(setup, monkeypatch):
    """The metric-shaped config (k = 13, log2) through the line table and
    through the J = 5 expanded table: identical regions and scores."""
    ctx, ds, host, torch = setup
    from kmer_spans_amd import device as D
    k = 13
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    out = []
    for lines in (True, False):
        if not lines:
            monkeypatch.setenv("KS_NO_LINES", "1")
        tab = D.DeviceTable.from_counts(ctx, counts, k, "log2", total=words, expand=True)
        assert tab.positions_per_read == (6 if lines else 5)  # wide 128-B lines / the (k+4)-mer table
        assert tab.code_bits == (13 if lines else 12)
        ctx.set_scan_algo(1)
        out.append(D.scan(ctx, ds, k, tab, 100, 20.0)[:2])
        ctx.set_scan_algo(-1)
        tab.close()
    _same(out[0][0], out[0][1], out[1][0], out[1][1], "line vs expanded")


def _skewed_table(rng, k, nhead, ntail, tail_share):
    """w with nhead frequent values and ntail rare ones (tail_share of the
    k-mers): the wide line's 11-bit L3 codes escape for the rare ones."""
    head = np.round(rng.normal(size=nhead) * 64) / 64 + rng.normal(size=nhead) * 1e-3
    tail = rng.normal(size=ntail) * 3.0
    n = 4 ** k
    w = head[rng.integers(0, nhead, size=n)]
    sel = rng.random(n) < tail_share
    w[sel] = tail[rng.integers(0, ntail, size=int(sel.sum()))]
    return w


@pytest.mark.parametrize("k,ntail,share", [(13, 5000, 0.06), (12, 4000, 0.03), (13, 0, 0.0)])
def test_wide_lines(oracle, setup, monkeypatch, k, ntail, share):
    """Wide 128-B lines (13-bit own / L1 / L2 codes, 11-bit L3 codes with
    escapes to the base code table, J = own + 3): regions, scores and both
    visit routes against the oracle, on tables with escapes."""
    ctx, ds, host, torch = setup
    from kmer_spans_amd import device as D
    rng = np.random.default_rng(k + ntail)
    w = _skewed_table(rng, k, 600, ntail, share) if ntail else \
        np.round(rng.normal(size=4 ** k) * 8) / 8  # few distinct values: no escape
    thr = 0.02
    tab = D.DeviceTable(ctx, w, k, thr, compress=True, expand=True)
    assert tab.positions_per_read == 16 - k + 3 and tab.code_bits == 13, (tab.positions_per_read, tab.code_bits)
    if ntail:
        assert 0 < tab.escape_fraction <= 0.10, tab.escape_fraction
    o = oracle.scan(host, k, w, thr, 30, 3.0, visits=True)
    for route in ("count", "atomic"):
        if route == "atomic":
            monkeypatch.setenv("KS_VISITS_ATOMIC", "1")
        ctx.set_scan_algo(1)
        vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        pos, sc, st = D.scan(ctx, ds, k, tab, 30, 3.0, vis)
        _same(pos, sc, o["pos"], o["score"], ("wide", k, route))
        assert np.array_equal(vis.cpu().numpy(), o["counts"]), ("wide visits", k, route)
        monkeypatch.delenv("KS_VISITS_ATOMIC", raising=False)
    # tr_lr through the wide pass
    init = D.DeviceTable(ctx, w - thr, k, 0.0, compress=False)
    trans = D.DeviceTable(ctx, w - thr, k, 0.0, compress=True, expand=True)
    ot = oracle.tr_lr_regions(host, k, 40, w - thr, w - thr)
    pos, sc, st = D.tr_lr(ctx, ds, k, trans, init, 40)
    _same(pos, sc, ot["pos"], ot["score"], ("wide trlr", k))
    ctx.set_scan_algo(-1)
    for t_ in (tab, init, trans):
        t_.close()
