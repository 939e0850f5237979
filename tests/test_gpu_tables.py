"""GPU checks of ks_table_from_counts: the log2 / +-1 / weighted-rank score
tables built on the device from device counts must equal the host builders
(ks_log2_table / ks_pm1_table / ks_rank_table, themselves pinned to the
oracle in tests/test_lib.py) bit for bit, and a scan through such a table
must equal the oracle's scan with the host table (kmer_spans.c:189-202,
README.md:27-42, kmer_spans.R:25)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _counts(k, seed, kind):
    rng = np.random.default_rng(seed)
    n = 4 ** k
    if kind == "skewed":
        c = np.minimum(rng.geometric(0.03, n), 1 << 20).astype(np.int32)
        c[rng.integers(0, n, n // 5)] = 0
    elif kind == "wide":  # many distinct counts (> the LDS-staged map)
        c = rng.integers(0, 200_000, n).astype(np.int32)
    elif kind == "zeros":
        c = np.zeros(n, dtype=np.int32)
    else:  # huge odd counts: rank sums beyond 2^53 (exact-half ties)
        c = ((1 << 30) + 2 * rng.integers(0, 500, n) + 1).astype(np.int32)
    return c


@pytest.mark.parametrize("k,kind", [(3, "skewed"), (7, "skewed"), (9, "wide"), (11, "skewed"), (12, "huge"),
                                    (6, "zeros"), (11, "wide"), (12, "skewed"), (11, "zeros")])
def test_from_counts_equals_host_builders(k, kind):
    """(k >= 11 log2 / pm1: the distinct values from a value histogram, not a
    sort; the huge counts keep the sort)"""
    import torch
    import kmer_spans_amd as K
    from kmer_spans_amd import _lib, device as D
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    c = _counts(k, 10 + k, kind)
    dc = torch.from_numpy(c).cuda()
    for score, host in (("log2", lambda: K.log2_table(c, k)), ("pm1", lambda: K.pm1_table(c, k)),
                        ("rank", lambda: K.rank_table(c, k, 1.0 if kind == "huge" else float(c.sum()) or 1.0))):
        total = 1.0 if kind == "huge" else (float(c.sum()) or 1.0)
        w = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
        t = D.DeviceTable.from_counts(ctx, dc, k, score, total=total, thr=0.75 if score == "rank" else 0.0,
                                      w_out=w)
        want = np.asarray(host(), dtype=np.float64)
        got = w.cpu().numpy()
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), (score, k, kind)
        if score != "rank" and kind != "wide":
            assert t.compressed
        t.close()


@pytest.mark.parametrize("score", ["log2", "pm1", "rank"])
def test_scan_through_device_table(oracle, score):
    """Genome -> device counts -> device table (expanded) -> scan, against
    the oracle scanning with the host-built table."""
    import torch
    import kmer_spans_amd as K
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    k = 11
    parts, lens = genome.human_like(scale=0.004, seed=7, device="cuda", ncontigs=6)
    ds = D.from_parts(parts, lens, "cuda")
    host = [ds.host_seq(q) for q in range(ds.nseq)]
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    hc = counts.cpu().numpy()
    thr = 0.75 if score == "rank" else 0.0
    w_host = {"log2": lambda: K.log2_table(hc, k), "pm1": lambda: K.pm1_table(hc, k),
              "rank": lambda: K.rank_table(hc, k, words)}[score]()
    t = D.DeviceTable.from_counts(ctx, counts, k, score, total=words, thr=thr, expand=True)
    pos, sc, st = D.scan(ctx, ds, k, t, 100, 20.0)
    o = oracle.scan(host, k, np.asarray(w_host), thr, 100, 20.0)
    assert np.array_equal(pos, o["pos"])
    assert np.array_equal(np.ascontiguousarray(sc).view(np.uint64), o["score"].view(np.uint64))
    t.close()
