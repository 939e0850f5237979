"""The staggered two-part scan (scan_impl / scan_parts, ks_scan.hip): the
input cut at a sequence boundary, the later part started once the first has
queued its pass 1, on its own context.  Its records must equal the one-part
scan's and the oracle's bit for bit, for any cut, with and without the
parts' own halves; a part that needs the lane kernel sends the call down the
one-part path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=0.02, seed=11, device="cuda")
    ds = D.from_parts(parts, lens, "cuda")
    k = 11
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    w = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
    table = D.DeviceTable.from_counts(ctx, counts, k, "log2", total=words, expand=True, w_out=w)
    table.w = w.cpu().numpy()
    yield ctx, ds, k, table, D
    table.close()


def _scan(setup, monkeypatch, env):
    ctx, ds, k, table, D = setup
    for key, v in env.items():
        monkeypatch.setenv(key, v)
    try:
        return D.scan(ctx, ds, k, table, 100, 20.0)
    finally:
        for key in env:
            monkeypatch.delenv(key, raising=False)


@pytest.mark.parametrize("frac,halves", [(0.45, "0"), (0.2, "0"), (0.8, "0"), (0.5, "1")])
def test_parts_equal_one_part(setup, monkeypatch, oracle, frac, halves):
    one_pos, one_sc, _ = _scan(setup, monkeypatch, {"KS_PARTS_FRAC": "0"})
    pos, sc, st = _scan(setup, monkeypatch, {"KS_PARTS_FRAC": str(frac), "KS_PARTS_MIN": "1",
                                             "KS_PARTS_HALVES": halves})
    assert np.array_equal(pos, one_pos)
    assert np.array_equal(sc.view(np.uint64), one_sc.view(np.uint64))
    assert st["n_regions"] == pos.shape[1]
    ctx, ds, k, table, D = setup
    assert st["n_bases"] == int(ds.total)
    if frac == 0.45:  # and the oracle, once
        w = table.w
        host = ds.seq[:ds.total].cpu().numpy()
        seqs = [host[int(a):int(b)] for a, b in zip(ds.offsets[:-1], ds.offsets[1:])]
        o = oracle.scan(seqs, k, w, 0.0, 100, 20.0)
        assert np.array_equal(pos, o["pos"])
        assert np.array_equal(sc.view(np.uint64), o["score"].view(np.uint64))


def test_parts_short_runs_take_one_part(monkeypatch, oracle):
    """Only short sequences (each below the chunked path's run length): the
    parts abort and the one-part lane kernel scans the call."""
    import torch
    from kmer_spans_amd import _lib, device as D
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    rng = np.random.default_rng(2)
    lens = [int(x) for x in rng.integers(1000, 20000, size=300)]
    parts = [torch.from_numpy(np.frombuffer(b"ACGTN", dtype=np.uint8)[rng.integers(0, 5, size=n)].copy()).cuda()
             for n in lens]
    ds = D.from_parts(parts, lens, "cuda")
    k = 7
    w = rng.normal(size=4 ** k) * 0.5 + 0.1
    table = D.DeviceTable(ctx, w, k, 0.0)
    monkeypatch.setenv("KS_PARTS_MIN", "1")
    pos, sc, st = D.scan(ctx, ds, k, table, 20, 3.0)
    host = ds.seq[:ds.total].cpu().numpy()
    seqs = [host[int(a):int(b)] for a, b in zip(ds.offsets[:-1], ds.offsets[1:])]
    o = oracle.scan(seqs, k, w, 0.0, 20, 3.0)
    assert np.array_equal(pos, o["pos"])
    assert np.array_equal(sc.view(np.uint64), o["score"].view(np.uint64))
    table.close()
