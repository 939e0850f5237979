"""GPU parity of the small-k scan with the table staged in LDS (north_star:
"the frequency table LDS-staged for small k"; k <= 7, k_pass1_lds) against
the oracle, and against the same scan with the LDS path switched off
(KS_NO_LDS_TABLE).  Long N-gapped contigs at log2 and +-1 give carry chains
through thousands of chunks (kmer_spans.c:261-306); visits through the
count-derived top-level histogram (:266-267)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _two_parts(monkeypatch):
    """The two-part scan (the default above ~2 M chunks, ks_scan_chunked.hip)
    on these small genomes too, as before round 5."""
    monkeypatch.setenv("KS_SPLIT_MIN_CHUNKS", "0")


@pytest.mark.parametrize("k,score", [(7, "log2"), (6, "pm1"), (4, "log2"), (7, "rank")])
def test_small_k_lds_table(oracle, k, score):
    import torch
    import kmer_spans_amd as K
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=0.002, seed=31 + k, device="cuda", ncontigs=5)
    ds = D.from_parts(parts, lens, "cuda")
    host = [ds.host_seq(q) for q in range(ds.nseq)]
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    hc = counts.cpu().numpy()
    thr = 0.75 if score == "rank" else 0.0
    w = {"log2": lambda: K.log2_table(hc, k), "pm1": lambda: K.pm1_table(hc, k),
         "rank": lambda: K.rank_table(hc, k, words)}[score]()
    o = oracle.scan(host, k, np.asarray(w), thr, 100, 20.0, visits=True)
    tab = D.DeviceTable.from_counts(ctx, counts, k, score, total=words, thr=thr, expand=True)
    ctx.set_scan_algo(1)
    try:
        for lds in (True, False):
            if not lds:
                os.environ["KS_NO_LDS_TABLE"] = "1"
            try:
                vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
                pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0, vis)
            finally:
                os.environ.pop("KS_NO_LDS_TABLE", None)
            assert st["scan_algo"] == 1
            assert np.array_equal(pos, o["pos"]), (k, score, lds)
            assert np.array_equal(np.ascontiguousarray(sc).view(np.uint64), o["score"].view(np.uint64)), (k, score, lds)
            assert np.array_equal(vis.cpu().numpy(), o["counts"]), (k, score, lds)
    finally:
        ctx.set_scan_algo(-1)
    tab.close()
    assert o["pos"].shape[1] > 0
