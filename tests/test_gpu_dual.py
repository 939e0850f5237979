"""GPU parity of the two-part scan (scan_impl: the input cut at the sequence
boundary nearest half its bases, both parts scanned at once on two
contexts): regions and the visit histogram must equal the oracle's
(kmer_spans.c:243-307, :266-267) and the one-part path's bit for bit.
KS_DUAL_MIN lowers the size at which the two-part path is taken."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("score,k", [("log2", 11), ("rank", 9), ("pm1", 12)])
def test_two_part_scan(oracle, score, k):
    import torch
    import kmer_spans_amd as K
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=0.003, seed=40 + k, device="cuda", ncontigs=7)
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
    got = {}
    try:
        for dual in (True, False):
            os.environ["KS_DUAL_MIN" if dual else "KS_NO_DUAL"] = "1"
            try:
                vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
                pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0, vis)
            finally:
                os.environ.pop("KS_DUAL_MIN", None)
                os.environ.pop("KS_NO_DUAL", None)
            assert np.array_equal(pos, o["pos"]), (score, k, dual)
            assert np.array_equal(np.ascontiguousarray(sc).view(np.uint64), o["score"].view(np.uint64)), (score, dual)
            assert np.array_equal(vis.cpu().numpy(), o["counts"]), (score, k, dual)
            assert st["n_regions"] == o["pos"].shape[1]
            got[dual] = st
    finally:
        ctx.set_scan_algo(-1)
    assert got[True]["n_bases"] == got[False]["n_bases"]
    assert got[True]["n_scored"] == got[False]["n_scored"]
    tab.close()
