"""Re-run tests/test_gpu_parity.py::test_random_regions_vs_oracle's cases
(host entry ks_kmer_regions, algo 0/1) several times and report every case
whose regions differ from the oracle, with the device-path result of the same
case beside it -- a failure that comes and goes names its race here."""
import random
import sys

import numpy as np

sys.path.insert(0, "tests")


def main():
    import torch  # noqa: F401
    from kmer_spans_amd import _lib, api as K, device as D
    from oracle import oracle as O
    from test_gpu_parity import _random_inputs
    O.lib()
    dctx = _lib.load().ks_default_ctx()
    bad = 0
    for rep in range(3):
        for algo in (1, 0):
            _lib.check(_lib.load().ks_ctx_set_scan_algo(dctx, algo))
            rng = random.Random(11 + algo)
            for case in range(300):
                k, seqs, w, mw, ms = _random_inputs(rng)
                g = K.kmer_regions(seqs, k, w, mw, ms)
                o = O.kmer_regions(seqs, k, w, mw, ms)
                same = g["pos"].shape == o["pos"].shape and np.array_equal(g["pos"], o["pos"]) and \
                    np.array_equal(g["score"].view(np.uint64), o["score"].view(np.uint64))
                if not same:
                    bad += 1
                    print(f"rep {rep} algo {algo} case {case}: k {k} mw {mw} ms {ms} lens {[len(s) for s in seqs]} "
                          f"gpu {g['pos'].shape} oracle {o['pos'].shape}", flush=True)
                    gp = {tuple(c) for c in g["pos"].T.tolist()}
                    op = {tuple(c) for c in o["pos"].T.tolist()}
                    print("  only gpu", sorted(gp - op)[:8], "only oracle", sorted(op - gp)[:8], flush=True)
                    print("  w kinds", "nan" if np.isnan(w).any() else "", "inf" if np.isinf(w).any() else "",
                          "distinct", len(np.unique(w)), flush=True)
                    for again in range(5):
                        g2 = K.kmer_regions(seqs, k, w, mw, ms)
                        print("  again", again, g2["pos"].shape, np.array_equal(g2["pos"], g["pos"]), flush=True)
                    if bad > 6:
                        return
    _lib.check(_lib.load().ks_ctx_set_scan_algo(dctx, -1))
    print("bad", bad)


if __name__ == "__main__":
    main()
