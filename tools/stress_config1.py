"""Config 1 (1 Mbp uniform, k = 7, +-1 from its own counts) through the host
entry N times against one oracle result; prints the mismatch count and the
first differing records (an intermittent wrong carry)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import kmer_spans_amd as K
    from kmer_spans_amd import genome
    from oracle import oracle as O
    n_iter = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    s = genome.uniform_xorshift(1_000_000, 1)
    c = K.kmer_counts(s, 7)
    w = K.pm1_table(c["counts"], 7)
    o = O.kmer_regions(s, 7, w, 100, 20)
    bad = 0
    for i in range(n_iter):
        g = K.kmer_regions(s, 7, w, 100, 20)
        if g["pos"].shape != o["pos"].shape or not np.array_equal(g["pos"], o["pos"]):
            bad += 1
            if bad <= 3:
                print("iter", i, "gpu", g["pos"].T.tolist()[:4], "oracle", o["pos"].T.tolist()[:4], flush=True)
    print("env", {k: v for k, v in os.environ.items() if k.startswith("KS_")}, "bad", bad, "of", n_iter, flush=True)


if __name__ == "__main__":
    main()
