"""Re-run tests/test_gpu_parity.py::test_random_regions_vs_oracle's cases
(host entry ks_kmer_regions, algo 0/1) several times and report every case
whose regions differ from the oracle, with the device-path result of the same
case beside it -- a failure that comes and goes names its race here."""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def poisoner(pattern):
    """hipMalloc / memset / hipFree of 2 GiB before each call, so that the
    call's fresh workspace allocations come back holding `pattern` bytes
    instead of zeros (a read of unwritten workspace then shows)."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    hip.hipFree.argtypes = [C.c_void_p]
    hip.hipDeviceSynchronize.argtypes = []

    def run():
        bufs = []
        for _ in range(8):
            p = C.c_void_p()
            if hip.hipMalloc(C.byref(p), 256 << 20) != 0:
                break
            hip.hipMemset(p, pattern, 256 << 20)
            bufs.append(p)
        hip.hipDeviceSynchronize()
        for p in bufs:
            hip.hipFree(p)
    return run


def main():
    import torch  # noqa: F401
    from kmer_spans_amd import _lib, api as K, device as D
    from oracle import oracle as O
    from test_gpu_parity import _random_inputs
    O.lib()
    dctx = _lib.load().ks_default_ctx()
    bad = 0
    for rep, pattern in enumerate((0xFF, 0x7F, 0x3F)):
        poison = poisoner(pattern)
        for algo in (1, 0):
            _lib.check(_lib.load().ks_ctx_set_scan_algo(dctx, algo))
            rng = random.Random(11 + algo)
            for case in range(300):
                k, seqs, w, mw, ms = _random_inputs(rng)
                poison()
                g = K.kmer_regions(seqs, k, w, mw, ms)
                o = O.kmer_regions(seqs, k, w, mw, ms)
                same = g["pos"].shape == o["pos"].shape and np.array_equal(g["pos"], o["pos"]) and \
                    np.array_equal(g["score"].view(np.uint64), o["score"].view(np.uint64))
                if not same:
                    bad += 1
                    print(f"pattern {pattern:#x} rep {rep} algo {algo} case {case}: k {k} mw {mw} ms {ms} lens {[len(s) for s in seqs]} "
                          f"gpu {g['pos'].shape} oracle {o['pos'].shape}", flush=True)
                    gp = {tuple(c) for c in g["pos"].T.tolist()}
                    op = {tuple(c) for c in o["pos"].T.tolist()}
                    print("  only gpu", sorted(gp - op)[:8], "only oracle", sorted(op - gp)[:8], flush=True)
                    print("  w kinds", "nan" if np.isnan(w).any() else "", "inf" if np.isinf(w).any() else "",
                          "distinct", len(np.unique(w)), flush=True)
                    for again in range(5):
                        poison()
                        g2 = K.kmer_regions(seqs, k, w, mw, ms)
                        print("  again", again, g2["pos"].shape, np.array_equal(g2["pos"], g["pos"]), flush=True)
                    if bad > 6:
                        return
    _lib.check(_lib.load().ks_ctx_set_scan_algo(dctx, -1))
    print("bad", bad)


if __name__ == "__main__":
    main()
