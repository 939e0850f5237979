"""Host-entry parity across a fork() of the calling process (diagnostics).

The round-4 intermittent wrong regions appeared only in full GPU suites,
whose earlier files (tests/test_fork.py) fork the pytest process after it has
used HIP; a bisect over the other earlier files never failed.  This runs the
random host-entry corpus of tests/test_gpu_parity.py (scan algorithm 1)
against the oracle: before any fork, while a forked child of this process is
alive (it sleeps), and after it exited.  Mismatches are printed per phase.

  python tools/probes/fork_stress.py [linger_seconds]
"""
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import kmer_spans_amd as K  # noqa: E402
from kmer_spans_amd import _lib  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.test_gpu_parity import _random_inputs  # noqa: E402


def corpus(tag, seed=12, n=300):
    rng = random.Random(seed)
    bad = 0
    t0 = time.time()
    for i in range(n):
        k, seqs, w, mw, ms = _random_inputs(rng)
        g = K.kmer_regions(seqs, k, w, mw, ms)
        o = O.kmer_regions(seqs, k, w, mw, ms)
        same = g["pos"].shape == o["pos"].shape and np.array_equal(g["pos"], o["pos"]) and \
            np.array_equal(g["score"].view(np.uint64), o["score"].view(np.uint64)) and \
            np.array_equal(g["counts"], o["counts"])
        if not same:
            bad += 1
            if bad <= 5:
                print(f"  [{tag}] case {i} k {k} lens {[len(s) for s in seqs]} gpu {g['pos'].T.tolist()[:4]} "
                      f"oracle {o['pos'].T.tolist()[:4]}", flush=True)
    print(f"[{tag}] {bad} of {n} cases differ ({time.time() - t0:.1f} s)", flush=True)
    return bad


def main():
    linger = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    L = _lib.load()
    L.ks_set_fork_broker(0)
    dctx = L.ks_default_ctx()
    _lib.check(L.ks_ctx_set_scan_algo(dctx, 1))
    total = corpus("before fork")
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:  # child: touch nothing of HIP, stay alive a while, leave without cleanup
        os.close(r)
        time.sleep(linger)
        os._exit(0)
    os.close(w)
    total += corpus("child alive", seed=12)
    total += corpus("child alive, other seed", seed=13)
    os.waitpid(pid, 0)
    total += corpus("after child exit", seed=12)
    pid = os.fork()
    if pid == 0:
        os._exit(0)
    os.waitpid(pid, 0)
    total += corpus("after short fork", seed=12)
    _lib.check(L.ks_ctx_set_scan_algo(dctx, -1))
    print("RESULT differing cases", total, flush=True)
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
