"""The free-ordering probe: does a
workspace free wait for work queued on the context's other streams?

KS_DEBUG_SPIN_MS queues a spin kernel on the side and high-priority streams
right before each workspace free of the library (a slot growing in ensure,
the policy-0 release at the end of a host call) and reports the drain and
the hipFree times.  Run once with the fix (all three streams drained) and
once with the round-4 drain of the main stream only: if hipFree lasts the
spin in the second case, hipFree orders the free after every stream's work
by itself and the round-4 "recycling edge" could not have let a kernel read
a freed-and-recycled buffer.  Results to JSON (one object per variant).

    python tools/probes/free_order_probe.py --out gpurun_out/free_order.json
"""
import argparse
import json
import os
import re
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SPIN = re.compile(r"\[spin\] (\S+) slot (-?\d+): spin ([\d.]+) ms queued on side\+hi, drain \(([^)]*)\) ([\d.]+) ms, "
                  r"hipFree ([\d.]+) ms")


def genome(n, seed):
    rng = np.random.default_rng(seed)
    b = np.frombuffer(b"ACGTacgt", dtype=np.uint8)[rng.integers(0, 8, size=n)].copy()
    for a in range(300_000, n, 900_000):
        b[a:a + 1200] = ord("N")
    return [b.tobytes().decode()]


def run(main_only, spin_ms):
    import kmer_spans_amd as K
    from kmer_spans_amd import _lib
    from oracle import oracle as O
    L = _lib.load()
    os.environ["KS_DEBUG_SPIN_MS"] = str(spin_ms)
    if main_only:
        os.environ["KS_DEBUG_DRAIN_MAIN_ONLY"] = "1"
    else:
        os.environ.pop("KS_DEBUG_DRAIN_MAIN_ONLY", None)
    k = 9
    w = np.round(np.random.default_rng(4).normal(size=4 ** k) * 4) / 4 + 0.1
    L.ks_release_cache()
    L.ks_set_host_cache(0)
    exact = True
    with tempfile.TemporaryFile(mode="w+") as f:
        sys.stderr.flush()
        saved = os.dup(2)
        os.dup2(f.fileno(), 2)
        try:
            for seqs in (genome(400_000, 1), genome(3_000_000, 2), genome(6_000_000, 3)):
                g = K.kmer_regions(seqs, k, w, 20, 3.0)
                o = O.kmer_regions(seqs, k, w, 20, 3.0)
                exact &= bool(np.array_equal(g["pos"], o["pos"]) and np.array_equal(g["counts"], o["counts"])
                              and np.array_equal(g["score"].view(np.uint64), o["score"].view(np.uint64)))
        finally:
            os.dup2(saved, 2)
            os.close(saved)
            L.ks_set_host_cache(2)
            L.ks_release_cache()
        f.seek(0)
        err = f.read()
    frees = [{"where": m[0], "slot": int(m[1]), "spin_ms": float(m[2]), "drain": m[3], "drain_ms": float(m[4]),
              "hipfree_ms": float(m[5])} for m in SPIN.findall(err)]
    os.environ.pop("KS_DEBUG_SPIN_MS", None)
    os.environ.pop("KS_DEBUG_DRAIN_MAIN_ONLY", None)
    return {"variant": "drain main stream only (round-4 ensure)" if main_only else "drain all three streams (fix)",
            "results_equal_oracle": exact, "frees": frees,
            "min_drain_plus_free_ms": min((x["drain_ms"] + x["hipfree_ms"] for x in frees), default=None)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spin-ms", type=float, default=300.0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = [run(False, a.spin_ms), run(True, a.spin_ms)]
    s = json.dumps({"spin_ms": a.spin_ms, "variants": res}, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
