"""Phase times of the host entry point (ks_kmer_regions with visits) on the
metric genome under environment variants, one process:
    python tools/host_ab.py [--scale S] [--reps R] VAR=VAL,VAR2=VAL ...
Each argument is one variant ("-" = defaults); KS_DEBUG_HOST phase lines go
to stderr, one JSON line per variant to stdout."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=float, default=1.0)
    p.add_argument("--k", type=int, default=13)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("variants", nargs="*", default=["-"])
    a = p.parse_args()
    os.environ["KS_DEBUG_HOST"] = "1"
    import torch
    import kmer_spans_amd as api
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=a.scale, seed=1, device="cuda", ncontigs=24)
    ds = D.from_parts(parts, lens, "cuda")
    del parts
    k = a.k
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    w_dev = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
    D.DeviceTable.from_counts(ctx, counts, k, "log2", total=words, expand=False, w_out=w_dev).close()
    w = w_dev.cpu().numpy()
    buf = ds.seq[:ds.total].cpu().numpy()
    host = [buf[int(x):int(y)] for x, y in zip(ds.offsets[:-1], ds.offsets[1:])]
    n_bases = float(sum(len(h) for h in host if len(h) >= k))
    ref = None
    for var in a.variants:
        env = {} if var == "-" else dict(kv.split("=", 1) for kv in var.split(","))
        for kk, vv in env.items():
            os.environ[kk] = vv
        ts = []
        for r in range(a.reps + 1):
            t0 = time.perf_counter()
            hr = api.kmer_regions(host, k, w, 100, 20.0)
            ts.append(time.perf_counter() - t0)
            if ref is None:
                ref = hr
        same = bool(np.array_equal(hr["pos"], ref["pos"]) and np.array_equal(hr["counts"], ref["counts"]))
        t = float(np.median(ts[1:]))
        print(json.dumps({"variant": var, "ms": round(t * 1e3, 2), "Gbases_per_s": round(n_bases / t / 1e9, 2),
                          "all_ms": [round(x * 1e3, 1) for x in ts], "same_as_first": same}), flush=True)
        for kk in env:
            del os.environ[kk]


if __name__ == "__main__":
    main()
