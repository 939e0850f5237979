"""Per-genome phase times of config 5 (bench.py --mode genomes): count,
score table from the counts (sort / map / compress), expanded table, scan --
each bracketed by a device sync, on one human-shaped genome, repeated.

  python tools/genome_phases.py [--ext-gib 32] [--reps 3] [--k 13] [--score log2]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ext-gib", type=float, default=32.0)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--k", type=int, default=13)
    p.add_argument("--score", default="log2")
    p.add_argument("--scale", type=float, default=1.0)
    a = p.parse_args()
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=a.scale, seed=1, device="cuda", ncontigs=24)
    ds = D.from_parts(parts, lens, "cuda")
    del parts
    k = a.k
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    rows = []
    for rep in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        counts.zero_()
        words = D.count(ctx, ds, k, counts)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        tab = D.DeviceTable.from_counts(ctx, counts, k, a.score, total=words, thr=0.75 if a.score == "rank" else 0.0,
                                        expand=True, max_ext_bytes=int(a.ext_gib * (1 << 30)))
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        row = {"count_ms": round((t1 - t0) * 1e3, 3), "table_ms": round((t2 - t1) * 1e3, 3),
               "scan_ms": round((t3 - t2) * 1e3, 3), "total_ms": round((t3 - t0) * 1e3, 3),
               "table": tab.setup_ms(), "J": tab.positions_per_read, "kernel": tab.pass1_kernel,
               "scan_phases": {kk: round(v, 3) for kk, v in st.items() if kk.startswith("ms_")}}
        tab.close()
        if rep:
            rows.append(row)
        print(json.dumps(row), flush=True)
    best = min(rows, key=lambda r: r["total_ms"])
    print("best", json.dumps(best))


if __name__ == "__main__":
    main()
