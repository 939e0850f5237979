"""In-process A/B of scan knobs read from the environment on every call.

One genome, one count, one table (so every variant scans through the same
allocations: no placement noise between processes), then R rounds in which
every variant runs S scan steps; prints per-variant min / median ms and the
phase breakdown of its best step, and checks every variant's regions equal
the first variant's.

  python tools/ab_inproc.py --rounds 4 --steps 3 base: half75:KS_SPLIT_FRAC=0.75
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("variants", nargs="+", help="NAME:ENV=V,ENV=V (NAME: alone = no change)")
    p.add_argument("--rounds", type=int, default=4)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--k", type=int, default=13)
    p.add_argument("--score", default="log2")
    p.add_argument("--scale", type=float, default=1.0)
    p.add_argument("--ncontigs", type=int, default=24)
    p.add_argument("--out", default=None)
    p.add_argument("--shard-of", type=int, default=1,
                   help="scan only the largest of N LPT shards (the whole genome's count and table)")
    p.add_argument("--rebuild", action="store_true",
                   help="rebuild the table every round (with KS_EXT_POOL=0: a new expanded-table allocation)")
    p.add_argument("--table-per-variant", action="store_true",
                   help="build one table per variant with its environment set (table-form A/Bs: KS_NO_LINES, "
                        "KS_NO_WIDE_LINES); all tables stay resident")
    a = p.parse_args()
    import numpy as np
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=a.scale, seed=1, device="cuda", ncontigs=a.ncontigs)
    ds = D.from_parts(parts, lens, "cuda")
    del parts
    counts = torch.zeros(4 ** a.k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, a.k, counts)
    thr = 0.75 if a.score == "rank" else 0.0
    variants = []
    for v in a.variants:
        name, _, envs = v.partition(":")
        env = dict(e.split("=", 1) for e in envs.split(",") if e)
        variants.append((name, env))
    tabs = {}
    if a.table_per_variant:
        for name, env in variants:
            old = {key: os.environ.get(key) for key in env}
            os.environ.update(env)
            tabs[name] = D.DeviceTable.from_counts(ctx, counts, a.k, a.score, total=words, thr=thr, expand=True)
            for key, v in old.items():
                if v is None:
                    os.environ.pop(key, None)
                else:
                    os.environ[key] = v
            print(name, "table J", tabs[name].positions_per_read, "code bits", tabs[name].code_bits,
                  tabs[name].setup_ms(), flush=True)
        tab = tabs[variants[0][0]]
    else:
        tab = D.DeviceTable.from_counts(ctx, counts, a.k, a.score, total=words, thr=thr, expand=True)
    if a.shard_of > 1:
        from kmer_spans_amd.dist import lpt_shards
        shards = lpt_shards([int(x) for x in lens], a.shard_of)
        mine = max(shards, key=lambda sh: sum(int(lens[q]) for q in sh))
        ds = ds.subset(sorted(mine))
        print("shard", a.shard_of, "contigs", sorted(mine), "bp", int(ds.total), flush=True)
    res = {n: [] for n, _ in variants}
    phases = {}
    ref = None
    for r in range(a.rounds):
        if a.rebuild and r:
            tab.close()
            torch.cuda.synchronize()
            tab = D.DeviceTable.from_counts(ctx, counts, a.k, a.score, total=words, thr=thr, expand=True)
        for name, env in variants:
            old = {key: os.environ.get(key) for key in env}
            os.environ.update(env)
            try:
                for _ in range(a.steps):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    pos, sc, st = D.scan(ctx, ds, a.k, tabs.get(name, tab), 100, 20.0)
                    torch.cuda.synchronize()
                    ms = (time.perf_counter() - t0) * 1e3
                    res[name].append(ms)
                    if ms <= min(res[name]):
                        phases[name] = {key: round(st[key], 3) for key in
                                        ("ms_runs", "ms_layout", "ms_scan", "ms_predict", "ms_carry", "ms_stitch",
                                         "ms_rescan", "ms_finish")}
                    if ref is None:
                        ref = (pos.copy(), np.ascontiguousarray(sc).copy())
                    elif not (np.array_equal(pos, ref[0]) and np.array_equal(sc, ref[1])):
                        raise SystemExit(f"variant {name}: regions differ from the first variant's")
            finally:
                for key, v in old.items():
                    if v is None:
                        os.environ.pop(key, None)
                    else:
                        os.environ[key] = v
        print(f"round {r}: " + "  ".join(f"{n} {min(res[n][-a.steps:]):.3f}" for n, _ in variants), flush=True)
    out = {}
    for name, env in variants:
        v = res[name]
        out[name] = {"env": env, "min_ms": round(min(v), 3), "median_ms": round(statistics.median(v), 3),
                     "best_phases": phases[name]}
        print(name, json.dumps(out[name]))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    for t_ in set(list(tabs.values()) + [tab]):
        t_.close()


if __name__ == "__main__":
    main()
