"""In-process A/B of device score-table builds (knobs read from the
environment per call): one genome, one count, then R rounds in which every
variant builds the log2 table with its expanded table (the pooled buffer is
reused) and scans once; prints each variant's build phases (min over rounds)
and checks that every variant's regions equal the first variant's.

  python tools/ab_table.py --rounds 3 u4: u1:KS_EXT_U1=1
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("variants", nargs="+", help="NAME:ENV=V,ENV=V (NAME: alone = no change)")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--k", type=int, default=13)
    p.add_argument("--score", default="log2")
    p.add_argument("--scale", type=float, default=1.0)
    p.add_argument("--ext-max-gib", type=float, default=0.0, help="expanded-table cap (0: the library's choice)")
    a = p.parse_args()
    import numpy as np
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=a.scale, seed=1, device="cuda", ncontigs=24)
    ds = D.from_parts(parts, lens, "cuda")
    del parts
    counts = torch.zeros(4 ** a.k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, a.k, counts)
    variants = []
    for v in a.variants:
        name, _, envs = v.partition(":")
        variants.append((name, dict(e.split("=", 1) for e in envs.split(",") if e)))
    best = {}
    ref = None
    for r in range(a.rounds):
        for name, env in variants:
            old = {key: os.environ.get(key) for key in env}
            os.environ.update(env)
            try:
                tab = D.DeviceTable.from_counts(ctx, counts, a.k, a.score, total=words,
                                                thr=0.75 if a.score == "rank" else 0.0, expand=True,
                                                max_ext_bytes=int(a.ext_max_gib * 2 ** 30))
                sm = tab.setup_ms()
                pos, score, _ = D.scan(ctx, ds, a.k, tab, 100, 20.0)
                tab.close()
                torch.cuda.synchronize()
            finally:
                for key, val in old.items():
                    if val is None:
                        os.environ.pop(key, None)
                    else:
                        os.environ[key] = val
            if ref is None:
                ref = (pos, score)
            elif not (np.array_equal(ref[0], pos) and np.array_equal(ref[1].view(np.uint64), score.view(np.uint64))):
                raise SystemExit(f"variant {name}: regions differ")
            if r == 0:
                continue  # first round: allocation of the pooled expanded-table buffer
            b = best.setdefault(name, {})
            for key, v in sm.items():
                b[key] = min(b.get(key, float("inf")), v)
        print(f"round {r}: " + "  ".join(f"{n} {best.get(n, {}).get('ext_build', float('nan')):.2f}"
                                           for n, _ in variants), flush=True)
    for name, b in best.items():
        print(name, {key: round(v, 3) for key, v in b.items()})


if __name__ == "__main__":
    main()
