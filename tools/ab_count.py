"""In-process A/B of count knobs read from the environment on every call:
one genome, R rounds of S counts per variant; every variant's histogram
must equal the first's.

  python tools/ab_count.py --k 13 base: g256:KS_PART_BLOCKS=256
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("variants", nargs="+")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--k", type=int, default=13)
    p.add_argument("--scale", type=float, default=1.0)
    a = p.parse_args()
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=a.scale, seed=1, device="cuda", ncontigs=24)
    ds = D.from_parts(parts, lens, "cuda")
    del parts
    counts = torch.zeros(4 ** a.k, dtype=torch.int32, device="cuda")
    ref = None
    res = {}
    for r in range(a.rounds):
        for v in a.variants:
            name, _, envs = v.partition(":")
            env = dict(e.split("=", 1) for e in envs.split(",") if e)
            old = {key: os.environ.get(key) for key in env}
            os.environ.update(env)
            try:
                for _ in range(a.steps):
                    counts.zero_()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    D.count(ctx, ds, a.k, counts)
                    torch.cuda.synchronize()
                    res.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
                    if ref is None:
                        ref = counts.clone()
                    elif not torch.equal(ref, counts):
                        raise SystemExit(f"variant {name}: counts differ")
            finally:
                for key, val in old.items():
                    if val is None:
                        os.environ.pop(key, None)
                    else:
                        os.environ[key] = val
        print(f"round {r}: " + "  ".join(f"{n} {min(v[-a.steps:]):.2f}" for n, v in res.items()), flush=True)
    for n, v in res.items():
        print(n, "min", round(min(v), 3), "median", round(statistics.median(v), 3))
    # cross-process comparison of library builds (KS_LIB_PATH): a checksum of the histogram
    idx = torch.arange(ref.numel(), device=ref.device, dtype=torch.int64) % 1000003 + 1
    print("checksum", int((ref.to(torch.int64) * idx).sum().item()), "total", int(ref.to(torch.int64).sum().item()))


if __name__ == "__main__":
    main()
