"""Why is the host entry's scan slower than the device-resident one?  The
same genome and log2 table scanned (with the visit histogram) through
tables built like ks_kmer_regions builds them (host w, no position-frequency
hint, its expanded-table cap) and with the device counts as the hint."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from kmer_spans_amd import _lib, device as D, genome
    k = 13
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=1.0, seed=1, device="cuda", ncontigs=24)
    ds = D.from_parts(parts, lens, "cuda")
    del parts
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    w = torch.empty(4 ** k, dtype=torch.float64, device="cuda")
    D.DeviceTable.from_counts(ctx, counts, k, "log2", total=words, expand=True, w_out=w).close()
    wh = w.cpu().numpy()
    cap = 16 * int(ds.total)
    forms = {}
    for name, kw in (("nohint", {}), ("hint", {"freq": counts})):
        t0 = time.perf_counter()
        tab = D.DeviceTable(ctx, wh, k, 0.0, compress=True, expand=True, **kw)
        torch.cuda.synchronize()
        forms[name] = (tab, time.perf_counter() - t0)
    vis = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    for name, (tab, tb) in forms.items():
        ts = []
        for _ in range(3):
            vis.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pos, sc, st = D.scan(ctx, ds, k, tab, 100, 20.0, vis)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(name, "J", tab.positions_per_read, "kernel", tab.pass1_kernel, "build ms", round(tb * 1e3, 1),
              "scan+visits ms", [round(x, 2) for x in ts], "replays", st["n_replay"],
              {key: round(v, 3) for key, v in st.items() if key.startswith("ms_")}, flush=True)


if __name__ == "__main__":
    main()
