"""Piece statistics of the weighted-rank closed form (ks_internal.h
RankPiece) on the metric genome's k-mer counts: distinct counts, their
multiplicities, position weights -- how many 2^18-bounded pieces a 32-bit
(piece, offset) rank code needs, and how much of the genome the hottest H
pieces cover.  python tools/probes/rank_pieces_stats.py [k]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from kmer_spans_amd import _lib, device as D, genome
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 13
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    parts, lens = genome.human_like(scale=1.0, seed=1, device="cuda", ncontigs=24)
    ds = D.from_parts(parts, lens, "cuda")
    del parts
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    c = counts.cpu().numpy().astype(np.int64)
    dv, dm = np.unique(c, return_counts=True)
    total = float(words)
    # pieces: class i spans sorted positions [S_i, S_i + m_i); R grows by d_i = c_i / total per position
    R = 0.0
    pieces = []  # (weight, length)
    for ci, mi in zip(dv.tolist(), dm.tolist()):
        d = ci / total
        if ci == 0:
            pieces.append((0, mi))
            continue
        start = R
        end = R + d * mi
        # binade crossings inside the class
        e0 = np.frexp(start)[1] if start > 0 else -1074
        e1 = np.frexp(end)[1]
        nb = max(1, e1 - e0 + 1)
        first_extra = 1 if mi > 1 else 0
        n_split = (mi + (1 << 18) - 1) >> 18
        npc = first_extra + max(nb, n_split)
        for _ in range(npc):
            pieces.append((ci * mi / npc, mi / npc))
        R = end
    w = np.array(sorted((p[0] for p in pieces), reverse=True))
    cum = np.cumsum(w) / max(w.sum(), 1)
    out = {"k": k, "words": int(words), "distinct_counts": int(dv.size), "pieces_est": len(pieces),
           "classes_mult_gt1": int((dm > 1).sum()), "max_mult": int(dm.max()),
           "cover_by_hot": {str(h): float(cum[min(h, len(cum)) - 1]) for h in (1024, 2048, 4096, 6144, 8192)}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
