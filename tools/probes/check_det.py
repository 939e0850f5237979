"""Determinism check: genome generation, k-mer counts and the score table
for a given k, computed twice in one process (diagnostics)."""
import sys, os, hashlib
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kmer_spans_amd import _lib, api, genome, device as D

k = int(sys.argv[1]) if len(sys.argv) > 1 else 15
scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
dev = torch.device("cuda", 0)
ctx = _lib.context(0)
D.bind_torch_stream(ctx)
for rep in range(2):
    parts, lens = genome.human_like(scale=scale, seed=1, device=dev, ncontigs=24)
    ds = D.from_parts(parts, lens, dev)
    del parts
    h = hashlib.sha1(ds.seq.cpu().numpy().tobytes()).hexdigest()[:16]
    counts = torch.zeros(4 ** k, dtype=torch.int32, device=dev)
    words = D.count(ctx, ds, k, counts)
    hc = counts.cpu().numpy()
    w = api.log2_table(hc, k)
    print(rep, "genome", h, "words", words, "counts_sum", int(hc.sum(dtype=np.int64)),
          "counts_hash", hashlib.sha1(hc.tobytes()).hexdigest()[:16],
          "distinct", len(np.unique(w)), flush=True)
    del ds, counts
    torch.cuda.empty_cache()
