"""How much of the genome's positions a 2^b-entry code set covers, when the
codes are assigned to the distinct score values by position frequency
(diagnostics for narrower expanded-table codes)."""
import sys, os
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kmer_spans_amd import _lib, api, genome, device as D

k = int(sys.argv[1]) if len(sys.argv) > 1 else 13
score = sys.argv[2] if len(sys.argv) > 2 else "log2"
dev = torch.device("cuda", 0)
ctx = _lib.context(0)
D.bind_torch_stream(ctx)
parts, lens = genome.human_like(scale=1.0, seed=1, device=dev, ncontigs=24)
ds = D.from_parts(parts, lens, dev)
del parts
counts = torch.zeros(4 ** k, dtype=torch.int32, device=dev)
words = D.count(ctx, ds, k, counts)
hc = counts.cpu().numpy()
w = api.log2_table(hc, k) if score == "log2" else api.pm1_table(hc, k)
vals, inv = np.unique(w, return_inverse=True)
posf = np.bincount(inv, weights=hc.astype(np.float64), minlength=len(vals))
kmf = np.bincount(inv, minlength=len(vals))
order = np.argsort(-posf)
cum = np.cumsum(posf[order]) / posf.sum()
print("k", k, score, "distinct", len(vals), "positions", posf.sum())
for b in (8, 10, 11, 12, 13):
    n = min((1 << b) - 1, len(vals))
    print(f"  {b}-bit codes ({n} direct): position coverage {cum[n - 1]:.6f}  escapes {1 - cum[n - 1]:.2e}")
order2 = np.argsort(-kmf)
cov2 = posf[order2[:4095]].sum() / posf.sum()
print("  12-bit by k-mer multiplicity: position coverage", cov2)
