"""Synthetic genomes for the benchmark configurations (BASELINE.json configs,
SURVEY.md 8(d)).  There is no network and no real genome: every input is
generated, deterministically from a seed, with torch on the target device.

human_like  -- config 3/4/5: 24 contigs with GRCh38 chr1-22,X,Y lengths
               (scaled), background A=T=0.295 C=G=0.205, planted Alu-like
               300 bp copies (12% divergence), L1-like <=6 kb copies (15%),
               (CA)n microsatellites 50-300 bp, 10 kb N gaps (~0.9% N).
chr1_like   -- config 2: one 250 Mbp contig built the same way.
uniform_xorshift -- config 1: 1 Mbp i.i.d. ACGT from xorshift64 (seed 1).
"""
from __future__ import annotations

import numpy as np
import torch

GRCH38 = [248956422, 242193529, 198295559, 190214555, 181538259, 170805979, 159345973, 145138636,
          138394717, 133797422, 135086622, 133275309, 114364328, 107043718, 101991189, 90338345,
          83257441, 80373285, 58617616, 64444167, 46709983, 50818468, 156040895, 57227415]
assert sum(GRCH38) == 3088269832

_ACGT = torch.tensor([ord("A"), ord("C"), ord("G"), ord("T")], dtype=torch.uint8)
_CA = torch.tensor([ord("C"), ord("A")], dtype=torch.uint8)


def _background(n: int, g: torch.Generator, device) -> torch.Tensor:
    u = torch.rand(n, generator=g, device=device)
    # A [0,.295) C [.295,.5) G [.5,.705) T [.705,1)
    idx = (u >= 0.295).to(torch.uint8) + (u >= 0.5).to(torch.uint8) + (u >= 0.705).to(torch.uint8)
    del u
    return _ACGT.to(device)[idx.long()]


def _plant(seq: torch.Tensor, cons: torch.Tensor, slot: int, div: float, g: torch.Generator,
           min_len: int | None = None) -> None:
    """One copy of `cons` (optionally truncated to a random length >= min_len)
    per slot of `slot` bp, at a random offset, with `div` substitutions."""
    L, Lc, dev = seq.numel(), cons.numel(), seq.device
    nslot = L // slot
    if nslot == 0 or slot <= Lc:
        return
    off = torch.randint(0, slot - Lc, (nslot,), generator=g, device=dev)
    start = torch.arange(nslot, device=dev, dtype=torch.int64) * slot + off
    if min_len is None:
        lens = torch.full((nslot,), Lc, device=dev, dtype=torch.int64)
    else:
        lens = torch.randint(min_len, Lc + 1, (nslot,), generator=g, device=dev)
    # 5' truncation as in L1 copies: keep the last `len` bases of the consensus
    cpy = torch.repeat_interleave(torch.arange(nslot, device=dev), lens)
    first = torch.cumsum(lens, 0) - lens
    within = torch.arange(cpy.numel(), device=dev, dtype=torch.int64) - first[cpy]
    src = cons.to(dev)[(Lc - lens[cpy]) + within]
    mut = torch.rand(cpy.numel(), generator=g, device=dev) < div
    rnd = _ACGT.to(dev)[torch.randint(0, 4, (cpy.numel(),), generator=g, device=dev)]
    src = torch.where(mut, rnd, src)
    seq[start[cpy] + within] = src


def _microsats(seq: torch.Tensor, slot: int, g: torch.Generator) -> None:
    L, dev = seq.numel(), seq.device
    nslot = L // slot
    if nslot == 0 or slot <= 300:
        return
    off = torch.randint(0, slot - 300, (nslot,), generator=g, device=dev)
    lens = torch.randint(50, 301, (nslot,), generator=g, device=dev)
    start = torch.arange(nslot, device=dev, dtype=torch.int64) * slot + off
    cpy = torch.repeat_interleave(torch.arange(nslot, device=dev), lens)
    first = torch.cumsum(lens, 0) - lens
    within = torch.arange(cpy.numel(), device=dev, dtype=torch.int64) - first[cpy]
    seq[start[cpy] + within] = _CA.to(dev)[within % 2]


def _ngaps(seq: torch.Tensor, frac: float, g: torch.Generator, gap: int = 10000) -> None:
    L, dev = seq.numel(), seq.device
    slot = int(gap / frac)
    nslot = L // slot
    if nslot == 0:
        return
    off = torch.randint(0, slot - gap, (nslot,), generator=g, device=dev)
    start = torch.arange(nslot, device=dev, dtype=torch.int64) * slot + off
    idx = (start[:, None] + torch.arange(gap, device=dev)[None, :]).reshape(-1)
    seq[idx] = ord("N")


def contig(length: int, seed: int, device="cuda", repeats: bool = True) -> torch.Tensor:
    """One human-shaped contig (uint8 tensor of ASCII bases)."""
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    s = _background(length, g, device)
    if repeats:
        gc = torch.Generator(device=device)
        gc.manual_seed(12345)  # consensus sequences are shared by all contigs
        alu = _background(300, gc, device)
        l1 = _background(6000, gc, device)
        _plant(s, alu, 3000, 0.12, g)              # ~10% Alu-like
        _plant(s, l1, 50000, 0.15, g, min_len=500)  # ~6.5% L1-like
        _microsats(s, 30000, g)                    # (CA)n
        _ngaps(s, 0.009, g)                        # ~0.9% N in 10 kb gaps
    return s


def human_like(scale: float = 1.0, seed: int = 1, device="cuda", ncontigs: int = 24):
    """Config 3 genome (scale=1: 3,088,269,832 bp).  Returns (parts, lens)."""
    lens = [max(1, int(round(L * scale))) for L in GRCH38[:ncontigs]]
    parts = [contig(L, seed + i, device) for i, L in enumerate(lens)]
    return parts, lens


def uniform_xorshift(n: int = 1_000_000, seed: int = 1) -> bytes:
    """Config 1: i.i.d. ACGT from xorshift64 (x ^= x<<13; x ^= x>>7; x ^= x<<17),
    base = 'ACGT'[x >> 62] after each step."""
    out = np.empty(n, dtype=np.uint8)
    lut = np.frombuffer(b"ACGT", dtype=np.uint8)
    x = seed & 0xFFFFFFFFFFFFFFFF
    M = 0xFFFFFFFFFFFFFFFF
    vals = np.empty(n, dtype=np.uint64)
    for i in range(n):
        x ^= (x << 13) & M
        x ^= x >> 7
        x ^= (x << 17) & M
        vals[i] = x
    out[:] = lut[(vals >> np.uint64(62)).astype(np.int64)]
    return out.tobytes()
