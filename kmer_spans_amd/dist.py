"""Multi-GPU: one process per GPU, contigs sharded, span records gathered.

N-free runs (hence contigs) are independent (restarts never leave a run,
kmer_spans.c:281,303), so the scan shards with no exchange on the data path.
The only collectives are after the scan:
  * span-record gather to rank 0 (all_gather of the per-rank record counts,
    then a gather of the padded records to rank 0; payload = 32 B/region) --
    RCCL over xGMI with the "nccl" backend, gloo in the CPU tests;
  * an int32 sum of per-rank histograms when one genome's counts or visits
    are split across ranks (exact, order-independent).
Contigs, or their pieces cut inside N gaps, are assigned by LPT (longest
processing time first) on length: shard_pieces, the library's own planner.
"""
from __future__ import annotations

import heapq

import numpy as np
import torch
import torch.distributed as tdist


def lpt_shards(lengths, n: int):
    """Greedy LPT: contig ids per shard, each shard's ids in ascending order."""
    heap = [(0, s) for s in range(n)]
    heapq.heapify(heap)
    shards = [[] for _ in range(n)]
    for q in sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i)):
        load, s = heapq.heappop(heap)
        shards[s].append(q)
        heapq.heappush(heap, (load + int(lengths[q]), s))
    return [sorted(x) for x in shards]


def shard_pieces(seqs, n: int):
    """The library's shard plan (ks_shard_plan, csrc/ks_multi.cpp -- the one
    planner of the drop-in multi-device entry points and of bench.py): per
    shard a list of (sequence id, lo, hi) ordered by (id, lo).  Whole
    sequences by LPT on length, unless that leaves a shard more than 0.5 %
    above the fair share; then the sequences longer than half a share are cut
    in the middle of their N gaps of >= 1000 bases.  Runs never interact
    across N bases -- the scan restarts after every N (kmer_spans.c:261-265,
    281, 303), and the count's end-of-string quirk (:143) cannot apply at a
    cut with N on both sides -- so scanning and counting the pieces is exactly
    scanning and counting the sequences.  seqs: host uint8 arrays / bytes."""
    from . import _lib
    out = [[] for _ in range(n)]
    for p, q, lo, hi in _lib.shard_plan(seqs, n):
        out[p].append((q, lo, hi))
    return out


def _pack(pos: np.ndarray, score: np.ndarray) -> np.ndarray:
    rec = np.zeros((pos.shape[1], 4), dtype=np.int64)
    if pos.shape[1]:
        rec[:, 0:3] = pos.T
        rec[:, 3] = np.ascontiguousarray(score[0]).view(np.int64)
    return rec


def _unpack(rec: np.ndarray):
    pos = np.ascontiguousarray(rec[:, 0:3].T.astype(np.int32))
    score = np.zeros((2, rec.shape[0]), dtype=np.float64)
    score[0] = np.ascontiguousarray(rec[:, 3]).view(np.float64)
    return pos, score


def gather_regions(pos: np.ndarray, score: np.ndarray, device=None):
    """Gather every rank's (pos[3,n], score[2,n]) to rank 0.

    Returns (list of pos, list of score) indexed by rank on rank 0 and
    ([], []) elsewhere.  Uses the process group's backend: CUDA tensors for
    nccl (RCCL), CPU tensors for gloo."""
    world, rank = tdist.get_world_size(), tdist.get_rank()
    dev = device if tdist.get_backend() == "nccl" else torch.device("cpu")
    n = torch.tensor([pos.shape[1]], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    tdist.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    m = max(max(ns), 1)
    rec = np.zeros((m, 4), dtype=np.int64)
    rec[:pos.shape[1]] = _pack(pos, score)
    t = torch.from_numpy(rec).to(dev)
    outs = [torch.zeros_like(t) for _ in range(world)] if rank == 0 else None
    tdist.gather(t, outs, dst=0)
    if rank != 0:
        return [], []
    P, S = [], []
    for r in range(world):
        p, s = _unpack(outs[r][:ns[r]].cpu().numpy())
        P.append(p)
        S.append(s)
    return P, S


def merge_shards(shard_ids, pos_list, score_list, one_based: bool = False, offsets=None):
    """Map shard-local seq ids back to global contig ids and order the union
    by (seq_id, beg) -- the reference's emission order.  one_based: the
    records carry 1-based seq ids (tr_lr_regions_r, kmer_spans.c:699).
    offsets (pieces, shard_pieces): per shard the start of each local sequence
    inside its contig, added to beg / end."""
    if not pos_list:
        return np.zeros((3, 0), np.int32), np.zeros((2, 0), np.float64)
    one = 1 if one_based else 0
    ps, ss = [], []
    for r, (ids, p, s) in enumerate(zip(shard_ids, pos_list, score_list)):
        p = p.copy()
        if p.shape[1]:
            loc = p[0] - one
            p[0] = np.asarray(ids, dtype=np.int32)[loc] + one
            if offsets is not None:
                off = np.asarray(offsets[r], dtype=np.int64)[loc]
                p[1] = (p[1].astype(np.int64) + off).astype(p.dtype)
                p[2] = (p[2].astype(np.int64) + off).astype(p.dtype)
        ps.append(p)
        ss.append(s)
    pos = np.concatenate(ps, axis=1)
    score = np.concatenate(ss, axis=1)
    order = np.lexsort((pos[1], pos[0]))
    return pos[:, order], score[:, order]


def allreduce_histogram(h: torch.Tensor) -> torch.Tensor:
    """Exact int32 sum of per-rank count/visit histograms (wraps mod 2^32
    like the reference's int counters)."""
    tdist.all_reduce(h, op=tdist.ReduceOp.SUM)
    return h
