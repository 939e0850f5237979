"""Multi-rank (world_size 2, gloo, CPU) tests of the sharding and the
span-record gather/merge used by the multi-GPU path (kmer_spans_amd/dist.py)."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp


def test_lpt_shards_balance():
    from kmer_spans_amd import dist, genome
    L = genome.GRCH38
    for n in (1, 2, 4, 8):
        sh = dist.lpt_shards(L, n)
        assert sorted(q for s in sh for q in s) == list(range(len(L)))
        loads = [sum(L[q] for q in s) for s in sh]
        assert max(loads) / (sum(L) / n) < 1.04  # 1.0363 at 8 GPUs


def _worker(rank, world, port, q):
    import torch.distributed as tdist
    from kmer_spans_amd import dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(rank)
    n = 5 + 3 * rank
    pos = np.zeros((3, n), np.int32)
    pos[0] = rng.integers(0, 2, n)          # shard-local seq ids
    pos[1] = np.sort(rng.integers(0, 1000, n))
    pos[2] = pos[1] + 7
    score = np.zeros((2, n))
    score[0] = rng.normal(size=n)
    P, S = dist.gather_regions(pos, score)
    import torch
    h = torch.full((16,), rank + 1, dtype=torch.int32)
    dist.allreduce_histogram(h)
    if rank == 0:
        q.put((P, S, h.numpy()))
    tdist.destroy_process_group()


def test_gather_regions_gloo_world2():
    from kmer_spans_amd import dist
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    P, S, h = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [p.shape[1] for p in P] == [5, 8]
    assert np.array_equal(h, np.full(16, 3))
    # shard 0 holds contigs [1, 3], shard 1 holds [0, 2]
    pos, score = dist.merge_shards([[1, 3], [0, 2]], P, S)
    assert pos.shape[1] == 13
    keys = list(zip(pos[0], pos[1]))
    assert keys == sorted(keys)
    assert set(pos[0]) <= {0, 1, 2, 3}
    # bitwise score round trip
    allsc = np.concatenate([s[0] for s in S])
    assert sorted(allsc.view(np.uint64)) == sorted(score[0].view(np.uint64))


def _genome(seed=7):
    """A multi-contig genome with N gaps (host bytes) and its log2 table."""
    rng = np.random.default_rng(seed)
    lens = [40000, 9000, 26000, 3000, 17000, 5, 31000]
    seqs = []
    for L in lens:
        b = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=L, p=[0.3, 0.2, 0.2, 0.3])
        for _ in range(L // 8000):
            a = int(rng.integers(0, max(L - 300, 1)))
            b[a:a + int(rng.integers(1, 300))] = ord("N")
        if L > 2000:  # a low-complexity stretch so that regions exist
            a = int(rng.integers(0, L - 1500))
            b[a:a + 1200] = np.frombuffer((b"CA" * 600), np.uint8)
        seqs.append(b.tobytes())
    return seqs, lens


def _shard_worker(rank, world, port, q):
    import torch
    import torch.distributed as tdist
    from kmer_spans_amd import dist
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    k = 6
    seqs, lens = _genome()
    shards = dist.lpt_shards(lens, world)
    mine = [seqs[i] for i in shards[rank]]
    # per-shard counts, summed exactly across ranks (the shard-mode table)
    _, c = O.kmer_counts(mine, k)
    h = torch.from_numpy(c.astype(np.int32))
    dist.allreduce_histogram(h)
    w = O.log2_table(h.numpy(), k)
    r = O.scan(mine, k, w, 0.0, 20, 3.0)
    P, S = dist.gather_regions(r["pos"], r["score"])
    t = O.tr_lr_regions(mine, k, 15, w, w)
    PT, ST = dist.gather_regions(t["pos"], t["score"])
    if rank == 0:
        q.put((shards, h.numpy(), P, S, PT, ST))
    tdist.destroy_process_group()


def test_sharded_equals_unsharded_gloo_world2(oracle):
    """Contigs LPT-sharded over two ranks, scanned per shard, gathered to rank
    0 and merged == the unsharded scan, bit for bit (regions, order, scores),
    for kmer_regions (0-based seq ids) and tr_lr (1-based, kmer_spans.c:699);
    the all-reduced shard counts == the unsharded counts."""
    from kmer_spans_amd import dist
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() + 17) % 1000
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    shards, h, P, S, PT, ST = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    O = oracle
    k = 6
    seqs, _ = _genome()
    _, c = O.kmer_counts(seqs, k)
    assert np.array_equal(h, c)
    w = O.log2_table(c, k)
    full = O.scan(seqs, k, w, 0.0, 20, 3.0)
    pos, score = dist.merge_shards(shards, P, S)
    assert full["pos"].shape[1] > 5
    assert np.array_equal(pos, full["pos"])
    assert np.array_equal(score.view(np.uint64), full["score"].view(np.uint64))
    tfull = O.tr_lr_regions(seqs, k, 15, w, w)
    tpos, tscore = dist.merge_shards(shards, PT, ST, one_based=True)
    assert tfull["pos"].shape[1] > 5
    assert np.array_equal(tpos, tfull["pos"])
    assert np.array_equal(tscore.view(np.uint64), tfull["score"].view(np.uint64))


def _gapped_genome(seed=11):
    """A genome with one dominant contig carrying N gaps of >= 1000 bases
    (where the library's shard plan may cut), plus short contigs."""
    rng = np.random.default_rng(seed)
    lens = [120000, 9000, 26000, 3000, 17000, 5, 31000]
    seqs = []
    for L in lens:
        b = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=L, p=[0.3, 0.2, 0.2, 0.3])
        for _ in range(L // 8000):  # short N runs everywhere
            a = int(rng.integers(0, max(L - 300, 1)))
            b[a:a + int(rng.integers(1, 300))] = ord("N")
        if L > 2000:  # a low-complexity stretch so that regions exist
            a = int(rng.integers(0, L - 1500))
            b[a:a + 1200] = np.frombuffer((b"CA" * 600), np.uint8)
        if L >= 100000:  # assembly gaps of 1000-1500 Ns
            for a in range(9000, L - 3000, 15000):
                b[a:a + int(rng.integers(1000, 1500))] = ord("N")
        seqs.append(b.tobytes())
    return seqs, lens


def test_pieces_cut_in_n_gaps_equal_whole(oracle):
    """The library's shard plan (ks_shard_plan via dist.shard_pieces: contigs
    cut in the middle of N gaps of >= 1000 bases when whole contigs do not
    balance), the pieces scanned and counted per shard and merged with the
    pieces' offsets == the whole genome's scan and counts, bit for bit
    (kmer_regions and 1-based tr_lr)."""
    from kmer_spans_amd import dist
    O = oracle
    k = 6
    seqs, lens = _gapped_genome(11)
    psh = dist.shard_pieces(seqs, 3)
    rows = sorted((q, lo, hi) for sh in psh for q, lo, hi in sh)
    # every non-empty sequence covered once, in order, by its pieces
    for q, L in enumerate(lens):
        mine = [(lo, hi) for qq, lo, hi in rows if qq == q]
        assert mine[0][0] == 0 and mine[-1][1] == L
        assert all(a[1] == b[0] for a, b in zip(mine, mine[1:]))
        for lo, _ in mine[1:]:  # a cut lies inside an N gap of >= 1000 bases
            s = seqs[q]
            assert s[lo - 1:lo + 1] == b"NN"
            a = lo
            while a > 0 and s[a - 1:a] == b"N":
                a -= 1
            e = lo
            while e < L and s[e:e + 1] == b"N":
                e += 1
            assert e - a >= 1000
    assert sum(1 for r in rows if r[0] == 0) >= 3  # the dominant contig was cut
    loads = [sum(hi - lo for _, lo, hi in sh) for sh in psh]
    assert max(loads) / (sum(lens) / 3) < 1.15
    for sh in psh:
        assert sh == sorted(sh)
    ids = [[q for q, _, _ in sh] for sh in psh]
    offs = [[lo for _, lo, _ in sh] for sh in psh]
    piece_seqs = [[seqs[q][lo:hi] for q, lo, hi in sh] for sh in psh]
    h = sum(O.kmer_counts(ps, k)[1].astype(np.int64) for ps in piece_seqs if ps)
    _, c = O.kmer_counts(seqs, k)
    assert np.array_equal(h, c)
    w = O.log2_table(c, k)
    full = O.scan(seqs, k, w, 0.0, 20, 3.0)
    rs = [O.scan(ps, k, w, 0.0, 20, 3.0) for ps in piece_seqs]
    pos, score = dist.merge_shards(ids, [r["pos"] for r in rs], [r["score"] for r in rs], offsets=offs)
    assert full["pos"].shape[1] > 5
    assert np.array_equal(pos, full["pos"])
    assert np.array_equal(score.view(np.uint64), full["score"].view(np.uint64))
    tfull = O.tr_lr_regions(seqs, k, 15, w, w)
    ts = [O.tr_lr_regions(ps, k, 15, w, w) for ps in piece_seqs]
    tpos, tscore = dist.merge_shards(ids, [t["pos"] for t in ts], [t["score"] for t in ts], one_based=True,
                                     offsets=offs)
    assert np.array_equal(tpos, tfull["pos"])
    assert np.array_equal(tscore.view(np.uint64), tfull["score"].view(np.uint64))


def test_shard_plan_grch38_balance():
    """The planner on GRCh38-shaped contig lengths with 10 kb N gaps every
    ~5 Mbp (lengths scaled 1/100): whole contigs at 2 shards, gap cuts that
    bring the 8-shard maximum to within 1 % of the mean."""
    from kmer_spans_amd import dist, genome
    lens = [L // 100 for L in genome.GRCH38]
    seqs = []
    for L in lens:
        b = np.full(L, ord("A"), np.uint8)
        for a in range(20000, L - 20000, 50000):
            b[a:a + 1000] = ord("N")
        seqs.append(b)
    for n, tol in ((2, 1.005), (4, 1.01), (8, 1.01)):
        psh = dist.shard_pieces(seqs, n)
        loads = [sum(hi - lo for _, lo, hi in sh) for sh in psh]
        assert sum(loads) == sum(lens)
        assert max(loads) / (sum(lens) / n) < tol, (n, max(loads) / (sum(lens) / n))
