"""The multi-GPU path's collectives on the GPU with RCCL (torch.distributed
backend "nccl"): a world of one rank on the one GPU of the test box, so the
code the 8-GPU scaling run executes -- the exact int32 count all-reduce, the
span-record gather to rank 0 and the merge with the pieces' offsets
(kmer_spans_amd/dist.py) -- runs on device tensors and device-
scanned records, checked against the oracle.  The reference pattern it
replaces: mclapply over scaffolds (test.R:550-567) around kmer_regions_r
(kmer_spans.c:490-546)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _genome():
    """Three contigs; the first carries 1-1.5 kb N gaps the planner cuts in."""
    rng = np.random.default_rng(12)
    out = []
    for L in (3_000_000, 800_000, 1_200_000):
        b = np.frombuffer(b"ACGTacgt", dtype=np.uint8)[rng.integers(0, 8, size=L)].copy()
        for a in range(150_000, L - 5000, 400_000):
            b[a:a + int(rng.integers(1000, 1500))] = ord("N")
        for a in range(60_000, L - 5000, 500_000):
            b[a:a + 2400] = np.frombuffer(b"CA" * 1200, np.uint8)
        out.append(b)
    return out


def test_rccl_world1_allreduce_gather_merge(oracle, capsys):
    """RCCL world of one: the genome planned into two shards by the library's
    planner (dist.shard_pieces), each shard counted and scanned on the GPU;
    the shard histograms all-reduced on the device (RCCL) and summed == the
    oracle's counts; each shard's records gathered through RCCL and merged
    with the pieces' offsets == the oracle's scan of the whole genome."""
    import torch
    import torch.distributed as tdist
    from kmer_spans_amd import _lib, api, device as D, dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert tdist.get_backend() == "nccl"
        with capsys.disabled():
            print(f"\n[rccl] backend {tdist.get_backend()} RCCL {torch.cuda.nccl.version()}")
        host = _genome()
        k = 11
        psh = dist.shard_pieces(host, 2)
        assert sum(len(sh) for sh in psh) > 3  # cut in the gaps
        ctx = _lib.context(0)
        D.bind_torch_stream(ctx)
        dss = []
        total = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
        words = 0.0
        for sh in psh:
            parts = [torch.from_numpy(host[q][lo:hi].copy()).cuda() for q, lo, hi in sh]
            ds = D.from_parts(parts, [hi - lo for _, lo, hi in sh], "cuda")
            dss.append(ds)
            h = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
            words += D.count(ctx, ds, k, h)
            dist.allreduce_histogram(h)  # RCCL all-reduce on the device histogram
            total += h
        n_all, oc = oracle.kmer_counts([x.tobytes() for x in host], k)
        assert np.array_equal(total.cpu().numpy(), oc) and words == n_all
        w = api.log2_table(oc, k)
        tab = D.DeviceTable(ctx, w, k, 0.0, compress=True, expand=True, freq=total)
        P, S = [], []
        for ds in dss:
            pos, score, _ = D.scan(ctx, ds, k, tab, 100, 20.0)
            gp, gs = dist.gather_regions(pos, score, torch.device("cuda", 0))  # RCCL all_gather + gather
            assert len(gp) == 1 and np.array_equal(gp[0], pos)
            assert np.array_equal(gs[0].view(np.uint64), score.view(np.uint64))
            P.append(gp[0])
            S.append(gs[0])
        tab.close()
        ids = [[q for q, _, _ in sh] for sh in psh]
        offs = [[lo for _, lo, _ in sh] for sh in psh]
        mpos, mscore = dist.merge_shards(ids, P, S, offsets=offs)
        o = oracle.scan([x.tobytes() for x in host], k, w, 0.0, 100, 20.0)
        assert o["pos"].shape[1] > 3
        assert np.array_equal(mpos, o["pos"])
        assert np.array_equal(mscore.view(np.uint64), o["score"].view(np.uint64))
    finally:
        tdist.destroy_process_group()


def test_bench_force_dist_runs_the_rccl_path(tmp_path):
    """bench.py --gpus 1 --force-dist: the driver's multi-GPU command path
    (process group over RCCL, count all-reduce, record gather + merge, parity
    reduced over ranks) at a small scale, as one rank: the line names the
    nccl backend, the merged records are in (seq_id, beg) order and equal the
    oracle's."""
    out = tmp_path / "b.json"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--force-dist", "--scale", "0.02",
           "--steps", "2", "--warmup", "1", "--no-host-path", "--no-rank", "--no-visits", "--cpu-sample", "2e6",
           "--out", str(out)]
    env = dict(os.environ)
    for key in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(key, None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(out.read_text())
    assert line["dist"]["backend"] == "nccl"
    assert line["merged_order_ok"] is True
    assert line["parity_sample"] is True
    assert line["n_gpus"] == 1 and line["value"] > 0
