#!/usr/bin/env python3
"""Benchmark of the span-scan hot path (BASELINE.json metric):

  Gbases/sec scanned, k=13, log-ratio score, 3.1 Gbp human-shaped genome,
  spans bit-exact.

One *step* = one ks_scan_dev pass (run segmentation + scan + region
ordering/D2H) over the whole device-resident genome.  The genome is
synthetic (kmer_spans_amd.genome.human_like, GRCh38 contig lengths, repeats
and N gaps) and generated on the GPU; the log2(f/f_med) table is built from
the genome's own k-mer counts before timing.  With N ranks (torchrun), every
rank scans its own genome (different seed): weak scaling, no collective on
the data path; span records are gathered to rank 0 over RCCL after timing.

Prints ONE JSON line on rank 0 (the driver's contract) with the roofline of
the dominant kernel (timed with hipEvents on the library's stream inside the
timed steps) and the CPU oracle timed on a bounded sample on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
ALGO_BYTES_PER_BASE = 9.0      # 1 B sequence + 8 B FP64 table entry (k >= 8)
RANDOM_WALL_GPS = 48.0         # measured random-request ceiling (profiles/r1_gather_bench2.jsonl)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--scale", type=float, default=1.0, help="genome scale (1.0 = 3.09 Gbp)")
    p.add_argument("--k", type=int, default=13)
    p.add_argument("--score", choices=["log2", "pm1", "rank"], default="log2")
    p.add_argument("--trlr", action="store_true",
                   help="scan with tr_lr_regions semantics (transition = init = the score table)")
    p.add_argument("--min-width", type=int, default=100)
    p.add_argument("--min-score", type=float, default=20.0)
    p.add_argument("--algo", type=int, default=-1, help="-1 auto, 0 lane-per-run, 1 chunked")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--cpu-sample", type=float, default=2.0e8, help="bases in the CPU-baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-expand", action="store_true", help="do not build the expanded (k+J-1)-mer table")
    p.add_argument("--ncontigs", type=int, default=24, help="1 = the chr1-like single contig of config 2")
    p.add_argument("--host-path", action="store_true",
                   help="also time the host-pointer entry point (ks_kmer_regions: staging + PCIe + scan)")
    p.add_argument("--out", default=None, help="also write the JSON line to this file")
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    ndev = torch.cuda.device_count()
    gpu = local % max(ndev, 1)  # ranks > GPUs only when rehearsing N>1 on a small box
    if dist:
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if ndev >= world:  # one process per GPU: RCCL over xGMI
            tdist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:              # rehearsal with shared GPUs: RCCL refuses duplicate GPUs
            tdist.init_process_group("gloo")
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

    from kmer_spans_amd import _lib, api, genome
    from kmer_spans_amd import device as D

    k = args.k
    ctx = _lib.context(gpu)
    D.bind_torch_stream(ctx)
    if args.algo >= 0:
        ctx.set_scan_algo(args.algo)

    # ---- synthetic genome (device-resident) + score table from its counts
    t0 = time.time()
    parts, lens = genome.human_like(scale=args.scale, seed=args.seed + 1000 * rank, device=dev,
                                    ncontigs=args.ncontigs)
    ds = D.from_parts(parts, lens, dev)
    del parts
    torch.cuda.synchronize()
    t_gen = time.time() - t0
    counts = torch.zeros(4 ** k, dtype=torch.int32, device=dev)
    t0 = time.time()
    words = D.count(ctx, ds, k, counts)
    torch.cuda.synchronize()
    t_count = time.time() - t0
    hc = counts.cpu().numpy()
    thr = 0.0
    if args.score == "log2":
        w = api.log2_table(hc, k)
    elif args.score == "pm1":
        w = api.pm1_table(hc, k)
    else:
        w, thr = api.rank_table(hc, k, words), 0.75
    t0 = time.time()
    if args.trlr:  # tr_lr tables carry no threshold: transition = init = w - thr
        w, thr = np.asarray(w, dtype=np.float64) - thr, 0.0
    table = D.DeviceTable(ctx, w, k, thr, compress=True, expand=not args.no_expand, freq=counts)
    init_table = D.DeviceTable(ctx, w, k, thr, compress=False) if args.trlr else None
    torch.cuda.synchronize()
    t_table = time.time() - t0

    def step():
        if args.trlr:
            return D.tr_lr(ctx, ds, k, table, init_table, args.min_width)
        return D.scan(ctx, ds, k, table, args.min_width, args.min_score)

    for _ in range(args.warmup):
        step()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        pos, score, st = step()
        stats.append(st)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev if tdist.get_backend() == "nccl" else "cpu")
        tdist.all_reduce(e, op=tdist.ReduceOp.MAX)
        elapsed = float(e.item())

    n_bases = int(stats[-1]["n_bases"])
    total_bases = n_bases * world
    ms_step = elapsed / args.steps * 1e3
    value = total_bases / (elapsed / args.steps) / 1e9

    # ---- span records to rank 0 (RCCL gather; not on the timed path)
    n_regions_all = int(pos.shape[1])
    if dist:
        from kmer_spans_amd.dist import gather_regions
        allpos, _ = gather_regions(pos, score, dev)
        n_regions_all = sum(int(p.shape[1]) for p in allpos) if rank == 0 else n_regions_all

    # ---- dominant kernel roofline (hipEvents on the library stream)
    ms_kernel = float(np.mean([s["ms_scan"] for s in stats]))
    achieved = ALGO_BYTES_PER_BASE * n_bases / (ms_kernel * 1e-3) / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                "kernel": "k_scan_lane" if stats[-1]["scan_algo"] == 0 else "k_pass1p",
                "kernel_ms": round(ms_kernel, 3), "algo_bytes_per_base": ALGO_BYTES_PER_BASE}
    # HBM traffic per launch of the dominant kernel: rocprofv3 PMC passes of this
    # same workload (tools/gpu_pmc.sh), committed under profiles/
    pmc_path = os.path.join(ROOT, "profiles", "r1_pmc_summary.json")
    if os.path.exists(pmc_path) and stats[-1]["scan_algo"] == 1 and not args.trlr:
        pmc = json.load(open(pmc_path))
        wl = pmc.get("workload", {})
        if (wl.get("k") == k and wl.get("score") == args.score and wl.get("scale") == args.scale
                and wl.get("ncontigs") == args.ncontigs and not args.no_expand):
            for name, cs in pmc.get("kernels", {}).items():
                if name.startswith("k_pass1") and "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
                    roofline["traffic"] = round((cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1e3)  # KB -> B
                    roofline["traffic_source"] = f"profiles/r1_pmc_summary.json ({name}, FETCH+WRITE)"
                    roofline["traffic_note"] = "PMC pass of the same workload and build (tools/gpu_pmc.sh), not this run"
                    break

    # ---- the bound that applies to a gather pass: random requests.  Every
    # table read of k_pass1p is one random request (64-B fetch) whatever its
    # width; the chip's measured ceiling for such requests from tables of
    # 32-128 GiB is ~48 G/s (tools/gather_bench2.hip, profiles/r1_gather_bench2.jsonl:
    # u64 entries 47.2-49.1 G/s).  Reported beside the HBM-bytes roofline.
    if stats[-1]["scan_algo"] == 1:
        J = max(1, int(table.positions_per_read))
        n_scored = int(stats[-1]["n_scored"])
        reads = n_scored / J + (n_scored * float(table.escape_fraction) if table.code_bits == 12 else 0.0)
        ra = {"table_reads_per_launch": int(reads), "positions_per_read": J,
              "achieved_G_per_s": round(reads / (ms_kernel * 1e-3) / 1e9, 2), "wall_G_per_s": RANDOM_WALL_GPS,
              "frac": round(reads / (ms_kernel * 1e-3) / 1e9 / RANDOM_WALL_GPS, 4),
              "wall_source": "profiles/r1_gather_bench2.jsonl (random u64 reads, 32-128 GiB tables)"}
        if roofline.get("traffic") and roofline.get("traffic_source", "").find("FETCH") >= 0:
            pmc = json.load(open(pmc_path))
            for name, cs in pmc.get("kernels", {}).items():
                if name.startswith("k_pass1p") and "FETCH_SIZE" in cs:
                    req = cs["FETCH_SIZE"] * 1e3 / 64.0  # FETCH_SIZE = TCC_EA0_RDREQ x 64 B
                    ra["memory_read_requests_per_launch"] = int(req)
                    ra["memory_requests_G_per_s"] = round(req / (ms_kernel * 1e-3) / 1e9, 2)
                    break
        roofline["random_access"] = ra

    # ---- PCIe-inclusive rate of the host entry point (reported, never `value`)
    host_path = None
    if args.host_path and rank == 0 and not args.trlr:
        hs = [ds.host_seq(q) for q in range(ds.nseq)]
        t0 = time.perf_counter()
        hr = api.kmer_regions(hs, k, w, args.min_width, args.min_score, visits=False) if thr == 0.0 else None
        t_host = time.perf_counter() - t0
        if hr is not None:
            host_path = {"seconds": round(t_host, 4), "Gbases_per_s": round(n_bases / t_host / 1e9, 3),
                         "regions_equal": bool(np.array_equal(hr["pos"], pos)),
                         "note": "ks_kmer_regions from host memory: pinned staging + H2D + table upload/compress + scan"}
        del hs

    # ---- CPU baseline: the oracle (single thread) on a bounded sample
    cpu = None
    parity = None
    if rank == 0 and not args.no_cpu:
        from oracle import oracle as O
        order = np.argsort(np.diff(ds.offsets))
        ids, acc = [], 0
        for q in order:  # smallest contigs first until the sample size is reached
            ids.append(int(q))
            acc += int(ds.offsets[q + 1] - ds.offsets[q])
            if acc >= args.cpu_sample:
                break
        ids.sort()
        host = [ds.host_seq(q) for q in ids]
        t0 = time.perf_counter()
        if args.trlr:
            o = O.tr_lr_regions(host, k, args.min_width, w, w)
        else:
            o = O.scan(host, k, w, thr, args.min_width, args.min_score)
        t_cpu = time.perf_counter() - t0
        cpu = {"value": round(acc / t_cpu / 1e9, 5), "unit": "Gbases/s", "cores": 1, "kind": "port",
               "sample": f"oracle/ks_oracle.c scan of {len(ids)} contigs ({acc} bp) of the same genome, same table",
               "seconds": round(t_cpu, 3), "host_cpu": cpu_model(), "host_nproc": os.cpu_count()}
        # parity of the sampled contigs: GPU records vs oracle records
        one = 1 if args.trlr else 0  # tr_lr ids are 1-based
        sel = np.isin(pos[0] - one, ids)
        gp = pos[:, sel].copy()
        remap = {q: i for i, q in enumerate(ids)}
        gp[0] = [remap[int(x) - one] + one for x in gp[0]]
        gs = score[:, sel]
        parity = bool(np.array_equal(gp, o["pos"]) and
                      np.array_equal(gs.view(np.uint64), o["score"].view(np.uint64)))

    line = {
        "metric": "Gbases/sec scanned (k=13, log-ratio score) at 1/2/4/8 MI355X; spans bit-exact",
        "value": round(value, 4), "unit": "Gbases/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"human-shaped synthetic genome ({n_bases} bp, {ds.nseq} contigs, scale {args.scale}), "
                               f"k={k}, {args.score} score from its own counts, min_width {args.min_width}, "
                               f"min_score {args.min_score}, device-resident",
                   "k": k, "score": args.score, "genome_bp": n_bases, "parallelism": f"contig-shard x{world}",
                   "scan": "tr_lr_regions" if args.trlr else "kmer_regions",
                   "scan_algo": int(stats[-1]["scan_algo"]), "table_compressed": table.compressed,
                   "table_distinct": table.distinct, "positions_per_read": table.positions_per_read,
                   "code_bits": table.code_bits, "escape_fraction": round(table.escape_fraction, 6)},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "parity_sample": parity,
        "regions": n_regions_all,
        "replayed_chunks": int(stats[-1]["n_replay"]),
        "host_path": host_path,
        "phase_ms": {key: round(float(np.mean([s[key] for s in stats])), 3)
                     for key in ("ms_runs", "ms_scan", "ms_rescan", "ms_finish", "ms_total")},
        "setup_s": {"genome": round(t_gen, 2), "count": round(t_count, 3), "table": round(t_table, 3)},
    }
    if rank == 0:
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(s + "\n")
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
