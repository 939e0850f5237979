#!/usr/bin/env python3
"""Benchmark of the span-scan hot path (BASELINE.json metric):

  Gbases/sec scanned, k=13, log-ratio score, 3.1 Gbp human-shaped genome,
  spans bit-exact, at 1/2/4/8 MI355X.

One *step* = one ks_scan_dev pass (run segmentation + scan + region
ordering/D2H) over the device-resident sequences of a rank.  Genomes are
synthetic (kmer_spans_amd.genome: GRCh38 contig lengths, repeats, N gaps),
generated on the GPU from seeds; the score table is built from the genome's
own k-mer counts before timing (the table is an input of
kmer_regions_r), and its cost is reported beside the value as `setup_ms` and
an end-to-end rate.

Multi-GPU: `python bench.py --gpus N` starts N ranks itself
(one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE set before any HIP call in
the children; the parent never touches the GPU and kills the other ranks as
soon as one fails), or runs as one rank under torchrun.  Backend "nccl" (RCCL
over xGMI) when every rank has its own GPU, gloo for rehearsals with more
ranks than GPUs.  Modes:
  shard   (default; strong scaling, the north-star curve) ONE genome, contigs
          LPT-sharded over the ranks; per-rank counts summed with an exact
          int32 all-reduce before the table is built; records gathered to
          rank 0 and merged (dist.merge_shards).  At N=1 this is the whole
          genome (the same seeds as `genome`).
  genome  (weak scaling) every rank scans its own genome.
  genomes (config 5) every rank processes --genomes-per-rank genomes; each
          timed end to end: count + table (+ expanded table) + scan.
No collective runs on the data path: the only exchanges are the count
all-reduce (shard) and the record gather after timing.

Prints ONE JSON line on rank 0 (the driver's contract) with the roofline of
the dominant kernel (hipEvents on the library's stream inside the timed
steps), and after timing: the parity verdict of EVERY contig (the CPU oracle
on a thread pool, per rank on its own shard), at N=1 the CPU oracle timed on
one pinned core over a bounded sample, the weighted-rank sub-line (BASELINE
config 3, `configs.rank`, same genome and counts) with its own all-contig
parity, the visit-histogram line and the host-pointer entry point.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
ALGO_BYTES_PER_BASE = 9.0      # 1 B sequence + 8 B FP64 table entry (k >= 8)
ALGO_BYTES_PER_BASE_LDS = 1.0  # k <= 7, the table LDS-staged (k_pass1_lds): the sequence byte only


def algo_bytes_per_base(kernel: str) -> float:
    """SURVEY 8(d)'s algorithmic bytes per scanned base of the dominant
    kernel: 1 B when the table lives in LDS (k <= 7, k_pass1_lds), else 9 B."""
    return ALGO_BYTES_PER_BASE_LDS if kernel.startswith("k_pass1_lds") else ALGO_BYTES_PER_BASE
RANDOM_WALL_GPS = 50.0         # measured random-request ceiling, contiguous 128 GiB table (profiles/r2/frag_probe.txt)
# Random 128-B line reads from a 128 GiB table (the wide-line table's size):
# 48.2 G lines/s = 6.17 TB/s of line bytes, the chip's measured ceiling for
# this access; rocprofv3 FETCH_SIZE counts 64 B per such read (one 128-B
# request tallied at 64 B, as the guide's gfx950 note says of wide streaming
# reads), 64 B per 32- or 64-B line read (profiles/r6/linecal/line_rates.txt)
LINE128_CEILING_GBS = 6170.0
FETCH_B_PER_READ = {"k_pass1w": 128.0}   # physical bytes per FETCH_SIZE-tallied 64 B request: line bytes
METRIC = "Gbases/sec scanned (k=13, log-ratio score) at 1/2/4/8 MI355X; spans bit-exact"
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1, help="ranks to run (one process per GPU)")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--mode", choices=["shard", "genome", "genomes"], default="shard")
    p.add_argument("--genomes-per-rank", type=int, default=2, help="--mode genomes: genomes per rank")
    p.add_argument("--count-priority", type=int, default=None,
                   help="genomes mode, pipelined: the next genome's count/table stream priority (torch's scale)")
    p.add_argument("--genomes-serial", action="store_true",
                   help="--mode genomes: no overlap of genome g+1's count and table with genome g's scan")
    p.add_argument("--scale", type=float, default=1.0, help="genome scale (1.0 = 3.09 Gbp)")
    p.add_argument("--k", type=int, default=13)
    p.add_argument("--score", choices=["log2", "pm1", "rank"], default="log2")
    p.add_argument("--trlr", action="store_true",
                   help="scan with tr_lr_regions semantics (transition = init = the score table)")
    p.add_argument("--min-width", type=int, default=100)
    p.add_argument("--min-score", type=float, default=20.0)
    p.add_argument("--algo", type=int, default=-1, help="-1 auto, 0 lane-per-run, 1 chunked")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--shard-of", type=int, default=1,
                   help="(one rank) scan only one shard of an N-way LPT split of the genome, with the whole "
                        "genome's table: the fixed per-step cost at shard size")
    p.add_argument("--shard-index", type=int, default=-1, help="--shard-of: which shard (default: the largest)")
    p.add_argument("--whole-contigs", action="store_true",
                   help="shard mode: LPT over whole contigs instead of pieces cut inside N gaps")
    p.add_argument("--cpu-sample", type=float, default=2.0e8,
                   help="bases of the timed CPU-baseline sample besides the largest contig")
    p.add_argument("--cpu-threads", type=int, default=16, help="host threads of the (untimed) parity leg")
    p.add_argument("--parity", choices=["all", "sample", "none"], default="all",
                   help="contigs compared with the CPU oracle after timing")
    p.add_argument("--no-cpu", action="store_true", help="no CPU baseline, no parity leg")
    p.add_argument("--no-rank", action="store_true", help="skip the weighted-rank sub-line (N=1 default line)")
    p.add_argument("--rank-steps", type=int, default=5)
    p.add_argument("--no-visits", action="store_true",
                   help="skip the visits_path line (profiling runs: its scans run beside a concurrent count)")
    p.add_argument("--no-host-path", action="store_true", help="skip the host-pointer entry point line")
    p.add_argument("--no-expand", action="store_true", help="do not build the expanded (k+J-1)-mer table")
    p.add_argument("--ext-max-gib", type=float, default=None,
                   help="cap on the expanded table (GiB); default: no cap beyond HBM (J = 5, 128 GiB at k = 13) "
                        "for the scan modes, 32 GiB (J = 4) for --mode genomes, where it is built per genome")
    p.add_argument("--ncontigs", type=int, default=24, help="1 = the chr1-like single contig of config 2")
    p.add_argument("--out", default=None, help="also write the JSON line to this file")
    p.add_argument("--force-dist", action="store_true",
                   help="run the torch.distributed path (RCCL with one GPU per rank) even at --gpus 1: a world of "
                        "one rank, so the multi-GPU code (count all-reduce, record gather + merge) runs on one GPU")
    p.add_argument("--multi-devices", default="0,0",
                   help="N=1: device list of the multi-device host-entry line (ks_set_devices; '' skips it)")
    return p.parse_args(argv)


# ----------------------------------------------------------------- launcher

def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(n: int, argv=None) -> int:
    """Start n ranks of this script as child processes (the parent makes no
    HIP call: it only sets the rank environment) and return the worst exit
    code.  The children are polled: when one exits non-zero the others are
    killed at once instead of blocking in a collective until its timeout."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] +
                                      (sys.argv[1:] if argv is None else argv), env=env))
    worst = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            worst = max(worst, abs(rc))
            if rc != 0:
                for q in live:
                    q.kill()
                for q in live:
                    q.wait()
                    worst = max(worst, abs(q.returncode or 0))
                live = []
                break
        time.sleep(0.1)
    return worst


# ------------------------------------------------------------------ helpers

def pmc_traffic(kernel_prefix, build_id, workload):
    """HBM bytes per step of the dominant kernel (all its launches: pass 1
    runs as two launches, one per part of the runs) from the committed PMC
    passes (tools/gpu_pmc.sh + tools/pmc_assemble.py -> profiles/
    pmc_summary.json), used only when they were taken on this very build
    (library build id) and workload.
    FETCH_SIZE counts 64 B per memory-side read request; the kernel's only
    streaming read (the packed bases, total/4 bytes, 16-B loads) is under-
    counted by half on gfx950 (MI355X_MICROARCH.md, HBM), so that half is
    added back; WRITE_SIZE is exact for the 8-B stores."""
    if not os.path.exists(PMC_SUMMARY):
        return None, "no PMC summary"
    pmc = json.load(open(PMC_SUMMARY))
    if pmc.get("build_id") != build_id:
        return None, f"stale: PMC summary of build {pmc.get('build_id')}, this library is {build_id}"
    want = {key: workload.get(key) for key in pmc.get("workload", {})}
    if pmc.get("workload") != want:
        return None, "PMC summary is for another workload"
    steps = float(pmc.get("steps", 1))
    fetch = write = 0.0
    names = []
    for name, cs in pmc.get("kernels", {}).items():
        if name.startswith(kernel_prefix) and "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            n = cs.get("dispatches", 1) / steps  # launches per step (pass 1: one per part of the runs)
            fetch += cs["FETCH_SIZE"] * 1e3 * n
            write += cs["WRITE_SIZE"] * 1e3 * n
            names.append(name)
    if names:
        # gfx950 corrections (MI355X_MICROARCH.md HBM section; calibrated on this
        # access pattern in profiles/r6/linecal/line_rates.txt): the packed-base
        # stream (16-B loads) is tallied at half its bytes; each table line read
        # is one request tallied at 64 B, which moves 128 B for a 128-B wide line
        stream = pmc.get("streaming_read_bytes_per_step", {}).get(kernel_prefix, 0.0)
        line_fetch = max(0.0, fetch - stream / 2.0)  # the tallied bytes of the table reads
        per_req = FETCH_B_PER_READ.get(kernel_prefix, 64.0)
        corrected = line_fetch / 64.0 * per_req + stream + write
        return {"bytes": int(round(corrected)), "fetch": int(fetch), "write": int(write),
                "streaming_read": int(stream), "table_read_requests": int(line_fetch / 64.0),
                "bytes_per_table_request": per_req, "kernels": names,
                "correction": "FETCH_SIZE counts 64 B per request: the packed-base stream's half is added back and "
                              "each table read counts its line's bytes (128 B for wide lines: calibrated, "
                              "profiles/r6/linecal/line_rates.txt)",
                "per": "step (all launches of the kernel)"}, "ok"
    return None, "kernel not in the PMC summary"


def sample_ids(offsets, budget):
    """Contigs of the timed CPU sample: the largest one (longest carry chain
    at the metric config) plus the smallest ones up to `budget` more bases."""
    lens = np.diff(offsets)
    big = int(np.argmax(lens))
    ids, acc = [big], int(lens[big])
    for q in np.argsort(lens):
        q = int(q)
        if q == big:
            continue
        if acc - int(lens[big]) >= budget:
            break
        ids.append(q)
        acc += int(lens[q])
    return sorted(ids), acc


def host_contigs(ds):
    """Every sequence's bytes on the host (one D2H copy), as numpy views."""
    buf = ds.seq[:max(ds.total, 1)].cpu().numpy()
    return [buf[int(a):int(b)] for a, b in zip(ds.offsets[:-1], ds.offsets[1:])]


class Oracle:
    """The CPU oracle (oracle/, test infrastructure) as the checker of one
    scan configuration: per-contig records on a host thread pool (ctypes
    releases the GIL), the timed single-core baseline, the all-contig
    parity verdict."""

    def __init__(self, host, k, w, thr, min_width, min_score, trlr, threads):
        from oracle import oracle as O
        self.O = O
        self.host, self.k, self.w, self.thr = host, k, w, thr
        self.mw, self.ms, self.trlr = min_width, min_score, trlr
        self.one = 1 if trlr else 0
        self.threads = max(1, min(threads, len(os.sched_getaffinity(0))))
        self.per = {}  # contig -> (pos, score) with seq id = the contig's own

    def _run(self, seqs):
        if self.trlr:
            return self.O.tr_lr_regions(seqs, self.k, self.mw, self.w, self.w)
        return self.O.scan(seqs, self.k, self.w, self.thr, self.mw, self.ms)

    def _keep(self, ids, o):
        for i, q in enumerate(ids):
            sel = o["pos"][0] - self.one == i
            p = o["pos"][:, sel].copy()
            p[0] = q + self.one
            self.per[q] = (p, o["score"][:, sel])

    def baseline(self, ids):
        """Single-thread timing on one pinned core (the reference is single
        threaded); the records are kept for the parity verdict."""
        old = os.sched_getaffinity(0)
        os.sched_setaffinity(0, {min(old)})
        try:
            t0 = time.perf_counter()
            o = self._run([self.host[q] for q in ids])
            t = time.perf_counter() - t0
        finally:
            os.sched_setaffinity(0, old)
        self._keep(ids, o)
        return t

    def fill(self, ids):
        """Records of the given contigs (largest first) on the thread pool."""
        todo = sorted((q for q in ids if q not in self.per), key=lambda q: -self.host[q].size)
        with ThreadPoolExecutor(self.threads) as ex:
            for q, o in zip(todo, ex.map(lambda q: self._run([self.host[q]]), todo)):
                self._keep([q], o)

    def visits_sum(self, ids):
        """The oracle's visit histogram of kmer_regions_r (kmer_spans.c:266-267,
        every visited index including the restart loop's re-visits) over the
        given contigs: per-contig histograms on the thread pool, summed as
        the reference's int32 counts (uint32 wrap-around)."""
        total = np.zeros(4 ** self.k, dtype=np.uint32)
        todo = sorted(ids, key=lambda q: -self.host[q].size)

        def one(q):
            return self.O.scan([self.host[q]], self.k, self.w, self.thr, self.mw, self.ms, visits=True)["counts"]
        with ThreadPoolExecutor(self.threads) as ex:
            for v in ex.map(one, todo):
                total += v.view(np.uint32)
        return total

    def parity(self, pos, score, ids):
        """GPU records restricted to contigs ids equal the oracle's, bitwise."""
        ids = sorted(ids)
        sel = np.isin(pos[0] - self.one, ids)
        ps = [self.per[q][0] for q in ids]
        ss = [self.per[q][1] for q in ids]
        op = np.concatenate(ps, axis=1) if ps else np.zeros((3, 0), np.int32)
        osc = np.concatenate(ss, axis=1) if ss else np.zeros((2, 0), np.float64)
        return bool(np.array_equal(pos[:, sel], op) and
                    np.array_equal(score[:, sel].view(np.uint64), osc.view(np.uint64)))


class Timer:
    """Wall time of device work: synchronize on both sides."""

    def __enter__(self):
        torch.cuda.synchronize()
        self.t = time.perf_counter()
        return self

    def __exit__(self, *a):
        torch.cuda.synchronize()
        self.ms = (time.perf_counter() - self.t) * 1e3


def phase_means(stats):
    return {key[3:]: round(float(np.mean([s[key] for s in stats])), 3) for key in stats[-1] if key.startswith("ms_")}


# --------------------------------------------------------------------- main

def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(args.gpus))
    if args.force_dist and "WORLD_SIZE" not in os.environ:  # a world of one rank (no HIP call yet)
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(_free_port()))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1 or args.force_dist
    ndev = torch.cuda.device_count()
    gpu = local % max(ndev, 1)  # ranks > GPUs only when rehearsing N>1 on a small box
    tdist = None
    if dist:
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if ndev >= world:  # one process per GPU: RCCL over xGMI
            tdist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:              # rehearsal with shared GPUs: RCCL refuses duplicate GPUs
            tdist.init_process_group("gloo")
        extra_dist = {"backend": tdist.get_backend(), "world": world}
        if tdist.get_backend() == "nccl":
            try:
                extra_dist["rccl_version"] = ".".join(str(x) for x in torch.cuda.nccl.version())
            except Exception:
                pass
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

    from kmer_spans_amd import _lib, api, genome
    from kmer_spans_amd import device as D

    k = args.k
    ctx = _lib.context(gpu)
    D.bind_torch_stream(ctx)
    if args.algo >= 0:
        ctx.set_scan_algo(args.algo)
    build_id = _lib.build_id()

    def barrier():
        if dist:
            tdist.barrier()

    def reduce_over_ranks(x: float, op) -> float:
        if not dist:
            return x
        e = torch.tensor([x], dtype=torch.float64, device=dev if tdist.get_backend() == "nccl" else "cpu")
        tdist.all_reduce(e, op=op)
        return float(e.item())

    def max_over_ranks(x: float) -> float:
        return reduce_over_ranks(x, tdist.ReduceOp.MAX if dist else None)

    def make_table(counts, words, score, ext_gib=None, warm=True):
        """Score table built on the device from the device counts
        (ks_table_from_counts: no 4^k host round trip), timed; w (the
        reference's weight vector) stays on the device for the parity leg."""
        t = {}
        thr = 0.75 if score == "rank" else 0.0
        cap = int((ext_gib if ext_gib is not None else (args.ext_max_gib or 0.0)) * (1 << 30))
        w_dev = torch.empty(4 ** k, dtype=torch.float64, device=dev)

        def build():
            return D.DeviceTable.from_counts(ctx, counts, k, score, total=words, thr=thr,
                                             expand=not args.no_expand, max_ext_bytes=cap, w_out=w_dev)
        if warm:  # first build: grows the workspace and allocates the expanded table (fresh VRAM is
            with Timer() as tm:  # cleared by the driver: seconds for 128 GiB), reported apart
                build().close()
            t["table_first_call"] = tm.ms
        with Timer() as tm:
            table = build()
        t["table_device"] = tm.ms
        t.update({f"table_{key}": v for key, v in table.setup_ms().items()})
        init = None
        if args.trlr:  # tr_lr tables carry no threshold: transition = init = w - thr
            init = D.DeviceTable(ctx, w_dev.cpu().numpy() - thr, k, 0.0, compress=False)
        return w_dev, thr, table, init, t

    def scan_once(ds, table, init):
        if args.trlr:
            return D.tr_lr(ctx, ds, k, table, init, args.min_width)
        return D.scan(ctx, ds, k, table, args.min_width, args.min_score)

    def timed_steps(ds, table, init, steps, warmup):
        for _ in range(warmup):
            scan_once(ds, table, init)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        stats = []
        out = None
        for _ in range(steps):
            out = scan_once(ds, table, init)
            stats.append(out[2])
        torch.cuda.synchronize()
        barrier()
        return out[0], out[1], stats, max_over_ranks(time.perf_counter() - t0)

    setup = {}
    extra = {"dist": extra_dist} if dist else {}
    # ------------------------------------------------------------ the input
    t0 = time.time()
    lens_all = [max(1, int(round(L * args.scale))) for L in genome.GRCH38[:args.ncontigs]]
    shards = None
    offsets = None  # per shard: each local sequence's start inside its contig (pieces)
    pieces_mine = None
    if args.mode == "shard":
        from kmer_spans_amd.dist import lpt_shards, shard_pieces
        nsh = world if dist else max(1, args.shard_of)
        if nsh > 1 and not args.whole_contigs:
            # the library's shard plan (ks_shard_plan via dist.shard_pieces: LPT
            # over pieces cut inside N gaps when whole contigs do not balance;
            # exact: runs never cross an N); every rank generates the genome
            # and plans the same cut, so every rank knows every shard's pieces
            parts_all = [genome.contig(lens_all[q], args.seed + q, dev) for q in range(len(lens_all))]
            psh = shard_pieces([x.cpu().numpy() for x in parts_all], nsh)
            shards = [[q for q, _, _ in sh] for sh in psh]
            offsets = [[lo for _, lo, _ in sh] for sh in psh]
            if dist:
                pieces_mine = psh[rank]
            else:
                idx = args.shard_index if args.shard_index >= 0 else int(np.argmax([sum(hi - lo for _, lo, hi in sh)
                                                                                    for sh in psh]))
                pieces_mine = psh[idx]
            mine = [q for q, _, _ in pieces_mine]
            if dist:
                parts = [parts_all[q][lo:hi] for q, lo, hi in pieces_mine]
                ds = D.from_parts(parts, [hi - lo for _, lo, hi in pieces_mine], dev)
            else:  # --shard-of: the whole genome is counted, then only the shard is scanned
                parts = parts_all
                ds = D.from_parts(parts, lens_all, dev)
            del parts_all
        else:
            shards = lpt_shards(lens_all, nsh)
            if dist:
                mine = shards[rank]
            else:
                idx = args.shard_index if args.shard_index >= 0 else int(np.argmax([sum(lens_all[q] for q in s)
                                                                                    for s in shards]))
                mine = shards[idx] if nsh > 1 else list(range(len(lens_all)))
            # --shard-of at one rank: the whole genome is counted (its table is the one the
            # sharded run builds after the all-reduce), then only the shard is scanned
            gen = range(len(lens_all)) if (not dist and nsh > 1) else mine
            parts = [genome.contig(lens_all[q], args.seed + q, dev) for q in gen]
            ds = D.from_parts(parts, [lens_all[q] for q in gen], dev)
        genome_bp = sum(lens_all)
    else:
        mine = None
        parts, lens = genome.human_like(scale=args.scale, seed=args.seed + 1000 * rank, device=dev,
                                        ncontigs=args.ncontigs)
        ds = D.from_parts(parts, lens, dev)
        genome_bp = None
    del parts
    torch.cuda.synchronize()
    setup["genome_s"] = round(time.time() - t0, 2)

    if args.mode == "genomes":
        return run_genomes(args, ctx, ds, dev, rank, world, dist, tdist, barrier, max_over_ranks, make_table, D,
                           genome, build_id)

    # ------------------------------------------------------ counts -> table
    counts = torch.zeros(4 ** k, dtype=torch.int32, device=dev)
    with Timer() as tm:  # the first call also allocates the count's workspace
        words = D.count(ctx, ds, k, counts)
    setup["count_first_call_ms"] = round(tm.ms, 2)
    counts.zero_()
    with Timer() as tm:  # steady state (like table_device)
        words = D.count(ctx, ds, k, counts)
    setup["count_ms"] = round(tm.ms, 2)
    if args.mode == "shard" and dist:  # the table of the whole genome: exact int32 sum of per-shard counts
        from kmer_spans_amd.dist import allreduce_histogram
        with Timer() as tm:
            if tdist.get_backend() == "nccl":
                allreduce_histogram(counts)
                wt = torch.tensor([words], dtype=torch.float64, device=dev)
            else:
                c = counts.cpu()
                allreduce_histogram(c)
                counts.copy_(c)
                wt = torch.tensor([words], dtype=torch.float64)
            tdist.all_reduce(wt)
            words = float(wt.item())
        setup["count_allreduce_ms"] = round(tm.ms, 2)
    if args.mode == "shard" and not dist and args.shard_of > 1:
        if pieces_mine is not None:
            full = ds
            ds = D.from_parts([full.seq[int(full.offsets[q]) + lo:int(full.offsets[q]) + hi] for q, lo, hi in pieces_mine],
                              [hi - lo for _, lo, hi in pieces_mine], dev)
            del full
        else:
            ds = ds.subset(mine)
        torch.cuda.empty_cache()
        extra["shard_of"] = {"n": args.shard_of, "contigs": sorted(set(mine)), "bp": int(ds.total),
                             "pieces": len(pieces_mine) if pieces_mine is not None else None,
                             "note": "one shard of an N-way LPT split (contigs cut inside N gaps) scanned with "
                                     "the whole genome's table"}
    w_dev, thr, table, init_table, tt = make_table(counts, words, args.score)
    setup.update({key: round(v, 2) for key, v in tt.items()})
    table_shape = {"table_compressed": table.compressed, "table_distinct": table.distinct,
                   "line_kind": table.line_kind, "pass1_kernel": table.pass1_kernel,
                   "positions_per_read": table.positions_per_read, "code_bits": table.code_bits,
                   "escape_fraction": round(table.escape_fraction, 6)}

    # ------------------------------------------------------------- timing
    pos, score, stats, elapsed = timed_steps(ds, table, init_table, args.steps, args.warmup)

    n_bases = int(stats[-1]["n_bases"])
    if args.mode == "shard":
        total_bases = genome_bp if (dist or args.shard_of <= 1) else n_bases
    else:
        total_bases = n_bases * world
    ms_step = elapsed / args.steps * 1e3
    value = total_bases / (elapsed / args.steps) / 1e9

    # ---- dominant kernel roofline (hipEvents on the library stream)
    ms_kernel = float(np.mean([s["ms_scan"] for s in stats]))
    kernel = "k_scan_lane" if stats[-1]["scan_algo"] == 0 else table.pass1_kernel
    bpb = algo_bytes_per_base(kernel)
    achieved = bpb * n_bases / (ms_kernel * 1e-3) / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                "kernel": kernel, "kernel_ms": round(ms_kernel, 3), "algo_bytes_per_base": bpb,
                "algo_bytes_per_launch": int(bpb * n_bases)}
    workload = {"k": k, "score": args.score, "scale": args.scale, "ncontigs": args.ncontigs,
                "expand": not args.no_expand, "trlr": args.trlr, "mode": args.mode, "world": world,
                "shard_of": args.shard_of}
    traffic, why = pmc_traffic(kernel, build_id, workload)
    if traffic:
        roofline["traffic"] = traffic["bytes"]
        roofline["traffic_detail"] = traffic
        roofline["traffic_source"] = "profiles/pmc_summary.json (rocprofv3 --pmc passes of this build and workload)"
    else:
        roofline["traffic_note"] = why
    # the bound that applies to a gather pass: random requests (every table
    # read is one 64-B request whatever its width; the chip's measured ceiling
    # for such requests from 32-128 GiB tables is ~48-50 G/s, tools/probes/line_bench.hip)
    # (not for the LDS-staged small-k passes: they make no random HBM reads)
    if stats[-1]["scan_algo"] == 1 and not kernel.startswith("k_pass1_lds"):
        J = max(1, int(table.positions_per_read))
        n_scored = int(stats[-1]["n_scored"])
        esc = float(table.escape_fraction)
        # escapes: 12-bit (k+4)-mer table: per scan index; wide lines (13-bit): per line (its L3 index)
        reads = n_scored / J + (n_scored * esc if table.code_bits == 12 else
                                n_scored / J * esc if table.code_bits == 13 else 0.0)
        ra = {"table_reads_per_launch": int(reads), "positions_per_read": J,
              "achieved_G_per_s": round(reads / (ms_kernel * 1e-3) / 1e9, 2), "wall_G_per_s": RANDOM_WALL_GPS,
              "frac": round(reads / (ms_kernel * 1e-3) / 1e9 / RANDOM_WALL_GPS, 4),
              "wall_source": "profiles/r3/line_bench.txt (random 16-128-B lines from a physically contiguous "
                             "128 GiB buffer, fetched by 1-8 lanes each: 49.9-50.3 G lines/s)"}
        if traffic:
            ra["memory_read_requests_per_launch"] = traffic["table_read_requests"]
            ra["memory_requests_G_per_s"] = round(traffic["table_read_requests"] / (ms_kernel * 1e-3) / 1e9, 2)
        roofline["random_access"] = ra
        if kernel == "k_pass1w":
            # the bytes the wide-line form moves: a whole 128-B line per read
            # (6 positions of 13/11-bit codes plus the 81 continuation codes a
            # read does not use) and the packed bases, against the chip's peak
            # and against the measured ceiling of random 128-B line reads
            pb = reads * 128.0 + n_bases / 4.0
            roofline["physical"] = {
                "bytes_per_launch": int(pb), "bytes_per_position": round(pb / n_scored, 2),
                "achieved": round(pb / (ms_kernel * 1e-3) / 1e9, 1), "unit": "GB/s",
                "frac_of_peak": round(pb / (ms_kernel * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "frac_of_line_ceiling": round(pb / (ms_kernel * 1e-3) / 1e9 / LINE128_CEILING_GBS, 4),
                "line_ceiling_GB_per_s": LINE128_CEILING_GBS,
                "note": "random 128-B line reads cannot move fewer bytes than their lines: at 6 positions per line "
                        "the form's floor is 21.3 B per position against the 9 algorithmic bytes; the ceiling is "
                        "tools/probes/line_bench.hip's 128-B group reads from a 128 GiB table "
                        "(profiles/r6/linecal/line_rates.txt)"}

    # ---- the same step with the visit histogram kmer_regions_r returns
    # (kmer_spans.c:266-267,523-537): device-resident, count-derived top-level
    # visits + rescan visits; not `value` (the metric counts regions only)
    visits_line = None
    vis_host = None
    if world == 1 and not args.trlr and not args.no_visits and stats[-1]["scan_algo"] == 1:
        vis = torch.zeros(4 ** k, dtype=torch.int32, device=dev)
        D.scan(ctx, ds, k, table, args.min_width, args.min_score, visits=vis)  # warm
        vt = []
        for _ in range(3):
            vis.zero_()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            vpos, vscore, _ = D.scan(ctx, ds, k, table, args.min_width, args.min_score, visits=vis)
            torch.cuda.synchronize()
            vt.append(time.perf_counter() - t1)
        tv = float(np.median(vt))
        vsum = int(vis.to(torch.int64).sum().item())
        vis_host = vis.cpu().numpy()
        visits_line = {"ms": round(tv * 1e3, 3), "Gbases_per_s": round(n_bases / tv / 1e9, 3),
                       "regions_equal": bool(np.array_equal(vpos, pos)),
                       "scores_equal": bool(np.array_equal(vscore.view(np.uint64), score.view(np.uint64))),
                       "visits_total": vsum, "scored_positions": int(stats[-1].get("n_scored", 0)),
                       "note": "ks_scan_dev with the visit histogram (device-resident), median of 3"}
        del vis, vpos, vscore

    # ---- span records to rank 0 (RCCL gather; not on the timed path)
    n_regions_all = int(pos.shape[1])
    if dist:
        # the span-record gather (the path's only exchange) and the
        # merge on rank 0, timed beside the step (max over ranks)
        from kmer_spans_amd.dist import gather_regions, merge_shards
        barrier()
        tg = time.perf_counter()
        allpos, allscore = gather_regions(pos, score, dev)
        mpos = None
        if rank == 0 and args.mode == "shard":
            mpos, _ = merge_shards(shards, allpos, allscore, one_based=args.trlr, offsets=offsets)
        gather_ms = max_over_ranks((time.perf_counter() - tg) * 1e3)
        extra["gather_ms"] = round(gather_ms, 3)
        extra["step_plus_gather_ms"] = round(ms_step + gather_ms, 3)
        if rank == 0:
            n_regions_all = sum(int(p.shape[1]) for p in allpos)
            if mpos is not None:
                extra["merged_regions"] = int(mpos.shape[1])
                extra["merged_order_ok"] = bool(np.all(np.diff(mpos[0].astype(np.int64) * (1 << 32) + mpos[1]) > 0))

    w = w_dev.cpu().numpy()
    host = None
    if not args.no_cpu or not args.no_host_path:
        host = host_contigs(ds)

    # ---- PCIe-inclusive rate of the drop-in host entry point (never `value`)
    host_path = None
    if world == 1 and not args.no_host_path and not args.trlr and thr == 0.0:
        L = _lib.load()

        def host_calls(policy, idle_s=20.0):
            L.ks_set_host_cache(policy)
            L.ks_set_host_cache_idle(idle_s)
            try:
                t0 = time.perf_counter()
                api.kmer_regions(host, k, w, args.min_width, args.min_score)  # first call (contexts, pinned staging)
                first = time.perf_counter() - t0
                th = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    hr = api.kmer_regions(host, k, w, args.min_width, args.min_score)
                    th.append(time.perf_counter() - t0)
            finally:
                L.ks_set_host_cache(2)
                L.ks_set_host_cache_idle(20.0)
            t_host = float(np.median(th))
            out = {"seconds": round(t_host, 4), "Gbases_per_s": round(n_bases / t_host / 1e9, 3),
                   "all_seconds": [round(x, 4) for x in th], "first_call_seconds": round(first, 4),
                   "spread": round(max(th) / min(th), 3),
                   "regions_equal": bool(np.array_equal(hr["pos"], pos)),
                   "scores_equal": bool(np.array_equal(hr["score"].view(np.uint64), score.view(np.uint64))),
                   "visits_equal": (bool(np.array_equal(hr["counts"], vis_host)) if vis_host is not None
                                    else None)}
            return out
        L.ks_release_cache()
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info(dev)[0]
        # the default policy (2): memory kept while calls come, returned after
        # the idle time (1 s here, 20 s by default)
        host_path = host_calls(2, idle_s=1.0)
        time.sleep(2.5)
        host_path["vram_returned_after_idle"] = bool(torch.cuda.mem_get_info(dev)[0] >= free0 - (64 << 20))
        host_path["note"] = ("ks_kmer_regions from host memory with the visit histogram (median of 3 after a first "
                             "call), default memory policy ks_set_host_cache(2): the call's workspace and table "
                             "buffer stay while calls keep coming and return to the driver once the context has "
                             "been idle (20 s by default, 1 s here; vram_returned_after_idle); the score table and "
                             "the bases (2-bit codes + N runs) cross PCIe through pinned buffers, table "
                             "compress/expand, k-mer count in pieces during staging, scan, visits D2H; "
                             "visits_equal against the device-resident visits line")
        host_path["return_at_end"] = host_calls(0)
        host_path["return_at_end"]["vram_returned"] = bool(torch.cuda.mem_get_info(dev)[0] >= free0 - (64 << 20))
        host_path["return_at_end"]["note"] = ("ks_set_host_cache(0): every call allocates its workspace and table "
                                              "buffer again (fresh VRAM, cleared by the driver) and returns them")

    # ---- the drop-in host entry spread over a device list (ks_set_devices;
    # default [0, 0]: two contexts on the one GPU), PCIe-inclusive, checked
    # against the device-resident line; the host-side visit sum and each
    # part's table upload reported (ks_multi_last_stats)
    if (world == 1 and not dist and args.multi_devices and not args.no_host_path and not args.trlr
            and thr == 0.0):
        L = _lib.load()
        L.ks_release_cache()
        extra["host_multi"] = host_multi_line(args, L, host, k, w, pos, score, vis_host, n_bases)

    # ---- CPU baseline (N=1, one pinned core, bounded sample) and the parity
    # verdict (every contig of this rank, oracle on a host thread pool)
    cpu = None
    parity = None
    table_equal_host = None
    if not args.no_cpu:
        if world == 1:  # the device-built table against the host builder (bitwise)
            hc = counts.cpu().numpy()
            wh = np.asarray(api.log2_table(hc, k) if args.score == "log2" else
                            api.pm1_table(hc, k) if args.score == "pm1" else
                            api.rank_table(hc, k, words), dtype=np.float64)
            table_equal_host = bool(np.array_equal(w.view(np.uint64), wh.view(np.uint64)))
            del hc, wh
        orc = Oracle(host, k, (w - thr) if args.trlr else w, thr, args.min_width, args.min_score, args.trlr,
                     args.cpu_threads)
        if rank == 0 and world == 1:
            ids, acc = sample_ids(ds.offsets, args.cpu_sample)
            t_cpu = orc.baseline(ids)
            lens = np.diff(ds.offsets)
            cpu = {"value": round(acc / t_cpu / 1e9, 5), "unit": "Gbases/s", "cores": 1, "kind": "port",
                   "sample": f"oracle/ks_oracle.c scan of {len(ids)} contigs ({acc} bp: the largest, "
                             f"{int(lens.max())} bp, plus the smallest) of the same genome, same table, "
                             f"one thread pinned to one core",
                   "seconds": round(t_cpu, 3), "host_cpu": cpu_model(), "host_nproc": os.cpu_count()}
        check = list(range(ds.nseq)) if args.parity == "all" else sorted(orc.per) if args.parity == "sample" else []
        if check:
            t0 = time.perf_counter()
            orc.fill(check)
            ok = orc.parity(pos, score, check)
            bp = int(sum(int(host[q].size) for q in check))
            extra["parity_seconds"] = round(time.perf_counter() - t0, 2)
            extra["parity_threads"] = orc.threads
            parity = bool(reduce_over_ranks(1.0 if ok else 0.0, tdist.ReduceOp.MIN if dist else None) > 0.5)
            extra["parity_bp"] = int(reduce_over_ranks(float(bp), tdist.ReduceOp.SUM if dist else None))
            extra["parity_contigs"] = "all" if args.parity == "all" else check
            if vis_host is not None and args.parity == "all":
                # the visit histogram kmer_regions_r returns (kmer_spans.c:266-267, 523-537) over the
                # whole genome: the oracle's per-contig histograms summed vs the visits line's
                t0 = time.perf_counter()
                ov = orc.visits_sum(check)
                extra["visits_parity"] = bool(np.array_equal(ov, vis_host.view(np.uint32)))
                extra["visits_parity_bp"] = bp
                extra["visits_parity_seconds"] = round(time.perf_counter() - t0, 2)
                del ov
        del orc

    # ---- weighted rank (BASELINE config 3) on the same genome and counts
    rank_line = None
    if (world == 1 and not args.no_rank and args.score == "log2" and not args.trlr and args.mode == "shard"
            and args.shard_of <= 1):
        table.close()
        rank_line = rank_subline(args, ctx, ds, counts, words, make_table, timed_steps, host, D)

    step_ms = ms_step
    e2e_ms = setup["count_ms"] + setup["table_device"] + step_ms
    line = {
        "metric": METRIC,
        "value": round(value, 4), "unit": "Gbases/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
        "scaling": "strong" if args.mode == "shard" else "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": f"human-shaped synthetic genome ({total_bases} bp, "
                               f"{args.ncontigs} contigs, scale {args.scale}), k={k}, {args.score} score from its "
                               f"own counts, min_width {args.min_width}, min_score {args.min_score}, device-resident"
                               + (", contigs (cut inside N gaps) LPT-sharded over the ranks" if args.mode == "shard" else
                                  ", one genome per rank"),
                   "k": k, "score": args.score, "genome_bp": total_bases,
                   "parallelism": f"{'contig-shard' if args.mode == 'shard' else 'genome-per-rank'} x{world}",
                   "mode": args.mode, "scan": "tr_lr_regions" if args.trlr else "kmer_regions",
                   "scan_algo": int(stats[-1]["scan_algo"]), **table_shape, "build_id": build_id},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "parity_sample": parity,
        "table_equal_host": table_equal_host,
        "regions": n_regions_all,
        "replayed_chunks": int(stats[-1]["n_replay"]),
        "visits_path": visits_line,
        "host_path": host_path,
        "phase_ms": phase_means(stats),
        "setup_ms": setup,
        "end_to_end": {"ms": round(e2e_ms, 2), "Gbases_per_s": round(n_bases / (e2e_ms * 1e-3) / 1e9, 3),
                       "what": "count + device score table from the counts (values, codes, 12-bit codes, "
                               "expanded table) + one scan step, per rank"},
        "configs": {"rank": rank_line} if rank_line is not None else None,
    }
    line.update(extra)
    if rank == 0:
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(s + "\n")
    if dist:
        tdist.destroy_process_group()


def multi_devices(args):
    return [int(x) for x in args.multi_devices.split(",") if x.strip() != ""]


def host_multi_line(args, L, host, k, w, pos, score, vis_host, n_bases):
    """kmer_regions_r from host memory over a device list (csrc/ks_multi.cpp:
    the library's shard plan, one context + host thread per entry, visit
    histograms summed on the host, regions merged): median of 3 after a first
    call, phases from ks_multi_last_stats, outputs vs the device-resident line."""
    import ctypes as C
    from kmer_spans_amd import _lib, api
    devs = multi_devices(args)
    arr = (C.c_int32 * len(devs))(*devs)
    _lib.check(L.ks_set_devices(arr, len(devs)))
    try:
        t0 = time.perf_counter()
        api.kmer_regions(host, k, w, args.min_width, args.min_score)
        first = time.perf_counter() - t0
        ts, st = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            hr = api.kmer_regions(host, k, w, args.min_width, args.min_score)
            ts.append(time.perf_counter() - t0)
            st.append(_lib.multi_last_stats())
    finally:
        _lib.check(L.ks_set_devices(None, 0))
        L.ks_release_cache()
    i = int(np.argsort(ts)[len(ts) // 2])
    t = ts[i]
    return {"devices": devs, "seconds": round(t, 4), "Gbases_per_s": round(n_bases / t / 1e9, 3),
            "all_seconds": [round(x, 4) for x in ts], "first_call_seconds": round(first, 4),
            "phases_ms": {key: (round(v, 2) if not isinstance(v, list) else
                                [{a: round(b, 2) for a, b in d.items()} for d in v]) for key, v in st[i].items()},
            "regions_equal": bool(np.array_equal(hr["pos"], pos)),
            "scores_equal": bool(np.array_equal(hr["score"].view(np.uint64), score.view(np.uint64))),
            "visits_equal": (bool(np.array_equal(hr["counts"], vis_host)) if vis_host is not None else None),
            "note": "ks_kmer_regions (NULL context) over the device list, PCIe-inclusive, median of 3: the library's "
                    "shard plan, one context + host thread per entry (each uploads the score table itself), the "
                    "visit histograms summed on the host (host_sum_ms), regions merged (merge_ms); per part: "
                    "body, staging + count, table upload + compression, scan"}


def rank_subline(args, ctx, ds, counts, words, make_table, timed_steps, host, D):
    """BASELINE config 3 (kmer_low_comp_regions, kmer_spans.c:548-621): the
    weighted-rank table (threshold 0.75) of the same genome's counts, scanned
    like the metric line; parity over every contig; the CPU phases of the
    reference operation (count, rank, scan) on one pinned core."""
    k = args.k
    w_dev, thr, table, init, tt = make_table(counts, words, "rank", warm=True)
    pos, score, stats, elapsed = timed_steps(ds, table, init, args.rank_steps, 1)
    n_bases = int(stats[-1]["n_bases"])
    ms = elapsed / args.rank_steps * 1e3
    out = {"what": "weighted rank (kmer_low_comp_regions, thr 0.75), k=13, same genome and counts",
           "value": round(n_bases / (ms * 1e-3) / 1e9, 4), "unit": "Gbases/s", "ms_per_step": round(ms, 3),
           "steps": args.rank_steps, "regions": int(pos.shape[1]), "replayed_chunks": int(stats[-1]["n_replay"]),
           "phase_ms": phase_means(stats), "table_ms": round(tt["table_device"], 2),
           "table_setup_ms": {key: round(v, 2) for key, v in tt.items()},
           "positions_per_read": table.positions_per_read, "parity": None}
    out["end_to_end"] = {"ms": round(float(tt["table_device"]) + ms, 2),
                         "what": "device rank table + one step (the count is shared with the metric line)"}
    table.close()
    if args.no_cpu or host is None:
        return out
    from oracle import oracle as O
    w = w_dev.cpu().numpy()
    hc = counts.cpu().numpy()
    old = os.sched_getaffinity(0)
    os.sched_setaffinity(0, {min(old)})
    try:  # the reference's rank build (glibc merge sort + sequential prefix), one core
        t0 = time.perf_counter()
        wo = O.rank_table(hc, k, words)
        t_rank = time.perf_counter() - t0
    finally:
        os.sched_setaffinity(0, old)
    out["table_equal_oracle"] = bool(np.array_equal(w.view(np.uint64), wo.view(np.uint64)))
    del wo
    orc = Oracle(host, k, w, thr, args.min_width, args.min_score, False, args.cpu_threads)
    ids, acc = sample_ids(ds.offsets, args.cpu_sample)
    old = os.sched_getaffinity(0)
    os.sched_setaffinity(0, {min(old)})
    try:
        t0 = time.perf_counter()
        O.kmer_counts([host[q] for q in ids], k)
        t_count = time.perf_counter() - t0
    finally:
        os.sched_setaffinity(0, old)
    t_scan = orc.baseline(ids)
    total = float(ds.total)
    out["cpu_baseline"] = {
        "kind": "port", "cores": 1, "unit": "Gbases/s",
        "value": round(total / (t_count * total / acc + t_rank + t_scan * total / acc) / 1e9, 5),
        "scan_value": round(acc / t_scan / 1e9, 5),
        "phases_s": {"count_sample": round(t_count, 3), "rank_table_full": round(t_rank, 3),
                     "scan_sample": round(t_scan, 3)},
        "sample": f"count and scan of {len(ids)} contigs ({acc} bp), extrapolated to {int(total)} bp; the rank "
                  f"table (4^{k} entries) built once in full; oracle/ks_oracle.c, one pinned core"}
    t0 = time.perf_counter()
    orc.fill(range(ds.nseq))
    out["parity"] = orc.parity(pos, score, range(ds.nseq))
    out["parity_bp"] = int(ds.total)
    out["parity_seconds"] = round(time.perf_counter() - t0, 2)
    if not args.no_host_path:
        out["host_low_comp"] = hl = host_low_comp_line(args, host, hc, w, pos, score, int(ds.total), n_bases)
        hl["parity"] = bool(hl["parity"] and out["parity"] and out["table_equal_oracle"] and hl["n"][0] == words)
        if multi_devices(args):
            import ctypes as C
            from kmer_spans_amd import _lib
            L = _lib.load()
            devs = multi_devices(args)
            L.ks_release_cache()
            _lib.check(L.ks_set_devices((C.c_int32 * len(devs))(*devs), len(devs)))
            try:
                hm = host_low_comp_line(args, host, hc, w, pos, score, int(ds.total), n_bases)
                hm["phases_ms"] = {key: (round(v, 2) if not isinstance(v, list) else v)
                                   for key, v in _lib.multi_last_stats().items() if key != "parts"}
            finally:
                _lib.check(L.ks_set_devices(None, 0))
                L.ks_release_cache()
            hm["devices"] = devs
            hm["parity"] = bool(hm["parity"] and out["parity"] and out["table_equal_oracle"] and hm["n"][0] == words)
            hm["note"] = ("ks_low_comp_regions (NULL context) over the device list: the library's shard plan; each "
                          "part stages + counts its pieces, the count histogram summed on the host in stripes "
                          "(host_sum_ms), each part builds the rank table from the sum and scans; median of 3 "
                          "(phases of the last call)")
            hl["multi"] = hm
    return out


def host_low_comp_line(args, host, counts_host, w_rank, pos, score, total, n_bases):
    """BASELINE config 3 as the R user calls it: kmer_low_comp_regions
    (kmer_spans.c:548-621, kmer_spans.R:72-79) from host memory -- the bases
    cross PCIe, counted in pieces meanwhile, the rank table built on the
    device, counts + w.rank returned over PCIe while the scan runs -- timed
    (median of 3, PCIe-inclusive, default memory policy), its outputs checked
    against the device-resident rank line (regions, scores), the device counts
    and the device rank table (itself equal to the oracle's, table_equal_oracle)."""
    from kmer_spans_amd import api
    k = args.k
    api.kmer_low_comp_regions(host, k, args.min_width, args.min_score, 0.75)  # warm (pinned buffers)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        r = api.kmer_low_comp_regions(host, k, args.min_width, args.min_score, 0.75)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    out = {"seconds": round(t, 4), "Gbases_per_s": round(n_bases / t / 1e9, 3),
           "all_seconds": [round(x, 4) for x in ts],
           "counts_equal": bool(np.array_equal(r["counts"], counts_host)),
           "w_rank_equal": bool(np.array_equal(r["w_rank"].view(np.uint64), w_rank.view(np.uint64))),
           "regions_equal": bool(np.array_equal(r["pos"].T, pos)),
           "scores_equal": bool(np.array_equal(np.ascontiguousarray(r["score"].T).view(np.uint64),
                                               np.ascontiguousarray(score).view(np.uint64))),
           "n": [float(x) for x in r["n"]],
           "note": f"ks_low_comp_regions from host memory, k={k}, thr 0.75, {total} bp (median of 3, PCIe-inclusive, "
                   "default memory policy); parity = counts, w.rank, regions and scores equal to the device-resident "
                   "rank line, whose table equals the oracle's (table_equal_oracle) and whose regions equal the "
                   "oracle's (parity)"}
    out["parity"] = out["counts_equal"] and out["w_rank_equal"] and out["regions_equal"] and out["scores_equal"]
    return out


def genome_cpu_baseline(args, ds, host, counts, words, orc, n_genomes):
    """one genome end to end on one pinned
    core (the reference's kmer.counts, the log2 table of its counts, and
    kmer_regions), timed on a sample of contigs for the count and the scan and
    extrapolated to the whole genome; the 256-genome job time is that times
    256, stated as an extrapolation."""
    from oracle import oracle as O
    k = args.k
    ids, acc = sample_ids(ds.offsets, args.cpu_sample)
    old = os.sched_getaffinity(0)
    os.sched_setaffinity(0, {min(old)})
    try:
        t0 = time.perf_counter()
        O.kmer_counts([host[q] for q in ids], k)
        t_count = time.perf_counter() - t0
        hc = counts.cpu().numpy()
        t0 = time.perf_counter()
        O.log2_table(hc, k)
        t_table = time.perf_counter() - t0
    finally:
        os.sched_setaffinity(0, old)
    t_scan = orc.baseline(ids)
    total = float(ds.total)
    t_genome = (t_count + t_scan) * total / acc + t_table
    return {"kind": "port", "cores": 1, "unit": "Gbases/s", "value": round(total / t_genome / 1e9, 5),
            "seconds_per_genome": round(t_genome, 2), "genomes": 256,
            "job_seconds_extrapolated": round(t_genome * 256, 1),
            "phases_s": {"count_sample": round(t_count, 3), "log2_table_full": round(t_table, 3),
                         "scan_sample": round(t_scan, 3)},
            "sample": f"count and scan of {len(ids)} contigs ({acc} bp) of one genome, extrapolated to its "
                      f"{int(total)} bp, plus the log2 table (4^{k} entries) in full; the 256-genome job time "
                      f"is that x 256 (an extrapolation); oracle/ks_oracle.c, one pinned core "
                      f"(this run: {n_genomes} genome(s))"}


def reduce_parity(ok, dist, tdist):
    """True iff every rank's parity verdict is true (gloo/nccl MIN)."""
    if not dist:
        return ok
    t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64,
                     device=torch.device("cuda", torch.cuda.current_device()) if tdist.get_backend() == "nccl" else "cpu")
    tdist.all_reduce(t, op=tdist.ReduceOp.MIN)
    return float(t.item()) > 0.5


def run_genomes(args, ctx, ds0, dev, rank, world, dist, tdist, barrier, max_over_ranks, make_table, D, genome,
                build_id):
    """Config 5: G genomes per rank, each end to end (count -> table ->
    scan) inside the timed region; genome generation is not timed (it stands
    in for reading the genome).  Records gathered to rank 0 after timing."""
    k = args.k
    G = max(1, args.genomes_per_rank)
    seeds = [args.seed + 1000 * (rank * G + g) for g in range(G)]
    dss = [ds0]
    for s_ in seeds[1:]:
        parts, lens = genome.human_like(scale=args.scale, seed=s_, device=dev, ncontigs=args.ncontigs)
        dss.append(D.from_parts(parts, lens, dev))
        del parts
    counts = torch.zeros(4 ** k, dtype=torch.int32, device=dev)

    def one(ds):
        counts.zero_()
        words = D.count(ctx, ds, k, counts)
        if args.trlr:  # (tr_lr needs the weights for its init table)
            _, _, table, init, _ = make_table(counts, words, args.score,
                                              ext_gib=args.ext_max_gib if args.ext_max_gib else 32.0, warm=False)
        else:  # the table alone: the weights of the parity leg are rebuilt after timing
            init = None
            table = D.DeviceTable.from_counts(ctx, counts, k, args.score, total=words,
                                              thr=0.75 if args.score == "rank" else 0.0, expand=not args.no_expand,
                                              max_ext_bytes=int((args.ext_max_gib or 32.0) * (1 << 30)))
        if args.trlr:
            out = D.tr_lr(ctx, ds, k, table, init, args.min_width)
        else:
            out = D.scan(ctx, ds, k, table, args.min_width, args.min_score)
        table.close()
        if init is not None:
            init.close()
        return out

    # pipelined (default, not with tr_lr): genome g + 1's count and score table
    # on a second context and stream from a host thread while genome g is
    # scanned -- independent work (the count is LDS-atomic bound, the table
    # build write bound, the scan request bound)
    pipelined = not args.trlr and not args.genomes_serial
    if pipelined:
        from kmer_spans_amd import _lib as L_
        import threading
        # its own context (workspace, streams): _lib.context(dev) is the cached
        # per-device context that ctx already is
        ctx2 = L_.Context(torch.cuda.current_device())
        s_b = torch.cuda.Stream(priority=args.count_priority) if args.count_priority is not None else torch.cuda.Stream()
        ctx2.set_stream(s_b.cuda_stream)
        counts2 = [torch.zeros(4 ** k, dtype=torch.int32, device=dev) for _ in range(2)]
        cap = int((args.ext_max_gib if args.ext_max_gib else 32.0) * (1 << 30))
        thr_g = 0.75 if args.score == "rank" else 0.0

        def count_table(ds, cbuf):
            with torch.cuda.stream(s_b):
                cbuf.zero_()
                words = D.count(ctx2, ds, k, cbuf)
                tab_ = D.DeviceTable.from_counts(ctx2, cbuf, k, args.score, total=words, thr=thr_g,
                                                 expand=not args.no_expand, max_ext_bytes=cap)
                s_b.synchronize()  # complete before ctx's stream scans with it
                return tab_

        def run_all():
            out = [None] * G
            tab = count_table(dss[0], counts2[0])
            for g in range(G):
                nxt = {}
                th = None
                if g + 1 < G:
                    th = threading.Thread(target=lambda g=g: nxt.setdefault("t", count_table(dss[g + 1],
                                                                                             counts2[(g + 1) % 2])))
                    th.start()
                out[g] = D.scan(ctx, dss[g], k, tab, args.min_width, args.min_score)
                tab.close()
                if th is not None:
                    th.join()
                    tab = nxt["t"]
            return out
        run_all()  # warm-up (both contexts' workspace, pinned staging)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        results = run_all()
        torch.cuda.synchronize()
        barrier()
        elapsed = max_over_ranks(time.perf_counter() - t0)
        del counts2
        ctx2.close()
    else:
        one(dss[0])  # warm-up (workspace, pinned staging)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        results = [one(ds) for ds in dss]
        torch.cuda.synchronize()
        barrier()
        elapsed = max_over_ranks(time.perf_counter() - t0)
    bases = sum(int(r[2]["n_bases"]) for r in results) * world
    n_regions = sum(int(r[0].shape[1]) for r in results)
    # parity of every genome of this rank after timing (each genome's own
    # table, rebuilt: the timed loop closed it), the oracle on a thread pool
    parity = None
    cpu = None
    if not args.no_cpu and args.parity != "none":
        ok = True
        first = True
        for ds, r in zip(dss, results):
            counts.zero_()
            words = D.count(ctx, ds, k, counts)
            w_dev, thr, table, init, _ = make_table(counts, words, args.score, ext_gib=1.0, warm=False)
            table.close()
            if init is not None:
                init.close()
            host = host_contigs(ds)
            orc = Oracle(host, k, (w_dev.cpu().numpy() - thr) if args.trlr else w_dev.cpu().numpy(), thr,
                         args.min_width, args.min_score, args.trlr, args.cpu_threads)
            if first and rank == 0 and not args.trlr:
                cpu = genome_cpu_baseline(args, ds, host, counts, words, orc, G * world)
            first = False
            orc.fill(range(ds.nseq))
            ok &= orc.parity(r[0], r[1], range(ds.nseq))
        parity = bool(reduce_parity(ok, dist, tdist))
    if dist:
        from kmer_spans_amd.dist import gather_regions
        pos = np.concatenate([r[0] for r in results], axis=1)
        sc = np.concatenate([r[1] for r in results], axis=1)
        allpos, _ = gather_regions(pos, sc, dev)
        if rank == 0:
            n_regions = sum(int(p.shape[1]) for p in allpos)
    line = {"metric": METRIC + " [config 5: genomes per rank, end to end]",
            "value": round(bases / elapsed / 1e9, 4), "unit": "Gbases/s", "n_gpus": world, "steps": G,
            "warmup": 1, "ms_per_step": round(elapsed / G * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"{G * world} human-shaped genomes (scale {args.scale}), {G} per rank, k={k}, "
                                   f"{args.score}, each: count + table + expanded table + scan",
                       "k": k, "score": args.score, "genomes": G * world, "mode": "genomes",
                       "parallelism": f"genome-per-rank x{world}", "build_id": build_id},
            "regions": n_regions, "parity_sample": parity, "parity_genomes": G * world if parity is not None else 0}
    if cpu is not None:
        line["cpu_baseline"] = cpu
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
