"""Ingest measurement: FASTA file -> HBM records, and
batched multi-k counting, on the human-shaped genome of bench.py.

  python tools/ingest_bench.py [--scale 1.0] [--ks 7,11,13] [--out f.json]

Writes the genome as a 60-column FASTA file (soft-masked stretches in lower
case) under $TMPDIR, then times ks_fasta_load (host read + H2D overlapped,
device parse), the batched counter against one ks_count_dev per k, and the
oracle's single-thread FASTA parse on one contig as the CPU baseline.  The
device parse of the first contig is checked against the oracle.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kmer_spans_amd import _lib, device as D, genome  # noqa: E402


def fasta_text(parts, width=60) -> torch.Tensor:
    """Device-built FASTA text of the contigs (uint8 tensor)."""
    pieces = []
    for i, p in enumerate(parts):
        hdr = torch.tensor(list(f">chr{i + 1} synthetic\n".encode()), dtype=torch.uint8, device=p.device)
        L = p.numel()
        s = p.clone()
        # soft-mask alternate 5 kb stretches (lower case), as in UCSC/Ensembl files
        pos = torch.arange(L, device=p.device)
        low = ((pos // 5000) % 2 == 1) & (s != ord("N"))
        s[low] += 32
        del pos, low
        full = L // width
        body = torch.empty((full, width + 1), dtype=torch.uint8, device=p.device)
        body[:, :width] = s[:full * width].view(full, width)
        body[:, width] = ord("\n")
        pieces += [hdr, body.view(-1)]
        if L % width:
            pieces += [s[full * width:], torch.tensor([ord("\n")], dtype=torch.uint8, device=p.device)]
    return torch.cat(pieces)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--ks", default="7,11,13")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    ks = [int(x) for x in args.ks.split(",")]
    ctx = _lib.context(0)
    D.bind_torch_stream(ctx)
    t = time.time()
    parts, lens = genome.human_like(args.scale, seed=1, device="cuda")
    text = fasta_text(parts)
    nbytes = text.numel()
    path = os.path.join(os.environ.get("TMPDIR", tempfile.gettempdir()), f"ks_ingest_{os.getpid()}.fa")
    text.cpu().numpy().tofile(path)
    del text
    t_gen = time.time() - t
    print(f"genome + FASTA ({nbytes / 1e9:.3f} GB) written in {t_gen:.1f}s", flush=True)
    res = {"metric": "FASTA ingest GB/s (file -> device records)", "file_bytes": nbytes,
           "genome_bp": int(sum(lens)), "scale": args.scale}
    try:
        loads = []
        for r in range(args.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fa = D.load_fasta(ctx, path, 0)
            wall = (time.perf_counter() - t) * 1e3
            loads.append({"wall_ms": wall, "upload_ms": fa.ms_upload, "parse_ms": fa.ms_parse})
            print(f"load {r}: wall {wall:.1f} ms upload {fa.ms_upload:.1f} parse {fa.ms_parse:.1f}", flush=True)
            if r < args.reps - 1:
                fa.close()
        assert fa.nseq == len(parts) and fa.total == sum(lens), (fa.nseq, fa.total)
        best = min(loads, key=lambda x: x["wall_ms"])
        res.update({"loads": loads, "value": nbytes / best["wall_ms"] / 1e6, "unit": "GB/s",
                    "parse_GBps": nbytes / best["parse_ms"] / 1e6})
        # parity: the first contig's bytes equal the upper-cased contig
        a, b = int(fa.offsets[0]), int(fa.offsets[1])
        want = parts[0].clone()
        assert torch.equal(D_slice(fa, a, b), want)
        res["parity_first_contig"] = True
        # batched counting vs one pass per k
        counts = [torch.zeros(4 ** k, dtype=torch.int32, device="cuda") for k in ks]
        D.count_multi(ctx, fa, ks, counts)
        torch.cuda.synchronize()
        tm = []
        for _ in range(args.reps):
            for c in counts:
                c.zero_()
            torch.cuda.synchronize()
            t = time.perf_counter()
            words = D.count_multi(ctx, fa, ks, counts)
            torch.cuda.synchronize()
            tm.append((time.perf_counter() - t) * 1e3)
        single = []
        ref = [c.clone() for c in counts]
        for _ in range(args.reps):
            tot = 0.0
            for k, c in zip(ks, counts):
                c.zero_()
                torch.cuda.synchronize()
                t = time.perf_counter()
                D.count(ctx, fa, k, c)
                torch.cuda.synchronize()
                tot += (time.perf_counter() - t) * 1e3
            single.append(tot)
        for c, r0 in zip(counts, ref):
            assert torch.equal(c, r0)
        res["count_multi"] = {"ks": ks, "words": words, "batched_ms": min(tm), "separate_ms": min(single),
                              "batched_Gbases_s": sum(lens) / min(tm) / 1e6}
        fa.close()
        # CPU baseline: the oracle's single-thread parse of the last contig's text
        from oracle import oracle as O
        data = open(path, "rb").read()
        cut = data.rfind(b">")
        sample = data[cut:]
        t = time.perf_counter()
        o = O.fasta_parse(sample)
        cpu_s = time.perf_counter() - t
        res["cpu_baseline"] = {"value": len(sample) / cpu_s / 1e9, "unit": "GB/s", "cores": 1, "kind": "port",
                               "sample": f"oracle orc_fasta_parse of the last contig's FASTA ({len(sample)} bytes)",
                               "seconds": cpu_s}
        fa2 = D.parse_fasta(ctx, sample)
        assert fa2.host_seqs() == o["seqs"] and fa2.names == o["names"]
        fa2.close()
        res["parity_cpu_sample"] = True
    finally:
        os.unlink(path)
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


def D_slice(fa, a, b) -> torch.Tensor:
    """Device bytes [a, b) of a FastaSeqs as a torch tensor (via host)."""
    return torch.from_numpy(np.frombuffer(fa.host_bytes()[a:b], dtype=np.uint8).copy()).cuda()


if __name__ == "__main__":
    main()
