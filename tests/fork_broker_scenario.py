"""The reference's own mclapply pattern through the fork broker (test.R:351
calls kmer.counts in the R session, then :554-565 calls kmer.counts and
window.kmer.dist inside mclapply workers).  Run as its own process by
tests/test_fork.py (the broker must be forked by a process that has not
touched HIP yet): the parent calls, forks workers that call the host entry
points, and prints one JSON line comparing every worker result with the
parent's own call.

  python tests/fork_broker_scenario.py gpu|cpu
"""
import json
import os
import sys

os.environ["KS_FORK_BROKER"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from kmer_spans_amd import api  # noqa: E402
from kmer_spans_amd._lib import KmerSpansError  # noqa: E402


def genome(seed, n=3, length=30_000):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        s = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=length)
        s[rng.integers(0, length, size=length // 200)] = ord("N")
        rep = np.frombuffer(b"CA" * 400, dtype=np.uint8)
        at = int(rng.integers(0, length - rep.size))
        s[at:at + rep.size] = rep
        out.append(s.tobytes().decode())
    return out


def work(seqs):
    """The calls a worker makes; results as plain lists (JSON)."""
    k = 6
    c = api.kmer_counts(seqs, k, with_f=False)
    w = np.log2(np.maximum(c["counts"], 1) / max(np.median(c["counts"]), 1.0))
    r = api.kmer_regions(seqs, k, w, 20, 5.0, visits=True)
    lc = api.kmer_low_comp_regions(seqs, k, 20, 2.0, 0.75)
    wd = api.window_kmer_dist(seqs, ["CACACA", "ACGTAC"], 60, freq=False, ret_flag=1)
    kms = api.kmer_seq(3)
    tr = api.lr_regions(seqs, (3, 10), kms, np.linspace(-1, 1, 64), np.linspace(1, -1, 64))
    return {
        "counts": c["counts"].tolist(), "n": c["n"]["n"],
        "reg_pos": r["pos"].tolist(), "reg_score": r["score"].tolist(), "visits": r["counts"].tolist(),
        "lc_pos": lc["pos"].tolist(), "lc_rank": lc["w_rank"].tolist(), "lc_n": lc["n"].tolist(),
        "wd": wd["dist"].tolist(), "wd_inc": wd["seq_i"].tolist(),
        "wd_scores": [s.tolist() if s is not None else None for s in wd["scores"]],
        "tr_pos": tr["pos"].tolist(), "tr_spectra": tr["kmer_scores"].tolist(),
    }


def in_child(fn):
    """fn() in a forked child; returns its JSON result (or the error text)."""
    r, wfd = os.pipe()
    pid = os.fork()
    if pid == 0:
        code = 0
        try:
            try:
                out = {"ok": fn()}
            except KmerSpansError as e:
                out = {"err": str(e)}
            data = json.dumps(out).encode()
            while data:
                data = data[os.write(wfd, data):]
        except BaseException:  # noqa: BLE001 -- never return into the parent's code
            code = 3
        os._exit(code)
    os.close(wfd)
    chunks = []
    while True:
        b = os.read(r, 1 << 20)
        if not b:
            break
        chunks.append(b)
    os.close(r)
    _, st = os.waitpid(pid, 0)
    assert os.WEXITSTATUS(st) == 0, st
    return json.loads(b"".join(chunks))


def main(mode):
    res = {"mode": mode}
    seqs = [genome(i) for i in range(3)]
    if mode == "gpu":
        parent = work(seqs[0])  # the parent uses the GPU first (test.R:351)
        kids = [in_child(lambda s=s: work(s)) for s in seqs]
        direct = [parent] + [work(s) for s in seqs[1:]]  # the parent's own results for the workers' inputs
        res["workers_ok"] = all("ok" in x for x in kids)
        res["workers_equal"] = res["workers_ok"] and all(x["ok"] == d for x, d in zip(kids, direct))
        res["regions"] = [len(d["reg_pos"][0]) for d in direct]
    else:
        try:
            api.kmer_counts(seqs[0], 6)
            res["parent"] = "ran"
        except KmerSpansError as e:
            res["parent"] = str(e)
        kid = in_child(lambda: api.kmer_counts(seqs[1], 6)["n"])
        res["worker_err"] = kid.get("err")
        bad = in_child(lambda: api.kmer_counts(seqs[1], 99)["n"])
        res["worker_arg_err"] = bad.get("err")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpu")
