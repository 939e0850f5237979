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


def start_child(fn):
    """fn() in a forked child started now; returns a function that waits for
    it and returns its JSON result (several children run at once)."""
    r, wfd = os.pipe()
    pid = os.fork()
    if pid == 0:
        os.close(r)
        code = 0
        try:
            try:
                out = {"ok": fn()}
            except KmerSpansError as e:
                out = {"err": str(e)}
            data = json.dumps(out).encode()
            while data:
                data = data[os.write(wfd, data):]
        except BaseException:  # noqa: BLE001
            code = 3
        os._exit(code)
    os.close(wfd)

    def wait():
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
    return wait


def file_work(tmp, seqs):
    """kmers.to.file with RELATIVE paths after a chdir (the broker resolves
    them in the worker's directory), read back."""
    os.chdir(tmp)
    with open("g.fa", "w") as f:
        for i, s in enumerate(seqs):
            f.write(f">s{i}\n{s}\n")
    info = api.kmers_to_file("g.fa", "rel_", [3, 5], min_l=10)
    rk = api.read_kmers(os.path.join(tmp, os.path.basename(info[1]))) if info[1] else False
    return {"out": os.path.basename(info[1]) if info[1] else None, "in_tmp": bool(info[1]) and
            os.path.exists(os.path.join(tmp, os.path.basename(info[1]))),
            "counts": [c.tolist() for c in rk["counts"]] if rk is not False else None}


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
        # mclapply(mc.cores = 20) shape: several workers at once (the broker
        # serves them on its server threads)
        waits = [start_child(lambda s=s: work(s)) for s in seqs * 2]
        conc = [w() for w in waits]
        res["concurrent_ok"] = all("ok" in x for x in conc)
        res["concurrent_equal"] = res["concurrent_ok"] and all(x["ok"] == d for x, d in zip(conc, direct * 2))
        import tempfile
        with tempfile.TemporaryDirectory() as tmp:
            fk = in_child(lambda: file_work(tmp, seqs[1]))
            own = [api.kmer_counts(seqs[1], kk, with_f=False)["counts"].tolist() for kk in (3, 5)]
            res["file_ok"] = "ok" in fk and fk["ok"]["in_tmp"] and fk["ok"]["counts"] == own
            if not res["file_ok"]:
                res["file_detail"] = fk.get("err") or {kk: v for kk, v in fk["ok"].items() if kk != "counts"}
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
        # a process outside the owner's tree (double fork: reparented away)
        # is refused by the broker's peer check
        import time
        r, wfd = os.pipe()
        pid = os.fork()
        if pid == 0:
            if os.fork() == 0:
                os.close(r)
                time.sleep(0.5)  # its parent has exited by now
                try:
                    api.kmer_counts(seqs[1], 6)
                    msg = "ran"
                except KmerSpansError as e:
                    msg = str(e)
                except BaseException as e:  # noqa: BLE001
                    msg = "other: " + repr(e)
                os.write(wfd, msg.encode())
                os._exit(0)
            os._exit(0)
        os.waitpid(pid, 0)
        os.close(wfd)
        res["stranger_err"] = os.read(r, 4096).decode()
        os.close(r)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpu")
