"""Fork safety of the C ABI: R's mclapply forks workers after the
parent may have used the library (test.R:351 then :554-559).  A child that
inherits a HIP context must get a clear KS_ERR_DEVICE status, never a hang or
a fault: nothing in the child may touch the parent's HIP state."""
import json
import os
import subprocess
import sys

import pytest

SCENARIO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fork_broker_scenario.py")


def _child_status(call):
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:  # child: report (status, message) through the pipe, never return to pytest
        code = 99
        try:
            rc, msg = call()
            os.write(w, f"{rc}|{msg}".encode())
            code = 0
        finally:
            os._exit(code)
    os.close(w)
    _, st = os.waitpid(pid, 0)
    data = os.read(r, 4096).decode()
    os.close(r)
    assert os.WEXITSTATUS(st) == 0
    rc, msg = data.split("|", 1)
    return int(rc), msg


@pytest.mark.gpu
def test_fork_after_use_is_refused_cleanly():
    import ctypes as C
    import numpy as np
    from kmer_spans_amd import _lib
    L = _lib.load()
    L.ks_set_fork_broker(0)  # (the refusal itself; the broker: test_fork_broker_* below)
    seqs = (C.c_char_p * 1)(b"ACGTACGTAC")
    lens = np.array([10], dtype=np.int64)
    counts = np.zeros(16, dtype=np.int32)
    n = C.c_double(0)
    # the parent initialises HIP through the default context
    _lib.check(L.ks_kmer_counts(None, seqs, lens.ctypes.data, 1, 2, counts.ctypes.data, C.byref(n)))

    def call():
        c2 = np.zeros(16, dtype=np.int32)
        n2 = C.c_double(0)
        rc = L.ks_kmer_counts(None, seqs, lens.ctypes.data, 1, 2, c2.ctypes.data, C.byref(n2))
        return rc, L.ks_last_error().decode()

    rc, msg = _child_status(call)
    assert rc == 2 and "fork" in msg  # KS_ERR_DEVICE with the explanation
    # the parent is unaffected
    _lib.check(L.ks_kmer_counts(None, seqs, lens.ctypes.data, 1, 2, counts.ctypes.data, C.byref(n)))
    assert n.value == 9


def test_fork_after_hip_init_is_refused_cpu():
    """Without a GPU the parent's first call fails (no device) but has
    initialised HIP; a forked child is still refused with the fork message
    before it makes any HIP call."""
    import ctypes as C
    import numpy as np
    import torch
    if torch.cuda.is_available():
        pytest.skip("covered by the GPU test")
    from kmer_spans_amd import _lib
    L = _lib.load()
    L.ks_set_fork_broker(0)
    seqs = (C.c_char_p * 1)(b"ACGTACGTAC")
    lens = np.array([10], dtype=np.int64)
    counts = np.zeros(16, dtype=np.int32)
    n = C.c_double(0)
    assert L.ks_kmer_counts(None, seqs, lens.ctypes.data, 1, 2, counts.ctypes.data, C.byref(n)) == 2

    def call():
        rc = L.ks_kmer_counts(None, seqs, lens.ctypes.data, 1, 2, counts.ctypes.data, C.byref(n))
        return rc, L.ks_last_error().decode()

    rc, msg = _child_status(call)
    assert rc == 2 and "fork" in msg


def _scenario(mode):
    """tests/fork_broker_scenario.py in a fresh process (the broker is forked
    by a process that has not touched HIP yet)."""
    env = dict(os.environ, KS_FORK_BROKER="1")
    p = subprocess.run([sys.executable, SCENARIO, mode], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_fork_broker_mclapply_pattern():
    """test.R:351 then :554-565: the parent calls, forked workers call
    kmer_counts, kmer_regions (with visits), kmer_low_comp_regions,
    window_kmer_dist (with positions) and lr_regions through the broker; every
    result equals the parent's own call on the same input; six workers at
    once (the broker's server threads) give the same results; a worker's
    kmers_to_file with relative paths after a chdir writes into ITS
    directory."""
    r = _scenario("gpu")
    assert r["workers_ok"], r
    assert r["workers_equal"], r
    assert sum(r["regions"]) > 0
    assert r["concurrent_ok"] and r["concurrent_equal"], r
    assert r["file_ok"], r


def test_fork_broker_plumbing_cpu():
    """Without a GPU: a worker's call reaches the broker (its error is the
    broker's "no device", not the fork refusal); argument errors are still
    raised in the worker."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("covered by the GPU test")
    r = _scenario("cpu")
    assert r["worker_err"] and "fork" not in r["worker_err"], r
    assert r["worker_err"] == r["parent"], r
    assert "less than 1+MAX_K" in r["worker_arg_err"], r
    # the broker serves only the owner's descendants (SO_PEERCRED + ancestry)
    assert "went away" in r["stranger_err"] or "not reachable" in r["stranger_err"], r
