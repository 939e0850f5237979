"""Fork safety of the C ABI: R's mclapply forks workers after the
parent may have used the library (test.R:351 then :554-559).  A child that
inherits a HIP context must get a clear KS_ERR_DEVICE status, never a hang or
a fault: nothing in the child may touch the parent's HIP state."""
import os

import pytest


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
