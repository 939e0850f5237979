"""ctypes wrapper of the R .Call shim compiled against tests/rstub (test-only)."""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "rstub")
LIB = os.path.join(STUB, "librshim.so")
INTSXP, REALSXP, STRSXP, VECSXP = 13, 14, 16, 19


def build():
    srcs = [os.path.join(ROOT, "kmer_spans_amd", "rcall", "kmer_spans_call.c"), os.path.join(STUB, "rstub.c")]
    libdir = os.path.join(ROOT, "kmer_spans_amd")
    subprocess.check_call(["gcc", "-O1", "-Wall", "-fPIC", "-shared", "-I", STUB, "-I", os.path.join(ROOT, "include"),
                           *srcs, "-L", libdir, "-lkmerspans", f"-Wl,-rpath,{libdir}", "-o", LIB])
    return LIB


class RShim:
    def __init__(self):
        build()
        L = C.CDLL(LIB)
        P = C.c_void_p
        for n, a, r in [("rs_init", [], C.c_int), ("rs_nroutines", [], C.c_int), ("rs_routine_name", [C.c_int], C.c_char_p),
                        ("rs_routine_nargs", [C.c_int], C.c_int), ("rs_str", [C.c_int, P, P], P),
                        ("rs_int", [C.c_int, P], P), ("rs_real", [C.c_int, P], P), ("rs_call", [C.c_char_p, P, C.c_int], P),
                        ("rs_type", [P], C.c_int), ("rs_length", [P], C.c_long), ("rs_nrow", [P], C.c_int),
                        ("rs_ncol", [P], C.c_int), ("rs_elt", [P, C.c_long], P), ("rs_data", [P], P),
                        ("rs_error", [], C.c_char_p), ("rs_reset", [], None)]:
            getattr(L, n).argtypes = a
            getattr(L, n).restype = r
        L.rs_init()
        self.L = L

    def routines(self):
        return {self.L.rs_routine_name(i).decode(): self.L.rs_routine_nargs(i) for i in range(self.L.rs_nroutines())}

    def str_(self, seqs):
        bs = [s.encode("latin-1") if isinstance(s, str) else bytes(s) for s in seqs]
        arr = (C.c_char_p * max(len(bs), 1))(*bs)
        lens = np.array([len(b) for b in bs] or [0], dtype=np.int32)
        return self.L.rs_str(len(bs), arr, lens.ctypes.data)

    def int_(self, v):
        v = np.ascontiguousarray(np.atleast_1d(v), dtype=np.int32)
        return self.L.rs_int(v.size, v.ctypes.data)

    def real(self, v):
        v = np.ascontiguousarray(np.atleast_1d(v), dtype=np.float64)
        return self.L.rs_real(v.size, v.ctypes.data)

    def call(self, name, *args):
        arr = (C.c_void_p * len(args))(*args)
        r = self.L.rs_call(name.encode(), arr, len(args))
        if not r:
            raise RuntimeError(self.L.rs_error().decode())
        return r

    def to_py(self, x):
        t, n = self.L.rs_type(x), self.L.rs_length(x)
        if t == VECSXP:
            return [self.to_py(self.L.rs_elt(x, i)) for i in range(n)]
        if t == INTSXP:
            a = np.ctypeslib.as_array(C.cast(self.L.rs_data(x), C.POINTER(C.c_int32)), shape=(max(n, 1),))[:n].copy()
        elif t == REALSXP:
            a = np.ctypeslib.as_array(C.cast(self.L.rs_data(x), C.POINTER(C.c_double)), shape=(max(n, 1),))[:n].copy()
        elif t == STRSXP:
            return [C.string_at(self.L.rs_data(self.L.rs_elt(x, i)), self.L.rs_length(self.L.rs_elt(x, i))).decode()
                    for i in range(n)]
        else:
            return None
        nr, nc = self.L.rs_nrow(x), self.L.rs_ncol(x)
        return a.reshape(nc, nr).T if nc > 1 or (nr != n) else a  # column-major matrices
