"""Timing of large hipMalloc / hipFree calls on the box (why did a 128 GiB
expanded-table allocation take 1.8 s in one run and 0.5 ms in another?)."""
import ctypes as C
import time

import torch

hip = C.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipFree.argtypes = [C.c_void_p]
hip.hipDeviceSynchronize.argtypes = []
hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]


def malloc(n):
    p = C.c_void_p()
    t = time.perf_counter()
    rc = hip.hipMalloc(C.byref(p), n)
    return p, (time.perf_counter() - t) * 1e3, rc


def free(p):
    t = time.perf_counter()
    hip.hipFree(p)
    return (time.perf_counter() - t) * 1e3


torch.zeros(1, device="cuda")
G = 1 << 30
p, ms, rc = malloc(128 * G)
print("fresh 128 GiB", round(ms, 2), rc, flush=True)
print("free", round(free(p), 2))
p, ms, rc = malloc(128 * G)
print("again 128 GiB", round(ms, 2), rc)
hip.hipMemset(p, 0, 128 * G)
hip.hipDeviceSynchronize()
print("free after touch", round(free(p), 2))
p, ms, rc = malloc(128 * G)
print("after touched free 128 GiB", round(ms, 2), rc)
free(p)
small = [malloc(256 << 20)[0] for _ in range(6)]
for q in small:
    hip.hipMemset(q, 0, 256 << 20)
hip.hipDeviceSynchronize()
for q in small:
    free(q)
p, ms, rc = malloc(128 * G)
print("after 6x256MB churn 128 GiB", round(ms, 2), rc)
free(p)
x = torch.empty(40 * G, dtype=torch.uint8, device="cuda")
x.fill_(1)
torch.cuda.synchronize()
p, ms, rc = malloc(128 * G)
print("with torch 40 GiB resident 128 GiB", round(ms, 2), rc)
hip.hipMemset(p, 0, 128 * G)
hip.hipDeviceSynchronize()
p2, ms, rc = malloc(32 * G)
print("second 32 GiB while 128+40 resident", round(ms, 2), rc)
free(p2)
free(p)
