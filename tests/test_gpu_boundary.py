"""The drop-in boundary under the library's own background work and other
threads (kmer_regions_r / kmer_low_comp_regions,
kmer_spans.c:490-546, 548-621):

* the memory-policy-2 janitor returning a context's memory must not make a
  call on that context fail: the call waits for the release and is exact;
* a multi-device kmer_low_comp_regions owns its contexts from its first
  phase to its end (the janitor cannot free the staged bases between the
  phases, and another thread's call is refused rather than interleaved);
* the pass-1 epoch guard fails a scan whose post-processing would read pass-1
  results of another call, and the next call is exact again;
* the free-ordering probe: a spin kernel queued on the side / high-priority
  streams right before a workspace free -- the free never completes before it.
"""
import os
import re
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _genome(n=6_000_000, seed=3):
    rng = np.random.default_rng(seed)
    b = np.frombuffer(b"ACGTacgt", dtype=np.uint8)[rng.integers(0, 8, size=n)].copy()
    for a in range(300_000, n, 900_000):
        b[a:a + 1200] = ord("N")
    for a in range(100_000, n, 700_000):  # low-complexity stretches: regions
        b[a:a + 3000] = np.frombuffer(b"CA" * 1500, np.uint8)
    return [b[: n // 2].tobytes().decode(), b[n // 2:].tobytes().decode(), "ACGTNNACGT" * 30]


class _Env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update({k: str(v) for k, v in self.kv.items()})

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _same(g, o):
    assert np.array_equal(g["pos"], o["pos"])
    assert np.array_equal(g["score"].view(np.uint64), o["score"].view(np.uint64))
    assert np.array_equal(g["counts"], o["counts"])


def test_call_waits_for_a_janitor_release(oracle):
    """Policy 2, 0.3 s idle time, the janitor held 2.5 s inside its release
    (KS_DEBUG_JANITOR_HOLD_MS): a kmer_regions call issued 1 s after the
    previous one arrives while the janitor holds the context; it waits for
    the release (no 'in use by another thread'), then returns the oracle's
    regions, scores and visits."""
    import kmer_spans_amd as K
    from kmer_spans_amd import _lib
    L = _lib.load()
    seqs = _genome()
    k = 11
    w = np.round(np.random.default_rng(2).normal(size=4 ** k) * 4) / 4 + 0.05
    o = oracle.kmer_regions(seqs, k, w, 40, 6.0)
    L.ks_release_cache()
    _lib.check(L.ks_set_host_cache(2))
    _lib.check(L.ks_set_host_cache_idle(0.3))
    try:
        with _Env(KS_DEBUG_JANITOR_HOLD_MS=2500):
            _same(K.kmer_regions(seqs, k, w, 40, 6.0), o)
            time.sleep(1.0)  # the janitor took the context at ~0.3 s and holds it until ~2.8 s
            t0 = time.perf_counter()
            g = K.kmer_regions(seqs, k, w, 40, 6.0)
            dt = time.perf_counter() - t0
        _same(g, o)
        assert dt >= 1.2, f"the call did not wait for the janitor's release ({dt:.2f} s)"
    finally:
        L.ks_set_host_cache_idle(20.0)
        L.ks_release_cache()


def test_multi_low_comp_owns_its_contexts_between_phases(oracle):
    """Device list [0, 0], policy 2 with a 50 ms idle time: the previous
    call leaves both contexts due for release almost at once; the next
    kmer_low_comp_regions sleeps 1.5 s between its count and scan phases
    (KS_DEBUG_MULTI_PHASE_SLEEP_MS) while the janitor's deadline passes and
    another thread keeps calling kmer_counts on the list.  The janitor cannot
    take the contexts, the other thread is refused ('in use by another
    thread') while the call runs and never interleaves, and the call's counts,
    ranks, regions and scores equal the oracle's."""
    import kmer_spans_amd as K
    from kmer_spans_amd import _lib, api
    L = _lib.load()
    seqs = _genome(4_000_000, 9)
    k = 9
    ol = oracle.low_comp_regions(seqs, k, 20, 5.0, 0.75)
    n_all, oc = oracle.kmer_counts(seqs, k)
    api.set_devices([0, 0])
    _lib.check(L.ks_set_host_cache(2))
    _lib.check(L.ks_set_host_cache_idle(0.05))
    try:
        K.kmer_low_comp_regions(seqs, k, 20, 5.0, 0.75)  # lists both contexts
        res, errs = {}, []
        stop = threading.Event()

        def main_call():
            try:
                with _Env(KS_DEBUG_MULTI_PHASE_SLEEP_MS=1500):
                    res["lc"] = K.kmer_low_comp_regions(seqs, k, 20, 5.0, 0.75)
            except Exception as e:  # surfaced below
                errs.append(e)
            finally:
                stop.set()

        th = threading.Thread(target=main_call)
        th.start()
        time.sleep(0.3)  # inside the call (its phase gap lasts 1.5 s)
        refused, done = 0, 0
        while not stop.is_set():
            try:
                c = K.kmer_counts(seqs, k)
                done += 1
                assert np.array_equal(c["counts"], oc)
            except _lib.KmerSpansError as e:
                assert "another thread" in str(e), e
                refused += 1
            time.sleep(0.05)
        th.join()
        assert not errs, errs
        assert refused > 0
        lc = res["lc"]
        assert np.array_equal(lc["counts"], ol["counts"])
        assert np.array_equal(lc["w_rank"].view(np.uint64), ol["w_rank"].view(np.uint64))
        assert np.array_equal(lc["n"], ol["n"])
        assert np.array_equal(lc["pos"].T, ol["pos"])
        assert np.array_equal(lc["score"].T[0].view(np.uint64), ol["score"][0].view(np.uint64))
        st = _lib.multi_last_stats()
        assert st["total_ms"] > 0
    finally:
        api.set_devices([])
        L.ks_set_host_cache_idle(20.0)
        L.ks_release_cache()


def test_epoch_guard_fails_a_stale_read_and_recovers(oracle):
    """KS_TEST_EPOCH_STALE makes the stitch expect another epoch than pass 1
    stamped (what reading an earlier call's pass-1 results looks like): the
    chunked scan fails with the epoch error instead of returning regions; the
    next call, without the switch, equals the oracle."""
    import torch
    from kmer_spans_amd import _lib, api, device as D
    ctx = _lib.Context(0)
    D.bind_torch_stream(ctx)
    seqs = _genome(8_000_000, 5)
    k = 11
    parts = [torch.from_numpy(np.frombuffer(s.encode(), np.uint8).copy()).cuda() for s in seqs]
    ds = D.from_parts(parts, [p.numel() for p in parts], "cuda")
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    D.count(ctx, ds, k, counts)
    w = api.log2_table(counts.cpu().numpy(), k)
    tab = D.DeviceTable(ctx, w, k, 0.0, compress=True, expand=True, freq=counts)
    ctx.set_scan_algo(1)
    try:
        with _Env(KS_TEST_EPOCH_STALE=1):
            with pytest.raises(_lib.KmerSpansError, match="epoch check failed"):
                D.scan(ctx, ds, k, tab, 100, 20.0)
        pos, score, _ = D.scan(ctx, ds, k, tab, 100, 20.0)
        o = oracle.scan(seqs, k, w, 0.0, 100, 20.0)
        assert pos.shape[1] > 0
        assert np.array_equal(pos, o["pos"])
        assert np.array_equal(score.view(np.uint64), o["score"].view(np.uint64))
    finally:
        tab.close()
        ctx.close()


_SPIN = re.compile(r"\[spin\] (\S+) slot (-?\d+): spin ([\d.]+) ms queued on side\+hi, drain \(([^)]*)\) ([\d.]+) ms, "
                   r"hipFree ([\d.]+) ms")


@pytest.mark.parametrize("main_only", [False, True])
def test_free_waits_for_the_other_streams(oracle, capfd, main_only):
    """KS_DEBUG_SPIN_MS=300: before each workspace free (slots growing in
    ensure; the policy-0 release at the end of a host call) a 300 ms spin
    kernel is queued on the context's side and high-priority streams.  With
    the all-stream drain (the fix) the drain lasts the spin; with the round-4
    drain of the main stream only (KS_DEBUG_DRAIN_MAIN_ONLY) the call's
    results are exact too, and the report says whether hipFree itself waited
    (tools/probes/free_order_probe.py records both for DESIGN.md)."""
    import kmer_spans_amd as K
    from kmer_spans_amd import _lib
    L = _lib.load()
    k = 9
    w = np.round(np.random.default_rng(4).normal(size=4 ** k) * 4) / 4 + 0.1
    small, big = _genome(400_000, 1), _genome(3_000_000, 2)
    L.ks_release_cache()
    _lib.check(L.ks_set_host_cache(0))
    env = {"KS_DEBUG_SPIN_MS": 300}
    if main_only:
        env["KS_DEBUG_DRAIN_MAIN_ONLY"] = 1
    try:
        with _Env(**env):
            for seqs in (small, big):  # the second call grows the slots the first one sized
                _same(K.kmer_regions(seqs, k, w, 20, 3.0), oracle.kmer_regions(seqs, k, w, 20, 3.0))
    finally:
        L.ks_set_host_cache(2)
        L.ks_release_cache()
    err = capfd.readouterr().err
    lines = [m.groups() for m in _SPIN.finditer(err)]
    assert lines, err[-2000:]
    for where, slot, spin, how, drain, free in lines:
        assert ("main" in how) == main_only
        if not main_only:
            assert float(drain) >= 0.8 * float(spin), (where, slot, drain)
