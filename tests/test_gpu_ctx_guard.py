"""One context, two threads (include/kmer_spans.h: a context takes one call
at a time): an entry point entered while another thread is inside one on the
same context fails with KS_ERR_ARG ("in use by another thread") instead of
racing on the context's workspace; each thread's completed calls stay exact."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_second_thread_is_refused():
    import torch
    from kmer_spans_amd import _lib, api, device as D, genome
    ctx = _lib.Context(0)
    D.bind_torch_stream(ctx)
    k = 11
    s = genome.contig(20_000_000, 7, device="cuda", repeats=True)
    ds = D.from_parts([s], [s.numel()], "cuda")
    counts = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    words = D.count(ctx, ds, k, counts)
    w = api.log2_table(counts.cpu().numpy(), k)
    tab = D.DeviceTable(ctx, w, k, 0.0, compress=True, expand=True, freq=counts)
    ref = D.scan(ctx, ds, k, tab, 100, 20.0)
    torch.cuda.synchronize()

    out, errs = [], []
    stop = threading.Event()

    def scans():
        try:
            done = 0
            while done < 30:
                try:
                    out.append(D.scan(ctx, ds, k, tab, 100, 20.0)[:2])
                    done += 1
                except _lib.KmerSpansError as e:
                    if "another thread" not in str(e):
                        raise
        except Exception as e:  # surfaced below
            errs.append(e)
        finally:
            stop.set()

    th = threading.Thread(target=scans)
    th.start()
    busy = 0
    c2 = torch.zeros(4 ** k, dtype=torch.int32, device="cuda")
    while not stop.is_set():
        try:
            c2.zero_()
            assert D.count(ctx, ds, k, c2) == words
        except _lib.KmerSpansError as e:
            assert "another thread" in str(e), e
            busy += 1
    th.join()
    assert not errs, errs
    assert busy > 0  # the calls did overlap
    for pos, sc in out:
        assert np.array_equal(pos, ref[0])
        assert np.array_equal(sc.view(np.uint64), ref[1].view(np.uint64))
    tab.close()
    ctx.close()
