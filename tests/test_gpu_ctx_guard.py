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


def test_refused_kmers_to_file_leaves_the_owner_alone(tmp_path):
    """ks_kmers_to_file on the default context while another thread is inside
    a kmer_regions call on it is refused, and the refusal does not release
    the owner's workspace (the end-of-call guard comes after the ownership
    check): the owner's results stay exact."""
    import kmer_spans_amd as K
    from kmer_spans_amd import _lib
    s = np.frombuffer(b"ACGT", dtype=np.uint8)[np.random.default_rng(3).integers(0, 4, size=24_000_000)].tobytes().decode()
    fa = tmp_path / "q.fa"
    fa.write_text(">a\n" + s[:5000] + "\n>b\n" + s[5000:9000] + "\n")
    k = 11
    w = np.round(np.random.default_rng(1).normal(size=4 ** k) * 4) / 4 + 0.05
    ref = K.kmer_regions(s, k, w, 40, 6.0)
    out, errs = [], []
    stop = threading.Event()

    def owner():
        # both threads race for the default context: the owner's own call
        # may be the refused one (kmers_to_file got there first); it tries
        # again, and every call it completes must be exact
        try:
            while len(out) < 6:
                try:
                    out.append(K.kmer_regions(s, k, w, 40, 6.0))
                except _lib.KmerSpansError as e:
                    if "another thread" not in str(e):
                        raise
        except Exception as e:  # surfaced below
            errs.append(e)
        finally:
            stop.set()

    th = threading.Thread(target=owner)
    th.start()
    refused = 0
    while not stop.is_set():
        try:
            K.kmers_to_file(str(fa), str(tmp_path / "o_"), [3], min_l=1)
        except _lib.KmerSpansError as e:
            assert "another thread" in str(e), e
            refused += 1
    th.join()
    assert not errs, errs
    assert refused > 0
    for r in out:
        assert np.array_equal(r["pos"], ref["pos"])
        assert np.array_equal(r["score"].view(np.uint64), ref["score"].view(np.uint64))
        assert np.array_equal(r["counts"], ref["counts"])
