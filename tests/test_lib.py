"""CPU-side checks of the product library: it loads, exports every symbol
include/kmer_spans.h declares, validates arguments before touching the
device (reference error strings), and its host table builders equal the
oracle's.  No compute call reaches the GPU here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exports_match_header():
    from kmer_spans_amd import _lib
    L = _lib.load()
    hdr = open(os.path.join(ROOT, "include", "kmer_spans.h")).read()
    declared = set(re.findall(r"\b(ks_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(_lib.EXPORTS), declared ^ set(_lib.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name
    assert b"gfx950" in L.ks_version()


def test_library_is_gfx950(tmp_path):
    import shutil
    import subprocess
    from kmer_spans_amd import _lib
    lib = tmp_path / "lib.so"  # objdump --offloading extracts bundles next to its input
    shutil.copy(_lib.LIB_PATH, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout + out.stderr


def test_validation_errors_before_device():
    import kmer_spans_amd as K
    with pytest.raises(K.KmerSpansError, match="k must be a positive integer less than 1\\+MAX_K"):
        K.kmer_counts("ACGT", 0)
    with pytest.raises(K.KmerSpansError, match="less than 1\\+MAX_K"):
        K.kmer_counts("ACGT", 16)
    with pytest.raises(K.KmerSpansError, match="seq_r must be a character vector"):
        K.kmer_counts([], 2)
    with pytest.raises(K.KmerSpansError, match="kmer sizes larger than or equal to 16"):
        K.api._lib.check(K.api.load().ks_kmer_regions(None, (C.c_void_p * 1)(0), np.zeros(1, np.int64).ctypes.data,
                                                      1, 16, np.zeros(1).ctypes.data, 1, 0, 0.0, None,
                                                      C.byref(C.c_double()), C.byref(K.api.Regions())))
    with pytest.raises(K.KmerSpansError, match="kmer_w contains 3 elements but should have 4"):
        K.api._lib.check(K.api.load().ks_kmer_regions(None, (C.c_void_p * 1)(0), np.zeros(1, np.int64).ctypes.data,
                                                      1, 1, np.zeros(3).ctypes.data, 3, 0, 0.0, None,
                                                      C.byref(C.c_double()), C.byref(K.api.Regions())))
    with pytest.raises(K.KmerSpansError, match="There should be a total of 4\\^k scores"):
        K.kmer_regions("ACGT", 1, [1.0, 2.0], 0, 0.0)
    with pytest.raises(K.KmerSpansError, match="threshold must be between 0 and 1"):
        K.kmer_low_comp_regions("ACGT", 1, 0, 0.0, thr=1.0)
    with pytest.raises(K.KmerSpansError, match="should be smaller than MAX_K"):
        K.kmer_seq(0)
    names = K.kmer_seq(1)
    with pytest.raises(K.KmerSpansError, match="params_r should have two integers"):
        K.lr_regions("ACGT", (1,), names, [0.0] * 4, [0.0] * 4)
    with pytest.raises(K.KmerSpansError, match="k should be a positive value less than MAX_K"):
        K.lr_regions("ACGT", (0, 0), names, [0.0] * 4, [0.0] * 4)
    with pytest.raises(K.KmerSpansError, match="min_length should be a positive integer"):
        K.lr_regions("ACGT", (1, -1), names, [0.0] * 4, [0.0] * 4)
    with pytest.raises(K.KmerSpansError, match="should all be 4\\^k long"):
        K.lr_regions("ACGT", (2, 0), names, [0.0] * 4, [0.0] * 4)
    with pytest.raises(K.KmerSpansError, match="seq_r should be a character vector of of positive length"):
        K.lr_regions([], (1, 0), names, [0.0] * 4, [0.0] * 4)


def test_named_scores_reordered():
    from kmer_spans_amd import api
    names = api.kmer_seq(1)
    w = api._ordered_scores(1, {"G": 4.0, "T": 3.0, "C": 2.0, "A": 1.0})
    assert names == ["A", "C", "T", "G"] and w.tolist() == [1.0, 2.0, 3.0, 4.0]
    with pytest.raises(api.KmerSpansError, match="all kmers not defined"):
        api._ordered_scores(1, {"A": 1, "C": 2, "T": 3, "X": 4})


@pytest.mark.parametrize("k", [1, 3, 7, 9])
def test_host_tables_match_oracle(oracle, k):
    import kmer_spans_amd as K
    rng = np.random.default_rng(100 + k)
    c = rng.integers(0, 1000, 4 ** k).astype(np.int32)
    c[rng.integers(0, 4 ** k, 4 ** k // 3)] = rng.integers(0, 5)  # ties
    assert np.array_equal(K.rank_table(c, k, float(c.sum())), oracle.rank_table(c, k, float(c.sum())))
    assert np.array_equal(K.log2_table(c, k), oracle.log2_table(c, k), equal_nan=True)
    assert np.array_equal(K.pm1_table(c, k), oracle.pm1_table(c, k), equal_nan=True)


def test_tables_zero_counts(oracle):
    import kmer_spans_amd as K
    c = np.zeros(16, dtype=np.int32)
    assert np.array_equal(K.log2_table(c, 2), oracle.log2_table(c, 2), equal_nan=True)
    c[3] = 5
    assert np.array_equal(K.log2_table(c, 2), oracle.log2_table(c, 2), equal_nan=True)
    assert np.array_equal(K.pm1_table(c, 2), oracle.pm1_table(c, 2), equal_nan=True)


def test_kmer_seq_matches_oracle(oracle):
    import kmer_spans_amd as K
    for k in (1, 2, 5):
        assert K.kmer_seq(k) == oracle.kmer_seq(k)


@pytest.mark.parametrize("case", ["huge_sum_ties", "dyadic", "skewed"])
def test_rank_table_closed_form(oracle, case):
    """The closed-form weighted-rank prefix (ks_internal.h RankPiece: runs of
    equal counts as integer progressions inside a binade, FP64 steps at the
    binade crossings) equals the sequential prefix bit for bit, including
    exact-half ties (odd counts added to a sum beyond 2^53) and long runs."""
    import kmer_spans_amd as K
    rng = np.random.default_rng({"huge_sum_ties": 1, "dyadic": 2, "skewed": 3}[case])
    if case == "huge_sum_ties":
        k = 12
        c = ((1 << 30) + 2 * rng.integers(0, 1000, 4 ** k) + 1).astype(np.int32)  # odd, sum > 2^53
        total = 1.0
    elif case == "dyadic":
        k = 10
        c = rng.integers(0, 40, 4 ** k).astype(np.int32)
        total = 2.0 ** -3  # d = 8c: exact steps, sums far past 2^53 ulp boundaries of small R
    else:
        k = 11
        c = np.minimum(rng.geometric(0.02, 4 ** k), 1 << 20).astype(np.int32)
        c[rng.integers(0, 4 ** k, 4 ** k // 4)] = 0
        total = float(c.astype(np.int64).sum())
    got, want = K.rank_table(c, k, total), oracle.rank_table(c, k, total)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
