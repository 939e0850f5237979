"""The R .Call shim (kmer_spans_amd/rcall/kmer_spans_call.c) through the
tests/rstub R C-API emulation: the six registered routines of the reference
(kmer_spans.c:795-802) with their arities, error strings, and -- on a GPU --
results equal to the oracle; plus kmers_to_file_r, the body of kmers.to.file
(kmer_spans.R:127-160) as one routine."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def R():
    from tests.rshim import RShim
    return RShim()


def test_registration_table(R):
    assert R.routines() == {"kmer_counts": 2, "kmer_regions_r": 5, "kmer_low_comp_regions": 5,
                            "kmer_seq_r": 1, "tr_lr_regions_r": 5, "windowed_kmer_count_distributions_r": 5,
                            "kmers_to_file_r": 5}


def test_reference_error_strings(R):
    cases = [
        (("kmer_counts", R.int_([1]), R.int_([2])), "seq_r must be a character vector of length at least one"),
        (("kmer_counts", R.str_(["ACGT"]), R.real([2.0])), "k_r must be an integer vector of length at least one"),
        (("kmer_counts", R.str_(["ACGT"]), R.int_([17])), "k must be a positive integer less than 1+MAX_K"),
        (("kmer_regions_r", R.str_(["ACGT"]), R.int_([1]), R.int_([1, 2, 3, 4]), R.int_([0]), R.real([0.0])),
         "kmer_w_r must be a double vector of length k^4"),
        (("kmer_regions_r", R.str_(["ACGT"]), R.int_([1]), R.real([1.0] * 4), R.int_([0, 1]), R.real([0.0])),
         "the minimum width must be an integer vector of length 1"),
        (("kmer_regions_r", R.str_(["ACGT"]), R.int_([1]), R.real([1.0] * 4), R.int_([0]), R.int_([0])),
         "the minimum score must be a REAL vector of length 1"),
        (("kmer_regions_r", R.str_(["ACGT"]), R.int_([16]), R.real([1.0] * 4), R.int_([0]), R.real([0.0])),
         "kmer sizes larger than or equal to 16 not currently supported"),
        (("kmer_regions_r", R.str_(["ACGT"]), R.int_([2]), R.real([1.0] * 4), R.int_([0]), R.real([0.0])),
         "kmer_w contains 4 elements but should have 16"),
        (("kmer_low_comp_regions", R.str_(["ACGT"]), R.int_([2]), R.int_([0]), R.real([0.0]), R.real([1.5])),
         "the threshold must be between 0 and 1"),
        (("kmer_low_comp_regions", R.str_(["ACGT"]), R.int_([2]), R.int_([0]), R.real([0.0]), R.int_([0])),
         "the threshold must be a REAL vector of length 1"),
        (("kmer_seq_r", R.int_([0])), "k_r (0) should be smaller than MAX_K (16) and larger than 0"),
        (("kmer_seq_r", R.int_([1, 2])), "k_r should be an integer of length 1"),
        (("tr_lr_regions_r", R.int_([0]), R.int_([1, 0]), R.str_(["A"]), R.real([0.0]), R.real([0.0])),
         "seq_r should be a character vector of of positive length"),
        (("tr_lr_regions_r", R.str_(["ACGT"]), R.int_([1]), R.str_(["A"]), R.real([0.0]), R.real([0.0])),
         "params_r should have two integers (k, and min_length)"),
        (("tr_lr_regions_r", R.str_(["ACGT"]), R.int_([1, 0]), R.int_([0]), R.real([0.0]), R.real([0.0])),
         "kmers_r should be a character vector"),
        (("tr_lr_regions_r", R.str_(["ACGT"]), R.int_([0, 0]), R.str_(["A"]), R.real([0.0]), R.real([0.0])),
         "k should be a positive value less than MAX_K"),
        (("tr_lr_regions_r", R.str_(["ACGT"]), R.int_([1, -1]), R.str_(["A"]), R.real([0.0]), R.real([0.0])),
         "min_length should be a positive integer"),
        (("tr_lr_regions_r", R.str_(["ACGT"]), R.int_([1, 0]), R.str_(["A"]), R.real([0.0]), R.real([0.0])),
         "kmers_r, freq_a, freq_b should all be 4^k long"),
        (("windowed_kmer_count_distributions_r", R.int_([0]), R.str_(["AC"]), R.int_([2]), R.int_([6]), R.int_([0])),
         "seq_r should be a character vector with at least one element"),
        (("windowed_kmer_count_distributions_r", R.str_(["ACGT"]), R.int_([0]), R.int_([2]), R.int_([6]), R.int_([0])),
         "kmers_r should be a character vector with at least one element"),
        (("windowed_kmer_count_distributions_r", R.str_(["ACGT"]), R.str_(["AC"]), R.int_([2, 3]), R.int_([6]),
          R.int_([0])), "k_r should be an integer vector with one element"),
        (("windowed_kmer_count_distributions_r", R.str_(["ACGT"]), R.str_(["AC"]), R.int_([2]), R.real([6.0]),
          R.int_([0])), "window_r should be an integer vector with one element"),
        (("windowed_kmer_count_distributions_r", R.str_(["ACGT"]), R.str_(["AC"]), R.int_([2]), R.int_([6]),
          R.real([0.0])), "ret_flag_r should a single integer"),
        (("windowed_kmer_count_distributions_r", R.str_(["ACGT"]), R.str_(["AC"]), R.int_([16]), R.int_([40]),
          R.int_([0])), "kmer sizes larger than or equal to 16 not currently supported"),
        (("windowed_kmer_count_distributions_r", R.str_(["ACGT"]), R.str_(["AC", "ACG"]), R.int_([2]), R.int_([6]),
          R.int_([0])), "All kmers specified must be of the same length"),
        (("windowed_kmer_count_distributions_r", R.str_(["ACGT"]), R.str_(["AC"]), R.int_([2]), R.int_([3]),
          R.int_([0])), "The window size must be at least two times k"),
    ]
    for args, msg in cases:
        with pytest.raises(RuntimeError, match=msg.replace("^", "\\^").replace("+", "\\+").replace("(", "\\(").replace(")", "\\)")):
            R.call(*args)


def test_kmer_seq_r(R, oracle):
    for k in (1, 3):
        assert R.to_py(R.call("kmer_seq_r", R.int_([k]))) == oracle.kmer_seq(k)


@pytest.mark.gpu
def test_shim_results_vs_oracle(R, oracle):
    rng = np.random.default_rng(2)
    seqs = ["".join(rng.choice(list("ACGTN"), 3000, p=[.24, .24, .24, .24, .04])), "CAAAAAATCAACCCCCC", "AC"]
    n, c = oracle.kmer_counts(seqs, 4)
    got = R.to_py(R.call("kmer_counts", R.str_(seqs), R.int_([4])))
    assert got[0][0] == n and np.array_equal(got[1], c)
    w = rng.normal(size=4 ** 4)
    o = oracle.kmer_regions(seqs, 4, w, 3, 1.0)
    got = R.to_py(R.call("kmer_regions_r", R.str_(seqs), R.int_([4]), R.real(w), R.int_([3]), R.real([1.0])))
    assert got[0][0] == o["n"] and np.array_equal(got[1], o["counts"])
    assert np.array_equal(np.asarray(got[2]).reshape(3, -1), o["pos"])
    # scores bitwise, with the reference's zero second row (kmer_spans.c:280)
    sc = np.ascontiguousarray(np.asarray(got[3], dtype=np.float64).reshape(2, -1))
    assert np.array_equal(sc.view(np.uint64), o["score"].view(np.uint64))
    lc = oracle.low_comp_regions(seqs, 3, 5, 2.0, 0.6)
    got = R.to_py(R.call("kmer_low_comp_regions", R.str_(seqs), R.int_([3]), R.int_([5]), R.real([2.0]), R.real([0.6])))
    assert np.array_equal(got[0], lc["n"]) and np.array_equal(got[1], lc["counts"])
    assert np.array_equal(np.asarray(got[2]).view(np.uint64), lc["w_rank"].view(np.uint64))
    assert np.array_equal(np.asarray(got[3]).reshape(3, -1), lc["pos"])
    sc = np.ascontiguousarray(np.asarray(got[4], dtype=np.float64).reshape(2, -1))
    assert np.array_equal(sc.view(np.uint64), lc["score"].view(np.uint64))


@pytest.mark.gpu
def test_config1_through_call_shim(R, oracle):
    """BASELINE config 1 through the .Call entry points: 1 Mbp i.i.d. ACGT
    (xorshift64, seed 1), k = 7, +-1 table from its own counts
    (README.md:37-42: f >= f_med -> 1 else -1), min_width 100, min_score 20.
    kmer_counts and kmer_regions_r results (counts, visit histogram, regions,
    scores) equal the oracle's bit for bit; SURVEY 8(d) expects one region."""
    from kmer_spans_amd import api, genome
    seq = genome.uniform_xorshift(1_000_000, 1).decode()
    got = R.to_py(R.call("kmer_counts", R.str_([seq]), R.int_([7])))
    n, c = oracle.kmer_counts([seq], 7)
    assert got[0][0] == n and np.array_equal(got[1], c)
    w = api.pm1_table(np.asarray(got[1], dtype=np.int32), 7)
    assert np.array_equal(np.asarray(w).view(np.uint64), oracle.pm1_table(c, 7).view(np.uint64))
    got = R.to_py(R.call("kmer_regions_r", R.str_([seq]), R.int_([7]), R.real(w), R.int_([100]), R.real([20.0])))
    o = oracle.kmer_regions([seq], 7, w, 100, 20.0)
    pos = np.asarray(got[2]).reshape(3, -1)
    assert got[0][0] == o["n"] == 1_000_000
    assert np.array_equal(got[1], o["counts"])
    assert np.array_equal(pos, o["pos"])
    sc = np.ascontiguousarray(np.asarray(got[3], dtype=np.float64).reshape(2, -1))
    assert np.array_equal(sc.view(np.uint64), o["score"].view(np.uint64))
    assert pos.shape[1] >= 1


@pytest.mark.gpu
def test_shim_tr_lr_vs_oracle(R, oracle):
    rng = np.random.default_rng(4)
    k = 3
    seqs = ["".join(rng.choice(list("ACGTN"), 2000, p=[.24, .24, .24, .24, .04])), "GGNGGG", "ACGTTTGGA"]
    names = oracle.kmer_seq(k)
    perm = rng.permutation(4 ** k)
    ks = rng.normal(size=4 ** k)
    tr = rng.normal(size=4 ** k) - 0.2
    got = R.to_py(R.call("tr_lr_regions_r", R.str_(seqs), R.int_([k, 2]), R.str_([names[p] for p in perm]),
                         R.real(ks[perm]), R.real(tr[perm])))
    o = oracle.tr_lr_regions(seqs, k, 2, ks, tr)
    spectra = np.asarray(got[0])  # 4^k x 2
    assert np.array_equal(spectra[:, 0], ks) and np.array_equal(spectra[:, 1], tr)
    assert np.array_equal(np.asarray(got[1]).reshape(3, -1), o["pos"])
    assert np.array_equal(np.asarray(got[2]).reshape(2, -1)[0], o["score"][0])


@pytest.mark.gpu
def test_shim_windowed_vs_oracle(R, oracle):
    rng = np.random.default_rng(4)
    seqs = ["".join(rng.choice(list("ACGTN"), 5000, p=[.24, .24, .24, .24, .04])), "CGCCAATGCG", "ACGTACGTAC" * 3]
    kmers = ["CG", "GC", "AA", "NN", "TT"]
    o = oracle.windowed_dist(seqs, kmers, 2, 12, 1)
    got = R.to_py(R.call("windowed_kmer_count_distributions_r", R.str_(seqs), R.str_(kmers), R.int_([2]),
                         R.int_([12]), R.int_([1])))
    assert np.array_equal(got[0], o["dist"])
    assert np.array_equal(got[1], o["seq_i"])
    for g, w in zip(got[2], o["scores"]):
        if w is None:
            assert g is None
        else:
            assert np.array_equal(g, w)
