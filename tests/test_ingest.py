"""Ingest: FASTA parsed on the device, batched
multi-k counting, and kmers.to.file / read.kmers count files
(kmer_spans.R:113-186).

CPU tests: the oracle's FASTA restatement on hand-checked cases, the count
file format through the library's host functions against the oracle's byte
image.  GPU tests: the device parser and the batched counter against the
oracle on random and edge-case inputs, and kmers_to_file end to end.

Parity note: the reference reads FASTA with Biostrings (absent here); the
line rules are restated from its documentation and are "parity unpinned"
beyond these hand-checked cases.
"""
import gzip
import os
import random

import numpy as np
import pytest


@pytest.fixture(scope="module")
def ctx():
    from kmer_spans_amd import _lib
    return _lib.context(0)


# ------------------------------------------------------------------ helpers

def _random_fasta(rng, nrec, maxlen, width=None, crlf=False, lower=0.3, comments=True, empty_lines=True,
                  alphabet="ACGT"):
    out = []
    recs = []
    for r in range(nrec):
        L = rng.randrange(0, maxlen + 1)
        seq = []
        i = 0
        while i < L:
            if rng.random() < 0.02:
                n = min(L - i, rng.randrange(1, 40))
                seq.append("N" * n)
                i += n
            else:
                c = rng.choice(alphabet)
                seq.append(c.lower() if rng.random() < lower else c)
                i += 1
        s = "".join(seq)
        nl = "\r\n" if crlf else "\n"
        name = f"rec{r} desc {rng.randrange(1000)}"
        out.append(">" + name + nl)
        if comments and rng.random() < 0.1:
            out.append(";comment line" + nl)
        w = width or rng.randrange(1, 120)
        for j in range(0, len(s), w):
            out.append(s[j:j + w] + nl)
            if empty_lines and rng.random() < 0.02:
                out.append(nl)
        recs.append((name, s.upper()))
    text = "".join(out)
    if rng.random() < 0.5 and text.endswith("\n"):
        text = text[:-1]  # no final newline
        if text.endswith("\r"):
            text = text[:-1]
    return text, recs


# ------------------------------------------------------------- CPU: oracle

def test_oracle_fasta_known_answers(oracle):
    r = oracle.fasta_parse(b">a b\nACgt\nNN\n\n;c\n>x\r\nac-+.\r\n>e\n")
    assert r["names"] == ["a b", "x", "e"]
    assert r["seqs"] == [b"ACGTNN", b"AC-+.", b""]
    assert r["n_records"] == 3 and r["bases_all"] == 11
    r = oracle.fasta_parse(b">a\nAC\n>b\nACGT", 3)
    assert r["names"] == ["b"] and r["seqs"] == [b"ACGT"] and r["bases_all"] == 6
    assert oracle.fasta_parse(b"")["n_records"] == 0
    assert oracle.fasta_parse(b"\n\n;x\n")["n_records"] == 0
    with pytest.raises(oracle.OracleError, match="before description at 0"):
        oracle.fasta_parse(b"AC\n>a\n")
    with pytest.raises(oracle.OracleError, match="invalid byte at 4"):
        oracle.fasta_parse(b">a\nAZ\n")
    with pytest.raises(oracle.OracleError, match="invalid byte at 5"):
        oracle.fasta_parse(b">a\nAC GT\n")  # blanks are not sequence letters
    with pytest.raises(oracle.OracleError, match="invalid byte at 3"):
        oracle.fasta_parse(b">a\n\rAC\n")  # a CR that does not end a line


def test_oracle_fasta_random_matches_generator(oracle):
    rng = random.Random(3)
    for _ in range(20):
        text, recs = _random_fasta(rng, rng.randrange(0, 6), 300, crlf=rng.random() < 0.3)
        r = oracle.fasta_parse(text.encode())
        assert r["names"] == [n for n, _ in recs]
        assert r["seqs"] == [s.encode() for _, s in recs]


def test_count_file_format_matches_oracle(oracle, tmp_path):
    import kmer_spans_amd as K
    rng = np.random.default_rng(5)
    ks = [1, 3, 2]
    counts = [rng.integers(-2**31, 2**31 - 1, size=4 ** k, dtype=np.int64).astype(np.int32) for k in ks]
    f = tmp_path / "counts_1_3_2.bin"
    K.write_kmers(f, ks, counts)
    assert f.read_bytes() == oracle.count_file_bytes(K.kmer_magic(), ks, counts)
    r = K.read_kmers(f)
    o = oracle.read_count_file(f.read_bytes(), K.kmer_magic())
    assert r["k"].tolist() == o["k"].tolist() == ks
    for a, b, c in zip(r["counts"], o["counts"], counts):
        assert np.array_equal(a, c) and np.array_equal(b, c)
    assert K.read_kmers(f, magic=1) is False
    # n < 1 -> FALSE; truncated file -> short vectors (readBin stops at EOF)
    g = tmp_path / "zero.bin"
    g.write_bytes(np.array([K.kmer_magic(), 0], dtype="<i4").tobytes())
    assert K.read_kmers(g) is False and oracle.read_count_file(g.read_bytes(), K.kmer_magic()) is False
    h = tmp_path / "short.bin"
    h.write_bytes(f.read_bytes()[:-20])
    r = K.read_kmers(h)
    o = oracle.read_count_file(h.read_bytes(), K.kmer_magic())
    assert [len(c) for c in r["counts"]] == [len(c) for c in o["counts"]] == [4, 64, 11]
    with pytest.raises(K.KmerSpansError):
        K.write_kmers(tmp_path / "bad.bin", [2], [np.zeros(3, dtype=np.int32)])


# ---------------------------------------------------------------- GPU: parse

def _check_parse(D, ctx, oracle, text, min_len=0):
    o = oracle.fasta_parse(text.encode() if isinstance(text, str) else text, min_len)
    fa = D.parse_fasta(ctx, text, min_len)
    try:
        assert fa.n_records == o["n_records"]
        assert fa.bases_all == o["bases_all"]
        assert fa.names == o["names"]
        assert fa.host_seqs() == o["seqs"]
        assert fa.bases_kept == sum(len(s) for s in o["seqs"])
    finally:
        fa.close()


@pytest.mark.gpu
def test_fasta_parse_edges(oracle, ctx):
    from kmer_spans_amd import device as D
    cases = [b">a b\nACgt\nNN\n\n;c\n>x\r\nac-+.\r\n>e\n", b">a\nAC\n>b\nACGT", b">only", b">\n\n\n",
             b"\n\n>a\nA\n;x\nC\r\n", b">a\r\n\r\nAC\r", b">a\n" + b"ACGT" * 2000, b";c\n>a\nAC\n"]
    for c in cases:
        for ml in (0, 2, 5):
            _check_parse(D, ctx, oracle, c, ml)
    fa = D.parse_fasta(ctx, b"")
    assert fa.nseq == 0 and fa.n_records == 0
    fa.close()


@pytest.mark.gpu
def test_fasta_parse_errors(ctx):
    import kmer_spans_amd as K
    from kmer_spans_amd import device as D
    with pytest.raises(K.KmerSpansError, match="invalid one-letter sequence code 'Z'.*line 2"):
        D.parse_fasta(ctx, b">a\nAZ\n")
    with pytest.raises(K.KmerSpansError, match="before the first description line"):
        D.parse_fasta(ctx, b"AC\n>a\n")
    with pytest.raises(K.KmerSpansError, match="line 3"):
        D.parse_fasta(ctx, b">a\nACGT\nAC GT\n")
    # an invalid byte deep in a large file (crosses many tiles)
    big = b">a\n" + b"ACGT" * 100000 + b"\n>b\n" + b"AC" * 5000 + b"*\n"
    with pytest.raises(K.KmerSpansError, match="'\\*'"):
        D.parse_fasta(ctx, big)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_fasta_parse_random(oracle, ctx, seed):
    from kmer_spans_amd import device as D
    rng = random.Random(seed)
    for _ in range(6):
        text, _ = _random_fasta(rng, rng.randrange(1, 30), rng.choice([50, 3000, 20000]),
                                width=rng.choice([None, 60, 4096, 1]), crlf=rng.random() < 0.3,
                                alphabet="ACGTRYKMSWBDHVN-.+")
        _check_parse(D, ctx, oracle, text, rng.choice([0, 0, 100, 5000]))


@pytest.mark.gpu
def test_fasta_load_file_and_gzip(oracle, ctx, tmp_path):
    from kmer_spans_amd import device as D
    rng = random.Random(11)
    text, _ = _random_fasta(rng, 40, 200000, width=60)
    o = oracle.fasta_parse(text.encode(), 1000)
    p = tmp_path / "g.fa"
    p.write_bytes(text.encode())
    q = tmp_path / "g.fa.gz"
    q.write_bytes(gzip.compress(text.encode(), compresslevel=1))
    for path in (p, q):
        fa = D.load_fasta(ctx, str(path), 1000)
        try:
            assert fa.names == o["names"] and fa.host_seqs() == o["seqs"]
            assert fa.bases_all == o["bases_all"]
        finally:
            fa.close()


@pytest.mark.gpu
def test_fasta_records_scan_like_host_upload(oracle, ctx):
    """A parsed FASTA is a ks_dev_seqs: the span scan over it equals the scan
    of the same sequences uploaded from host strings and the oracle."""
    import kmer_spans_amd as K
    from kmer_spans_amd import device as D
    rng = random.Random(5)
    text, recs = _random_fasta(rng, 12, 30000, width=70)
    fa = D.parse_fasta(ctx, text)
    seqs = [s for _, s in recs]
    k = 7
    cnt = K.kmer_counts(seqs, k)
    w = K.pm1_table(cnt["counts"], k)
    tab = D.DeviceTable(ctx, w, k, 0.0)
    pos, score, _ = D.scan(ctx, fa, k, tab, 50, 10.0)
    o = oracle.kmer_regions(seqs, k, w, 50, 10.0, visits=False)
    assert np.array_equal(pos, o["pos"])
    assert np.array_equal(score[0].view(np.uint64), o["score"][0].view(np.uint64))
    fa.close()


# ----------------------------------------------------------- GPU: multi-k

@pytest.mark.gpu
@pytest.mark.parametrize("ks", [[2], [1, 2, 3, 4, 5, 6, 7], [7, 8, 11], [13, 1, 6, 9], [15, 3],
                                [1, 2, 3, 4, 5, 6, 7, 8, 9, 10]])
def test_count_multi_vs_oracle(oracle, ctx, ks):
    import torch
    from kmer_spans_amd import device as D
    rng = random.Random(sum(ks))
    seqs = []
    for _ in range(7):
        L = rng.randrange(0, 20000)
        s = "".join(rng.choice("ACGTacgtNR") if rng.random() < 0.1 else rng.choice("ACGT") for _ in range(L))
        seqs.append(s)
    seqs += ["ACGT", "NNACG", "ACGTN" * 3, "A" * 16]  # Q1 cases
    ds = D.from_host(seqs)
    counts = [torch.zeros(4 ** k, dtype=torch.int32, device="cuda") for k in ks]
    words = D.count_multi(ctx, ds, ks, counts)
    for k, c, w in zip(ks, counts, words):
        n, oc = oracle.kmer_counts(seqs, k)
        assert w == n, k
        assert np.array_equal(c.cpu().numpy(), oc), k


# --------------------------------------------------------- GPU: end to end

@pytest.mark.gpu
def test_kmers_to_file_end_to_end(oracle, tmp_path):
    import kmer_spans_amd as K
    rng = random.Random(9)
    text, _ = _random_fasta(rng, 25, 40000, width=80)
    fa_path = tmp_path / "x.fa"
    fa_path.write_bytes(text.encode())
    o = oracle.fasta_parse(text.encode(), 5000)
    ks = [13, 2, 7]
    res = K.kmers_to_file(str(fa_path), str(tmp_path / "out_"), ks, min_l=5000)
    assert res[0] == str(fa_path)
    assert res[1] == str(tmp_path / "out_counts_13_2_7.bin")
    assert res[2:] == [float(o["bases_all"]), float(sum(map(len, o["seqs"]))), float(len(o["seqs"]))]
    counts = [oracle.kmer_counts(o["seqs"], k)[1] for k in ks]
    assert open(res[1], "rb").read() == oracle.count_file_bytes(K.kmer_magic(), ks, counts)
    r = K.read_kmers(res[1])
    assert r["k"].tolist() == ks
    # NA results: nothing left after the filter, a bad k, an unreadable file
    na = K.kmers_to_file(str(fa_path), str(tmp_path / "y_"), [5], min_l=10 ** 9)
    assert na[1] is None and na[2] == float(o["bases_all"]) and na[3] == 0.0 and na[4] == 0.0
    na = K.kmers_to_file(str(fa_path), str(tmp_path / "z_"), [16], min_l=0)
    assert na[1] is None and na[4] == float(o["n_records"])
    na = K.kmers_to_file(str(tmp_path / "missing.fa"), str(tmp_path / "w_"), [5])
    assert na[1:] == [None, 0.0, 0.0, 0.0]
    assert not os.path.exists(tmp_path / "y_counts_5.bin")
