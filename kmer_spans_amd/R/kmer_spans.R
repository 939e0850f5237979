## R front end of the MI355X span scanner: the span-scan functions of
## lmjakt/kmer_spans/kmer_spans.R (:5, :18-27, :41-52, :72-79, :84-86) with
## the same names, arguments and return values, calling the .Call shim in
## ../rcall/kmer_spans.so (built from kmer_spans_call.c, see INTEGRATION.md).
## Written for this repository; behaviour follows the reference line by line.

local({
    here <- dirname(sys.frame(1)$ofile)
    dyn.load(file.path(here, "..", "rcall", "kmer_spans.so"))
})

## magic number of the reference's binary count files (kmer_spans.R:5)
kmer.magic <- function() 310572L

## k-mer spectrum of a character vector (all sequences together):
## list(n = c(k=, n=), counts = integer(4^k), f = counts / sum(counts))
kmer.counts <- function(seq, k, with.f = TRUE) {
    k <- as.integer(k)
    res <- .Call("kmer_counts", seq, k)
    names(res) <- c("n", "counts")
    res$n <- c(k = k, n = res$n)
    if (with.f)
        res$f <- res$counts / sum(res$counts)
    res
}

## spans of high cumulative k-mer score, S = max(S + w[kmer], 0);
## kmer.scores must be named by k-mer (any order), 4^k of them
kmer.regions <- function(seq, k, kmer.scores, min.width, min.score) {
    if (length(kmer.scores) != 4^k)
        stop("There should be a total of 4^k scores")
    ks <- kmer.seq(k)
    if (!all(ks %in% names(kmer.scores)))
        stop("all kmers not defined")
    res <- .Call("kmer_regions_r", seq, as.integer(k), as.double(kmer.scores[ks]),
                 as.integer(min.width), as.double(min.score))
    names(res) <- c("n", "counts", "pos", "score")
    res
}

## spans enriched in frequent k-mers: score = weighted rank - thr
kmer.low.comp.regions <- function(seq, k, min.w, min.score, thr = 0.75) {
    res <- .Call("kmer_low_comp_regions", seq, as.integer(k), as.integer(min.w),
                 as.double(min.score), thr)
    names(res) <- c("n", "counts", "w.rank", "pos", "score")
    res$pos <- t(res$pos)
    res$score <- t(res$score)
    res
}

## k-mer strings in the internal A, C, T, G code order
kmer.seq <- function(k) .Call("kmer_seq_r", as.integer(k))
