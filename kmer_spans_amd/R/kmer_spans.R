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

## tr_lr regions (kmer_spans.R:88-99): params = c(k, min.length); kmers spell
## the entries of kmer.scores / trans.scores.  Returns list(kmer.scores =
## the remapped 4^k x 2 score matrix (rows in kmer.seq order),
## reg = data.frame(seq.i, beg, end, score, null)), 1-based.
lr.regions <- function(seq, params, kmers, kmer.scores, trans.scores) {
    res <- .Call("tr_lr_regions_r", seq, as.integer(params), kmers,
                 as.double(kmer.scores), as.double(trans.scores))
    names(res) <- c("kmer.scores", "pos", "scores")
    rownames(res$kmer.scores) <- kmer.seq(as.integer(params[1]))
    rownames(res$pos) <- c("seq.i", "beg", "end")
    rownames(res$scores) <- c("score", "null")
    reg <- data.frame(t(res$pos), t(res$scores))
    colnames(reg)[4:5] <- c("score", "null")
    list(kmer.scores = res$kmer.scores, reg = reg)
}

## distributions of per-window occurrence counts of the given k-mers
## (kmer_spans.R:103-118).  freq = TRUE divides dist by colSums(dist) with
## R's recycling, exactly as the reference writes it.
window.kmer.dist <- function(seq, kmers, window, freq = TRUE, ret.flag = 0L) {
    if (length(unique(nchar(kmers))) != 1)
        stop("All kmers must be of the same size")
    res <- .Call("windowed_kmer_count_distributions_r", seq, kmers,
                 nchar(kmers[1]), as.integer(window), as.integer(ret.flag))
    names(res) <- c("dist", "seq.i", "scores")
    colnames(res$dist) <- kmers
    if (!is.null(res$scores))
        for (i in seq_along(res$scores))
            colnames(res$scores[[i]]) <- kmers
    if (freq)
        res$dist <- res$dist / colSums(res$dist)
    res
}

## count k-mers of every k in a sequence file (plain or gzip FASTA, parsed on
## the GPU) into <out.prefix>counts_<k>_..._<k>.bin (kmer_spans.R:127-160).
## Returns list(seq.f, out.f or NA, seq.size, seq.fsize, seq.fl).
kmers.to.file <- function(seq.f, out.prefix, k, min.l = 1e5, magic = kmer.magic()) {
    .Call("kmers_to_file_r", as.character(seq.f), as.character(out.prefix),
          as.integer(k), as.double(min.l), as.integer(magic))
}

## read a count file written by kmers.to.file (kmer_spans.R:162-186):
## list(k, counts) or FALSE when the magic number or the k count is wrong
read.kmers <- function(fname, magic = kmer.magic()) {
    con <- file(fname, open = "rb")
    on.exit(close(con))
    if (readBin(con, "integer", n = 1) != magic)
        return(FALSE)
    nk <- readBin(con, "integer", n = 1)
    if (nk < 1)
        return(FALSE)
    lens <- readBin(con, "integer", n = nk)
    list(k = as.integer(log2(lens) / 2),
         counts = lapply(lens, function(n) readBin(con, "integer", n = n)))
}
