# rcp.R -- recoup's coverage -> profile hot path on the MI355X, through the .Call shim in
# r/src/recoup_amd_shim.c (C ABI: include/recoup_amd.h).  A maintainer drops this file into
# recoup's R/ and the shim into src/ (NAMESPACE: useDynLib(recoup, .registration = TRUE)); the
# functions below replace the bodies of the reference functions named in their headers and
# keep their arguments, return shapes and NULL semantics, so recoup() -- including the object
# reuse of R/recoup.R:126-135 (a stored $coverage list of Rle, re-profiled when binParams
# change) and sliceObj (R/util.R:209-210) -- is untouched.  `$coverage` stays the reference's
# object: a named list of S4Vectors::Rle (NULL where a region has no coverage), so save() /
# load() of a recoup object works as before.
#
# Devices: options(recoup.devices = c(0L, 1L, ...)) lists the GPUs (default 0).  With several
# GPUs the fused profile path splits the regions over them (one host thread per GPU inside
# the library), as cmclapply (R/util.R:364-382) splits them over cores.  The shim is not
# fork-safe: these functions run in the R main process, never inside cmclapply workers.

.rcpDevices <- function() as.integer(getOption("recoup.devices", 0L))

.rcpStrandCode <- function(s) match(as.character(s), c("+", "-", "*")) - 1L

# RNGkind(sample.kind =): splitVector's bin layouts come from set.seed(42); sample(...)
.rcpRngKind <- function() as.integer(RNGkind()[3] == "Rounding")

.rcpStat <- function(stat) match(stat[1], c("mean", "median")) - 1L

.rcpInterp <- function(interpolation)
    match(interpolation[1], c("auto", "spline", "linear", "neighborhood")) - 1L

# splitBySeqname (R/util.R:1-13) + the strand filter of calcCoverage (R/coverage.R:141-144):
# the reads go to the GPU once, sorted there by (chromosome, strand, start)
.rcpReads <- function(input, strand = NULL, devices = .rcpDevices()) {
    lv <- seqlevels(input)
    sn <- seqnames(input)  # an Rle: its runs go to the GPU, not one code per read
    # IRanges holds start and width: reads of a few lengths send width runs, not an end vector
    w <- Rle(width(input))
    ends <- if (nrun(w) <= length(input) %/% 4)
        list(as.integer(runValue(w)), as.numeric(runLength(w))) else end(input)
    args <- list(list(as.integer(runValue(sn)) - 1L, as.numeric(runLength(sn))), start(input), ends,
        .rcpStrandCode(strand(input)), as.numeric(seqlengths(input)[lv]),
        if (is.null(strand)) -1L else .rcpStrandCode(strand))
    if (length(devices) > 1)
        return(do.call(.Call, c(list("rcp_R_readsets"), args, list(devices),
            list(PACKAGE = "recoup"))))
    do.call(.Call, c(list("rcp_R_readset"), args, list(devices[1]), list(PACKAGE = "recoup")))
}

# One row per mask element: a GRanges element is one segment; a GRangesList element (the exon
# list of coverageRnaRef, R/coverage.R:79-124) its ranges, counted once per range a read hits
.rcpRows <- function(mask, levels, ignore.strand = TRUE) {
    if (is(mask, "GRangesList")) {
        flat <- unlist(mask, use.names = FALSE)
        n <- lengths(mask)
    } else {
        flat <- mask
        n <- rep(1L, length(mask))
    }
    list(segOff = c(0, cumsum(as.numeric(n))),
        chrom = match(as.character(seqnames(flat)), levels) - 1L,   # NA: chromosome absent
        start = start(flat), end = end(flat), strand = .rcpStrandCode(strand(flat)),
        group = integer(length(flat)),
        isList = c(is(mask, "GRangesList"), FALSE, FALSE, FALSE),
        ignoreStrand = as.logical(ignore.strand))
}

.rcpRowArgs <- function(rows)
    list(rows$segOff, rows$chrom, rows$start, rows$end, rows$strand, rows$group, rows$isList,
        rows$ignoreStrand)

# calcCoverage (R/coverage.R:126-174): the named list of Rle (NULL where findOverlaps finds no
# read, the chromosome is absent or the region runs past the chromosome), computed on the GPU
# and run-length encoded there
calcCoverage <- function(input, mask, strand = NULL, ignore.strand = TRUE, rc = NULL) {
    if (!is(mask, "GRanges") && !is(mask, "GRangesList"))
        stop("The mask argument must be a GRanges or GRangesList object")
    if (is.character(input) && file.exists(input)) {
        if (length(grep("\\.bam$", input, ignore.case = TRUE, perl = TRUE)) == 0)
            stop("recoup_amd reads BAM files; BigWig input is not on the GPU path")
        # coverageFromBam (R/coverage.R:228-295): every mapped alignment overlapping the region
        # ("keep" spans); calcCoverage skips the strand filter for a BAM (:141) and
        # coverageFromBam never reads ignore.strand
        input <- .rcpReadBam(input)
        strand <- NULL
        ignore.strand <- TRUE
    }
    if (!is(input, "GRanges"))
        stop("The input argument must be a GenomicRanges object or a valid BAM file")
    rs <- .rcpReads(input, strand, .rcpDevices()[1])
    rows <- .rcpRows(mask, seqlevels(input), ignore.strand)
    res <- do.call(.Call, c(list("rcp_R_coverage", rs), .rcpRowArgs(rows), list(PACKAGE = "recoup")))
    cov <- lapply(seq_along(res$valid), function(r) {
        if (!res$valid[r])
            return(NULL)
        i <- seq.int(res$runOff[r] + 1, length.out = res$runOff[r + 1] - res$runOff[r])
        Rle(res$values[i], res$lengths[i])
    })
    names(cov) <- names(mask)
    return(cov)
}

# The stored coverage list -> run arrays (runValue / runLength of every Rle element; anything
# that is not an Rle counts as NULL, as class(x) == "Rle" decides in R/profile.R)
.rcpRleArrays <- function(cvrg) {
    isNull <- !vapply(cvrg, function(x) is(x, "Rle"), TRUE)
    rv <- lapply(cvrg[!isNull], runValue)
    rl <- lapply(cvrg[!isNull], runLength)
    nr <- numeric(length(cvrg))
    nr[!isNull] <- lengths(rl)
    values <- unlist(rv, use.names = FALSE)
    values <- if (is.integer(values)) values else as.numeric(values)
    if (is.null(values)) values <- integer(0)
    list(runOff = c(0, cumsum(nr)), values = values,
        lengths = as.integer(unlist(rl, use.names = FALSE)), isNull = isNull)
}

# parts: where codes 0 whole, 1 center, 2 upstream, 3 downstream; nBins 0 = per base
.rcpProfileRle <- function(cvrg, where, flank, nBins, perBase, stat = "mean",
    interpolation = "auto") {
    a <- .rcpRleArrays(cvrg)
    res <- .Call("rcp_R_profile_rle", a$runOff, a$values, a$lengths, a$isNull,
        as.integer(where), as.integer(if (is.null(flank)) c(0, 0) else flank),
        as.integer(nBins), as.integer(perBase), .rcpStat(stat), .rcpInterp(interpolation),
        .rcpRngKind(), 1.0, .rcpDevices()[1], PACKAGE = "recoup")
    res$profile
}

# binCoverageMatrix (R/profile.R:153-212): splitVector of each element (or of its
# center / upstream / downstream slice), NULL -> zeros
binCoverageMatrix <- function(cvrg, binSize = 1000, stat = c("mean", "median"),
    interpolation = c("auto", "spline", "linear", "neighborhood"), flank = NULL,
    where = c("center", "upstream", "downstream"), rc = NULL) {
    w <- if (is.null(flank)) 0L else match(where[1], c("center", "upstream", "downstream"))
    .rcpProfileRle(cvrg, w, flank, binSize, 0L, stat, interpolation)
}

# baseCoverageMatrix (R/profile.R:100-151): per-base rows (whole, or the flank slices)
baseCoverageMatrix <- function(cvrg, flank = NULL, where = c("upstream", "downstream"),
    rc = NULL) {
    if (is.null(flank)) {
        ok <- which(vapply(cvrg, function(x) length(x) > 0, TRUE))
        size <- if (length(ok)) length(cvrg[[ok[1]]]) else 0L
        return(.rcpProfileRle(cvrg, 0L, NULL, 0L, size))
    }
    w <- match(where[1], c("upstream", "downstream"))
    .rcpProfileRle(cvrg, w + 1L, flank, 0L, flank[w])
}

# profileMatrix (R/profile.R:1-98) with every column part of a sample in ONE library call:
# the same parts, in the same order (left, center, right), as the reference's cbind
# the column parts of profileMatrix: one whole part when all rows have one length, else
# (upstream,) center (, downstream) with the flank bin counts of R/profile.R:24-60
.rcpParts <- function(equal, len1, flank, binParams) {
    if (equal)
        return(list(where = 0L, nBins = binParams$regionBinSize,
            perBase = if (binParams$regionBinSize == 0) len1 else 0L))
    where <- 1L
    nb <- binParams$regionBinSize
    pb <- 0L
    r <- flank / sum(flank)
    for (k in 1:2) {
        if (flank[k] == 0)
            next
        fb <- if (binParams$flankBinSize != 0) round(2 * binParams$flankBinSize * r[k]) else 0
        if (k == 1) {
            where <- c(2L, where); nb <- c(fb, nb); pb <- c(if (fb) 0L else flank[1], pb)
        } else {
            where <- c(where, 3L); nb <- c(nb, fb); pb <- c(pb, if (fb) 0L else flank[2])
        }
    }
    list(where = where, nBins = nb, perBase = pb)
}

profileMatrixFused <- function(input, flank, binParams, rc = NULL) {
    len <- lengths(input[[1]]$coverage)
    len <- len[len != 0]
    equal <- all(len == len[1])
    for (n in names(input)) {
        if (!is.null(input[[n]]$profile))
            next
        parts <- .rcpParts(equal, len[1], flank, binParams)
        # the equal-length branch calls binCoverageMatrix without interpolation= (its default)
        interp <- if (equal) "auto" else binParams$interpolation
        input[[n]]$profile <- .rcpProfileRle(input[[n]]$coverage, parts$where, flank,
            parts$nBins, parts$perBase, binParams$sumStat, interp)
        rownames(input[[n]]$profile) <- names(input[[n]]$coverage)
    }
    return(input)
}

# profileMatrix straight from the reads, for a caller that does not keep $coverage: the mask's
# rows over every sample's reads.  One GPU: all samples in ONE library call, passes kept two
# deep on separate HIP streams (one sample's locate and pileup tail overlap another's pileup);
# several GPUs (options(recoup.devices)): each sample's rows split over them.
profileMatrixFromReads <- function(input, mask, flank, binParams, ignore.strand = TRUE) {
    len <- width(mask)
    equal <- all(len == len[1])
    parts <- .rcpParts(equal, len[1], flank, binParams)
    interp <- if (equal) "auto" else binParams$interpolation
    rows <- .rcpRows(mask, seqlevels(input[[1]]$ranges), ignore.strand)
    binArgs <- list(as.integer(parts$where), as.integer(if (is.null(flank)) c(0, 0) else flank),
        as.integer(parts$nBins), as.integer(parts$perBase), .rcpStat(binParams$sumStat),
        .rcpInterp(interp), .rcpRngKind(), 1.0)
    devs <- .rcpDevices()
    todo <- which(vapply(input, function(x) is.null(x$profile), TRUE))
    if (length(devs) > 1) {
        for (i in todo) {
            rs <- .rcpReads(input[[i]]$ranges, NULL, devs)
            res <- do.call(.Call, c(list("rcp_R_profile_multi", rs), .rcpRowArgs(rows), binArgs,
                list(PACKAGE = "recoup")))
            input[[i]]$profile <- res$profile
            rownames(input[[i]]$profile) <- names(mask)
        }
        return(input)
    }
    rsl <- lapply(input[todo], function(x) .rcpReads(x$ranges, NULL, devs[1]))
    res <- do.call(.Call, c(list("rcp_R_profile_samples", rsl), .rcpRowArgs(rows), binArgs,
        list(2L, PACKAGE = "recoup")))
    for (k in seq_along(todo)) {
        input[[todo[k]]]$profile <- res[[k]]$profile
        rownames(input[[todo[k]]]$profile) <- names(mask)
    }
    return(input)
}

# readBam (R/ranges.R:111-146): BGZF inflated on host threads, CIGARs to reference spans
# (keep), N-split blocks (split) or quantile-filtered spans (remove), trim()med
.rcpReadBam <- function(file, spliceAction = c("keep", "remove", "split"), spliceRemoveQ = 0.75,
    threads = max(1L, parallel::detectCores() - 1L)) {
    sa <- match(spliceAction[1], c("keep", "remove", "split")) - 1L
    b <- .Call("rcp_R_read_bam", normalizePath(file), sa, as.numeric(spliceRemoveQ),
        as.integer(threads), PACKAGE = "recoup")
    GRanges(seqnames = factor(b$seqnames[b$chrom + 1L], levels = b$seqnames),
        ranges = IRanges(start = b$start, end = b$end), strand = c("+", "-")[b$strand + 1L],
        seqinfo = Seqinfo(b$seqnames, b$seqlengths))
}

# preprocessRanges normalize = "downsample" / "sampleto" (R/ranges.R:32-62):
# set.seed(seed); lapply(libSizes, function(x) sort(sample(x, size))) in R's RNG order
.rcpSampleSorted <- function(seed, libSizes, size)
    .Call("rcp_R_sample_sorted", as.integer(seed), .rcpRngKind(), as.numeric(libSizes),
        as.numeric(size), PACKAGE = "recoup")
