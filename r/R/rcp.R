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
# GPUs every step splits the regions over them, as cmclapply (R/util.R:364-382) splits them over
# cores (R/coverage.R:147-154, R/profile.R:198-199): a sample's reads are uploaded in one slice per
# GPU and redistributed so that each GPU holds only the reads its block of regions can overlap
# (rcp_shards), its coverage and profile computed there (one host thread per GPU inside the
# library); a stored $coverage list is profiled with its rows split the same way.  The shim is
# not fork-safe: these functions run in the R main process, never inside cmclapply workers.

.rcpDevices <- function() as.integer(getOption("recoup.devices", 0L))

.rcpStrandCode <- function(s) match(as.character(s), c("+", "-", "*")) - 1L

# RNGkind(sample.kind =): splitVector's bin layouts come from set.seed(42); sample(...)
.rcpRngKind <- function() as.integer(RNGkind()[3] == "Rounding")

.rcpStat <- function(stat) match(stat[1], c("mean", "median")) - 1L

.rcpInterp <- function(interpolation)
    match(interpolation[1], c("auto", "spline", "linear", "neighborhood")) - 1L

# splitBySeqname (R/util.R:1-13) + the strand filter of calcCoverage (R/coverage.R:141-144):
# the reads go to the GPU once, sorted there by (chromosome, strand, start).  `input` is what
# calcCoverage accepts (R/coverage.R:126-146): a GRanges of reads, or the per-chromosome list
# of GRanges that splitBySeqname makes (coverageAreaRef / coverageRnaRef pass that list,
# R/coverage.R:54-57,94-103): its elements are laid end to end with their merged seqinfo,
# which is what coverage() of a list element sees (the elements keep the whole seqinfo)
.rcpReadArgs <- function(input, levels = NULL) {
    if (is(input, "GRanges"))
        input <- list(input)
    input <- input[!vapply(input, is.null, TRUE)]
    if (!all(vapply(input, is, TRUE, "GRanges")))
        stop("The input argument must be a GenomicRanges object or a valid BAM/BigWig file ",
            "or a list of GenomicRanges")
    si <- if (length(input) == 0) Seqinfo() else if (length(input) == 1) seqinfo(input[[1]]) else
        Reduce(merge, lapply(unname(input), seqinfo))
    # `levels`: a code space shared with other samples (profileMatrixFromReads' one row table)
    lv <- if (is.null(levels)) seqlevels(si) else levels
    if (length(lv) == 0) # no reads and no seqlevels: one empty chromosome
        return(list(levels = ".", args = list(integer(0), integer(0), integer(0), integer(0), NA_real_)))
    # seqnames as their Rle runs (recoded into the merged levels): never one code per read
    sn <- lapply(input, function(g) {
        s <- seqnames(g)
        list(match(as.character(runValue(s)), lv) - 1L, as.numeric(runLength(s)))
    })
    chrom <- list(unlist(lapply(sn, `[[`, 1), use.names = FALSE),
        unlist(lapply(sn, `[[`, 2), use.names = FALSE))
    # IRanges holds start and width: reads of a few lengths send width runs, not an end vector
    one <- length(input) == 1
    w <- Rle(if (one) width(input[[1]]) else unlist(lapply(input, width), use.names = FALSE))
    n <- length(w)
    # reads in no particular order (recoup_test_data's are) have about one seqnames run per read:
    # then one code per read (it travels as 16-bit offsets, 2 bytes a read, not 12 a run)
    if (length(chrom[[1]]) > n %/% 4)
        chrom <- rep.int(chrom[[1]], chrom[[2]])
    else if (sum(chrom[[2]]) == 0)
        chrom <- integer(0)
    ends <- if (n > 0 && nrun(w) <= n %/% 4)
        list(as.integer(runValue(w)), as.numeric(runLength(w))) else
        if (one) end(input[[1]]) else unlist(lapply(input, end), use.names = FALSE)
    st <- if (one) start(input[[1]]) else unlist(lapply(input, start), use.names = FALSE)
    sd <- if (one) .rcpStrandCode(strand(input[[1]])) else
        unlist(lapply(input, function(g) .rcpStrandCode(strand(g))), use.names = FALSE)
    list(levels = lv, args = list(chrom, st, ends, sd, as.numeric(seqlengths(si)[lv])))
}

# A sample's reads on the GPU: an "rcpReadSet" (the library's readset as an external pointer,
# freed by .rcpFree or by the garbage collector, plus the seqlevels its chromosome codes index).
# Built once per sample by coverageBaseRef / coverageAreaRef / coverageRnaRef below, so one
# sample's reads cross PCIe once per recoup() call whatever the number of masks.  rowsOf: a
# function of the seqlevels giving the one row table the readset serves; with several devices
# the reads are then split over them for those rows (rcp_R_shards, `rows` kept in the object),
# else (no rowsOf) every device gets all of them (rcp_R_readsets, replicas).
.rcpReadSet <- function(input, strand = NULL, devices = .rcpDevices(), levels = NULL, rowsOf = NULL) {
    ra <- .rcpReadArgs(input, levels)
    sf <- if (is.null(strand)) -1L else .rcpStrandCode(strand)
    args <- c(ra$args, list(sf))
    if (length(devices) > 1 && !is.null(rowsOf)) {
        rows <- rowsOf(ra$levels)
        ptr <- do.call(.Call, c(list("rcp_R_shards"), args, .rcpRowArgs(rows), list(devices),
            list(PACKAGE = "recoup")))
        return(structure(list(ptr = ptr, levels = ra$levels, strand = strand, rows = rows),
            class = "rcpReadSet"))
    }
    ptr <- if (length(devices) > 1)
        do.call(.Call, c(list("rcp_R_readsets"), args, list(devices), list(PACKAGE = "recoup"))) else
        do.call(.Call, c(list("rcp_R_readset"), args, list(devices[1]), list(PACKAGE = "recoup")))
    structure(list(ptr = ptr, levels = ra$levels, strand = strand), class = "rcpReadSet")
}

.rcpIsReadSet <- function(x) inherits(x, "rcpReadSet")

# release the device arrays now instead of at the next garbage collection
.rcpFree <- function(rs) {
    if (.rcpIsReadSet(rs)) {
        if (!is.null(rs$rows))
            .Call("rcp_R_shards_free", rs$ptr, PACKAGE = "recoup")
        else for (p in if (is.list(rs$ptr)) rs$ptr else list(rs$ptr))
            .Call("rcp_R_free", p, PACKAGE = "recoup")
    }
    invisible(NULL)
}

# what calcCoverage reads for a sample of a recoup input list (R/coverage.R:32-39,53-62,94-97):
# its reads (strand filter, findOverlaps' ignore.strand), or its BAM file -- whose branch skips
# the strand filter (:141) and never reads ignore.strand (coverageFromBam, :228-295).
# rowsOf(levels, ignore.strand): the sample's row table (several devices: the reads split for it)
.rcpSampleReadSet <- function(x, strandedParams, rowsOf = NULL) {
    ign <- if (!is.null(x$ranges)) strandedParams$ignoreStrand else TRUE
    ro <- if (is.null(rowsOf)) NULL else function(lv) rowsOf(lv, ign)
    if (!is.null(x$ranges))
        return(list(rs = .rcpReadSet(x$ranges, strandedParams$strand, rowsOf = ro), ignore.strand = ign))
    list(rs = .rcpReadSet(.rcpReadBam(x$file), NULL, rowsOf = ro), ignore.strand = TRUE)
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

# rcp_R_coverage over a readset and a row table -> calcCoverage's named list of Rle
# (R/coverage.R:171-173; NULL where findOverlaps finds no read, the chromosome is absent or a
# subscript fails), run-length encoded on the GPU and rebuilt here without expanding it.  A
# readset split over several devices serves its own row table (rs$rows), every device at once.
# The runs also stay on the GPU(s): attr(, "rcpRuns") holds their handle and the addresses of
# the Rle vectors built here, and profileMatrix profiles them there while the list still holds
# those vectors (.rcpProfileRle) -- recoup() profiles the list coverageRef just returned
# (R/recoup.R:551-597, the forced heatmap pass :659-714), so its 12 bytes a run do not cross PCIe
# again.  options(recoup.deviceRuns = FALSE) releases them at once; otherwise the garbage
# collector does, with the list
.rcpCoverage <- function(rs, rows, names) {
    res <- if (!is.null(rs$rows)) .Call("rcp_R_shards_coverage", rs$ptr, PACKAGE = "recoup") else
        do.call(.Call, c(list("rcp_R_coverage", if (is.list(rs$ptr)) rs$ptr[[1]] else rs$ptr),
            .rcpRowArgs(rows), list(PACKAGE = "recoup")))
    cov <- lapply(seq_along(res$valid), function(r) {
        if (!res$valid[r])
            return(NULL)
        i <- seq.int(res$runOff[r] + 1, length.out = res$runOff[r + 1] - res$runOff[r])
        Rle(res$values[i], res$lengths[i])
    })
    names(cov) <- names
    if (isTRUE(getOption("recoup.deviceRuns", TRUE)))
        attr(cov, "rcpRuns") <- list(handle = res$handle,
            addr = .Call("rcp_R_rle_addresses", cov, PACKAGE = "recoup"))
    else
        .Call("rcp_R_cov_free", res$handle, PACKAGE = "recoup")
    cov
}

# calcCoverage (R/coverage.R:126-174): the named list of Rle, computed on the GPU.  `input` is
# any input the reference takes -- a GRanges of reads, splitBySeqname's per-chromosome list of
# GRanges (coverageAreaRef / coverageRnaRef, R/coverage.R:54-57,94-103), or a BAM file -- or a
# readset the caller prepared with .rcpReadSet (then `strand` must be the one it was built with)
calcCoverage <- function(input, mask, strand = NULL, ignore.strand = TRUE, rc = NULL) {
    if (!.rcpIsReadSet(input) && !is(input, "GRanges") && !is.list(input) && is.character(input)
        && !file.exists(input))
        stop("The input argument must be a GenomicRanges object or a valid ",
            "BAM/BigWig file or a list of GenomicRanges")
    if (!is(mask, "GRanges") && !is(mask, "GRangesList"))
        stop("The mask argument must be a GRanges or GRangesList object")
    own <- !.rcpIsReadSet(input)
    if (!own) {
        if (!identical(strand, input$strand))
            stop("the readset was prepared with another strand filter")
        # a readset split over several devices holds the reads of ITS row table only
        if (!is.null(input$rows) &&
            !identical(input$rows, .rcpRows(mask, input$levels, ignore.strand)))
            stop("the readset was split over the devices for another mask")
        rs <- input
    } else if (is.character(input)) {
        if (length(grep("\\.bam$", input, ignore.case = TRUE, perl = TRUE)) == 0)
            stop("recoup_amd reads BAM files; BigWig input is not on the GPU path")
        # coverageFromBam (R/coverage.R:228-295): every mapped alignment overlapping the region
        # ("keep" spans); calcCoverage skips the strand filter for a BAM (:141) and
        # coverageFromBam never reads ignore.strand
        ignore.strand <- TRUE
        rs <- .rcpReadSet(.rcpReadBam(input), NULL,
            rowsOf = function(lv) .rcpRows(mask, lv, ignore.strand))
    } else {
        # a GRanges, or a list of them; the reference's strand filter (:141-144) is the
        # readset's.  On a list the reference's input[strand(input) == strand] has no strand()
        # method to call (R/coverage.R:141-144 on splitBySeqname's plain list): an error there,
        # so one here too
        if (!is.null(strand) && !is.list(strand) && !is(input, "GRanges"))
            .rcpStrandOfListError()
        rs <- .rcpReadSet(input, strand, rowsOf = function(lv) .rcpRows(mask, lv, ignore.strand))
    }
    if (own)
        on.exit(.rcpFree(rs))
    .rcpCoverage(rs, if (is.null(rs$rows)) .rcpRows(mask, rs$levels, ignore.strand) else rs$rows, names(mask))
}

# calcCoverage's strand filter applied to a plain list (splitBySeqname's result): strand() has
# no method for "list" in GenomicRanges / BiocGenerics, so the reference stops there.  Parity
# unpinned (no fixture holds the message); recoup() never gets here, its strandedParams$strand
# is lost to argument misordering (R/argcheck.R:544-545, SURVEY Q2)
.rcpStrandOfListError <- function()
    stop("unable to find an inherited method for function 'strand' for signature '\"list\"'")

# coverageBaseRef / coverageAreaRef (R/coverage.R:26-77): per sample one readset and one
# calcCoverage over the regional ranges; coverageAreaRef's splitBySeqname (:54) is the
# readset's own chromosome index, so the reads are not split in R.  `split`: the caller is
# coverageAreaRef, whose calcCoverage gets that list -- and so cannot strand-filter it
.rcpCoverageRef <- function(input, genomeRanges, region, flank, strandedParams, split = FALSE) {
    mainRanges <- getRegionalRanges(genomeRanges, region, flank)
    names(input) <- sapply(input, function(x) return(x$id))
    for (n in names(input)) {
        message("Calculating ", region, " coverage for ", input[[n]]$name)
        if (split && !is.null(input[[n]]$ranges) && !is.null(strandedParams$strand)
            && !is.list(strandedParams$strand))
            .rcpStrandOfListError()
        s <- .rcpSampleReadSet(input[[n]], strandedParams,
            function(lv, ign) .rcpRows(mainRanges, lv, ign))
        rows <- if (is.null(s$rs$rows)) .rcpRows(mainRanges, s$rs$levels, s$ignore.strand) else s$rs$rows
        input[[n]]$coverage <- .rcpCoverage(s$rs, rows, names(mainRanges))
        .rcpFree(s$rs)
    }
    return(input)
}

coverageBaseRef <- function(input, genomeRanges, region, flank, strandedParams, rc = NULL)
    .rcpCoverageRef(input, genomeRanges, region, flank, strandedParams)

coverageAreaRef <- function(input, genomeRanges, region, flank, strandedParams, bamParams = NULL,
    rc = NULL)
    .rcpCoverageRef(input, genomeRanges, region, flank, strandedParams, split = TRUE)

# coverageRnaRef's rows (R/coverage.R:84-121): per gene c(upstream flank, the gene's exon list,
# downstream flank) as groups 0 / 1 / 2 of ONE row -- each group is one calcCoverage element
# (oriented by its own first range's strand, reads counted once per exon they overlap in the
# list group), and the row is NULL when any group is NULL, as the reference's merge is
.rcpRnaRows <- function(left, exons, right, levels, ignore.strand = TRUE) {
    G <- length(exons)
    if (length(left) != G || length(right) != G)
        stop("helperRanges and genomeRanges differ in length")
    nex <- lengths(exons)
    flat <- unlist(exons, use.names = FALSE)
    segOff <- c(0, cumsum(as.numeric(nex + 2)))
    n <- segOff[G + 1]
    first <- segOff[-(G + 1)] + 1
    last <- segOff[-1]
    isEx <- rep(TRUE, n)
    isEx[c(first, last)] <- FALSE
    code <- function(g) match(as.character(seqnames(g)), levels) - 1L
    chrom <- st <- en <- sd <- integer(n)
    grp <- rep(1L, n)
    chrom[first] <- code(left); st[first] <- start(left); en[first] <- end(left)
    sd[first] <- .rcpStrandCode(strand(left)); grp[first] <- 0L
    chrom[last] <- code(right); st[last] <- start(right); en[last] <- end(right)
    sd[last] <- .rcpStrandCode(strand(right)); grp[last] <- 2L
    chrom[isEx] <- code(flat); st[isEx] <- start(flat); en[isEx] <- end(flat)
    sd[isEx] <- .rcpStrandCode(strand(flat))
    list(segOff = segOff, chrom = chrom, start = st, end = en, strand = sd, group = grp,
        isList = c(FALSE, TRUE, FALSE, FALSE), ignoreStrand = as.logical(ignore.strand))
}

# coverageRnaRef (R/coverage.R:79-124): the three calcCoverage passes per sample (center over
# the exon lists, upstream and downstream flanks) and the per-gene c(le, ce, ri) merge become
# ONE pass over the sample's readset with 3-group rows
coverageRnaRef <- function(input, genomeRanges, helperRanges, flank,
    strandedParams = list(strand = NULL, ignoreStrand = TRUE), bamParams = NULL, rc = NULL) {
    hasCoverage <- sapply(input, function(x) is.null(x$coverage))
    if (!any(hasCoverage))
        return(input)
    # flank[1] == 0 gives 1-bp flanks on both sides: the reference tests flank[1] twice (:84-91)
    leftRanges <- getFlankingRanges(helperRanges, if (flank[1] == 0) 1 else flank[1], "upstream")
    rightRanges <- getFlankingRanges(helperRanges, if (flank[1] == 0) 1 else flank[2], "downstream")
    names(input) <- sapply(input, function(x) return(x$id))
    for (n in names(input)) {
        message("Calculating genebody coverage for ", input[[n]]$name)
        # theRanges is splitBySeqname's list (:94-95): no strand filter on it (see above)
        if (!is.null(input[[n]]$ranges) && !is.null(strandedParams$strand)
            && !is.list(strandedParams$strand))
            .rcpStrandOfListError()
        rowsOf <- function(lv, ign) .rcpRnaRows(leftRanges, genomeRanges, rightRanges, lv, ign)
        s <- .rcpSampleReadSet(input[[n]], strandedParams, rowsOf)
        rows <- if (is.null(s$rs$rows)) rowsOf(s$rs$levels, s$ignore.strand) else s$rs$rows
        input[[n]]$coverage <- .rcpCoverage(s$rs, rows, names(genomeRanges))
        .rcpFree(s$rs)
    }
    return(input)
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

# parts: where codes 0 whole, 1 center, 2 upstream, 3 downstream; nBins 0 = per base.  Several
# devices: the rows split over them (binCoverageMatrix's cmclapply over rows, R/profile.R:198-199).
# rowNames: the rownames the reference's matrix carries (NULL: none).  The shim sets the
# matrix's dimnames as the reference's rbind / cbind leave them (r/src/recoup_amd_shim.c,
# set_dimnames): rownames = rowNames, colnames "<bin>.<stat>" for binned parts, "" for per-base
# parts, none when no part is binned
# parts, where the list is still the one .rcpCoverage built: profiled from its runs on the GPU(s)
# (rcp_R_profile_cov; any element replaced -- R keeps the attribute -- or the handle released, as
# load() leaves it: the list's own vectors are uploaded instead)
.rcpProfileRle <- function(cvrg, where, flank, nBins, perBase, stat = "mean",
    interpolation = "auto", rowNames = NULL) {
    binArgs <- list(as.integer(where), as.integer(if (is.null(flank)) c(0, 0) else flank),
        as.integer(nBins), as.integer(perBase), .rcpStat(stat), .rcpInterp(interpolation),
        .rcpRngKind(), 1.0)
    h <- attr(cvrg, "rcpRuns")
    if (!is.null(h) && .Call("rcp_R_cov_alive", h$handle, PACKAGE = "recoup") &&
        identical(.Call("rcp_R_rle_addresses", cvrg, PACKAGE = "recoup"), h$addr))
        return(do.call(.Call, c(list("rcp_R_profile_cov", h$handle), binArgs,
            list(rowNames, PACKAGE = "recoup")))$profile)
    a <- .rcpRleArrays(cvrg)
    res <- do.call(.Call, c(list("rcp_R_profile_rle", a$runOff, a$values, a$lengths, a$isNull),
        binArgs, list(.rcpDevices(), rowNames, PACKAGE = "recoup")))
    res$profile
}

# binCoverageMatrix (R/profile.R:153-212): splitVector of each element (or of its
# center / upstream / downstream slice), NULL -> zeros.  The reference's rbind is named by
# names(cvrg) when it maps over cvrg itself (:159), unnamed when it maps over 1:length(cvrg)
# (the slices, :167-187)
binCoverageMatrix <- function(cvrg, binSize = 1000, stat = c("mean", "median"),
    interpolation = c("auto", "spline", "linear", "neighborhood"), flank = NULL,
    where = c("center", "upstream", "downstream"), rc = NULL) {
    w <- if (is.null(flank)) 0L else match(where[1], c("center", "upstream", "downstream"))
    .rcpProfileRle(cvrg, w, flank, binSize, 0L, stat, interpolation,
        if (is.null(flank)) names(cvrg) else NULL)
}

# baseCoverageMatrix (R/profile.R:100-151): per-base rows (whole, or the flank slices); rows
# named as binCoverageMatrix's, no colnames (as.numeric of an Rle has none)
baseCoverageMatrix <- function(cvrg, flank = NULL, where = c("upstream", "downstream"),
    rc = NULL) {
    if (is.null(flank)) {
        ok <- which(vapply(cvrg, function(x) length(x) > 0, TRUE))
        size <- if (length(ok)) length(cvrg[[ok[1]]]) else 0L
        return(.rcpProfileRle(cvrg, 0L, NULL, 0L, size, rowNames = names(cvrg)))
    }
    w <- match(where[1], c("upstream", "downstream"))
    .rcpProfileRle(cvrg, w + 1L, flank, 0L, flank[w])
}

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
        # binCoverageMatrix(binSize = 0) stops in splitVector's sample() (R/util.R:74-79)
        if (binParams$flankBinSize != 0 && fb == 0)
            stop("invalid 'size' argument")
        if (k == 1) {
            where <- c(2L, where); nb <- c(fb, nb); pb <- c(if (fb) 0L else flank[1], pb)
        } else {
            where <- c(where, 3L); nb <- c(nb, fb); pb <- c(pb, if (fb) 0L else flank[2])
        }
    }
    list(where = where, nBins = nb, perBase = pb)
}

# profileMatrix (R/profile.R:1-98), same signature and result: every sample's profile in ONE
# library call -- the unequal-length branch's upstream / center / downstream parts (three
# binCoverageMatrix or baseCoverageMatrix calls, :13-77) are one plan whose columns are their
# cbind (:78), rownames = names of the coverage list (:79).  The equal-length branch is the
# reference's own single binCoverageMatrix / baseCoverageMatrix call (:83-96), whose rows are
# named by rbind.  As in the reference, every sample is (re)profiled once any sample lacks one
profileMatrix <- function(input, flank, binParams, rc = NULL) {
    hasProfile <- sapply(input, function(x) is.null(x$profile))
    if (!any(hasProfile))
        return(input)
    len <- lengths(input[[1]]$coverage)
    len <- len[len != 0]
    equal <- all(len == len[1])
    for (n in names(input)) {
        message("Calculating profile for ", input[[n]]$name)
        cvrg <- input[[n]]$coverage
        if (equal) {
            input[[n]]$profile <- if (binParams$regionBinSize != 0)
                binCoverageMatrix(cvrg, binSize = binParams$regionBinSize,
                    stat = binParams$sumStat, rc = rc) else
                baseCoverageMatrix(cvrg, rc = rc)
            next
        }
        parts <- .rcpParts(FALSE, NA, flank, binParams)
        input[[n]]$profile <- .rcpProfileRle(cvrg, parts$where, flank, parts$nBins,
            parts$perBase, binParams$sumStat, binParams$interpolation, names(cvrg))
    }
    return(input)
}

# profileMatrix straight from the reads, for a caller that does not keep $coverage: the mask's
# rows over every sample's reads.  One GPU: all samples in ONE library call (rcp_R_profile_reads),
# one sample's upload beside the previous sample's pass and matrix download;
# several GPUs (options(recoup.devices)): each sample's rows split over them, each GPU holding
# only the reads of its rows (rcp_R_shards).
profileMatrixFromReads <- function(input, mask, flank, binParams, ignore.strand = TRUE) {
    len <- width(mask)
    equal <- all(len == len[1])
    parts <- .rcpParts(equal, len[1], flank, binParams)
    interp <- if (equal) "auto" else binParams$interpolation
    binArgs <- list(as.integer(parts$where), as.integer(if (is.null(flank)) c(0, 0) else flank),
        as.integer(parts$nBins), as.integer(parts$perBase), .rcpStat(binParams$sumStat),
        .rcpInterp(interp), .rcpRngKind(), 1.0)
    # dimnames as profileMatrix leaves them: rows named by the mask (rbind of the named coverage
    # list, or rownames<- after the cbind)
    devs <- .rcpDevices()
    todo <- which(vapply(input, function(x) is.null(x$profile), TRUE))
    # one row table for every sample: chromosome codes index the union of their seqlevels
    lv <- unique(unlist(lapply(input[todo], function(x) seqlevels(x$ranges)), use.names = FALSE))
    rows <- .rcpRows(mask, lv, ignore.strand)
    if (length(devs) > 1) {
        for (i in todo) {
            rs <- .rcpReadSet(input[[i]]$ranges, NULL, devs, lv, rowsOf = function(l) rows)
            res <- do.call(.Call, c(list("rcp_R_shards_profile", rs$ptr), binArgs,
                list(names(mask), PACKAGE = "recoup")))
            .rcpFree(rs)
            input[[i]]$profile <- res$profile
        }
        return(input)
    }
    # one GPU: every sample's reads handed over in one call, sample k + 1 uploaded while sample
    # k's matrix comes down (both PCIe directions at once)
    readArgs <- lapply(input[todo], function(x) c(.rcpReadArgs(x$ranges, lv)$args, list(-1L)))
    res <- do.call(.Call, c(list("rcp_R_profile_reads", readArgs, devs[1]), .rcpRowArgs(rows),
        binArgs, list(names(mask), PACKAGE = "recoup")))
    for (k in seq_along(todo))
        input[[todo[k]]]$profile <- res[[k]]$profile
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
