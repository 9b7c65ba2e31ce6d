/* recoup_amd_shim.c -- the .Call shim a recoup maintainer compiles into the R package
 * (src/ of recoup, linked with -lrecoup_amd) so that the R functions on the hot path run on the
 * MI355X through the C ABI of include/recoup_amd.h.  r/R/rcp.R holds the R side.
 *
 *   R function (reference file:line)                      .Call entry point here
 *   splitBySeqname + strand filter (R/util.R:1-13,           rcp_R_readset / rcp_R_readsets
 *       R/coverage.R:141-144)                                    (replicas) / rcp_R_shards (several
 *                                                                GPUs, the reads split for one mask)
 *   calcCoverage / coverageFromRanges (R/coverage.R:126-226) rcp_R_coverage / rcp_R_shards_coverage
 *                                                                -> list of Rle pieces
 *   binCoverageMatrix / baseCoverageMatrix / splitVector     rcp_R_profile_rle (the stored $coverage,
 *       (R/profile.R:100-212, R/util.R:15-85)                    a list of Rle, as R keeps it) /
 *                                                                rcp_R_profile_cov (its runs still on
 *                                                                the device: rcp_R_rle_addresses,
 *                                                                rcp_R_cov_alive, rcp_R_cov_free)
 *   profileMatrix straight from the reads (fused, one call   rcp_R_profile / rcp_R_profile_multi /
 *       per sample, or all samples at once; R/profile.R:1-98)   rcp_R_profile_samples / rcp_R_shards_profile /
 *                                                                rcp_R_profile_reads (reads on the host)
 *   readBam (R/ranges.R:111-146)                             rcp_R_read_bam
 *   preprocessRanges downsample / sampleto (R/ranges.R:32-62) rcp_R_sample_sorted
 *   (release a readset's / shard set's device arrays now)    rcp_R_free / rcp_R_shards_free
 *
 * Errors: every library call returns an RCP_E* code and is checked only AFTER it returned, so
 * Rf_error never longjmps through the library's C++ frames.  Memory R hands in is read in
 * place (INTEGER / REAL vectors); results are written straight into R-allocated vectors (the
 * profile matrix is R column-major, as rcp_profile writes it).  Not fork-safe: call it from the
 * R main process, not inside cmclapply's forked workers (R/util.R:364-382). */
#include <R.h>
#include <Rinternals.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "recoup_amd.h"

static void check(int rc) {
    if (rc != RCP_OK) Rf_error("recoup_amd: %s", rcp_last_error());
}

/* ------------------------------------------------------------------ reads */
static void readset_finalizer(SEXP p) {
    rcp_readset* rs = (rcp_readset*)R_ExternalPtrAddr(p);
    if (rs) {
        rcp_readset_destroy(rs);
        R_ClearExternalPtr(p);
    }
}

static void shards_finalizer(SEXP p) {
    rcp_shards* sh = (rcp_shards*)R_ExternalPtrAddr(p);
    if (sh) {
        rcp_shards_destroy(sh);
        R_ClearExternalPtr(p);
    }
}

static void cov_finalizer(SEXP p) {
    rcp_cov* c = (rcp_cov*)R_ExternalPtrAddr(p);
    if (c) {
        rcp_cov_free(c);
        R_ClearExternalPtr(p);
    }
}

static void bam_finalizer(SEXP p) {
    rcp_bam* b = (rcp_bam*)R_ExternalPtrAddr(p);
    if (b) {
        rcp_bam_free(b);
        R_ClearExternalPtr(p);
    }
}

static void rng_finalizer(SEXP p) {
    rcp_rng* g = (rcp_rng*)R_ExternalPtrAddr(p);
    if (g) {
        rcp_rng_free(g);
        R_ClearExternalPtr(p);
    }
}

/* An external pointer with a finalizer, made BEFORE the library hands out the handle it will
 * hold: the handle goes into it (R_SetExternalPtrAddr, no allocation) the moment the library
 * returns, so an R allocation failure (a longjmp) after that point can only leak to the
 * garbage collector, which runs the finalizer. */
static SEXP new_guard(R_CFinalizer_t fin) {
    SEXP p = PROTECT(R_MakeExternalPtr(NULL, R_NilValue, R_NilValue));
    R_RegisterCFinalizerEx(p, fin, TRUE);
    UNPROTECT(1);
    return p;
}

static rcp_reads_desc reads_of(SEXP chrom, SEXP start, SEXP end, SEXP strand, SEXP seqlen, SEXP sfilter) {
    R_xlen_t n = XLENGTH(start);
    int nchr = LENGTH(seqlen);
    int64_t* sl = (int64_t*)R_alloc(nchr > 0 ? nchr : 1, sizeof(int64_t));
    for (int c = 0; c < nchr; ++c) sl[c] = ISNA(REAL(seqlen)[c]) ? -1 : (int64_t)REAL(seqlen)[c];
    int8_t* st = (int8_t*)R_alloc(n > 0 ? n : 1, 1);
    for (R_xlen_t i = 0; i < n; ++i) st[i] = (int8_t)INTEGER(strand)[i];
    rcp_reads_desc d;
    memset(&d, 0, sizeof d);
    d.n = (int64_t)n;
    if (TYPEOF(chrom) == VECSXP) {
        /* list(runValue, runLength) of seqnames(reads): expanded on the GPU */
        SEXP rv = VECTOR_ELT(chrom, 0), rl = VECTOR_ELT(chrom, 1);
        int nr = LENGTH(rv);
        int64_t* len = (int64_t*)R_alloc(nr > 0 ? nr : 1, sizeof(int64_t));
        for (int k = 0; k < nr; ++k) len[k] = (int64_t)REAL(rl)[k];
        d.chrom = NULL;
        d.n_chrom_runs = nr;
        d.chrom_run_value = INTEGER(rv);
        d.chrom_run_length = len;
    } else {
        d.chrom = INTEGER(chrom);
    }
    d.start = INTEGER(start);
    if (TYPEOF(end) == VECSXP) {
        /* list(runValue, runLength) of width(reads): end = start + width - 1 formed on the GPU */
        SEXP wv = VECTOR_ELT(end, 0), wl = VECTOR_ELT(end, 1);
        int nw = LENGTH(wv);
        int64_t* wlen = (int64_t*)R_alloc(nw > 0 ? nw : 1, sizeof(int64_t));
        for (int k = 0; k < nw; ++k) wlen[k] = (int64_t)REAL(wl)[k];
        d.end = NULL;
        d.n_width_runs = nw;
        d.width_run_value = INTEGER(wv);
        d.width_run_length = wlen;
    } else {
        d.end = INTEGER(end);
    }
    d.strand = st;
    d.n_chrom = nchr;
    d.seqlen = sl;
    d.device = 0;
    d.on_device = 0;
    d.strand_filter = asInteger(sfilter);
    return d;
}

/* .Call("rcp_R_readset", chromCode, start, end, strandCode, seqlengths, strandFilter, device)
 * chromCode: 0-based seqlevel index per read, or list(runValue - 1L, as.numeric(runLength)) of
 * the seqnames Rle; end: per read, or list(runValue, as.numeric(runLength)) of the width Rle;
 * strandCode 0 '+', 1 '-', 2 '*'; seqlengths numeric (NA ok) */
SEXP rcp_R_readset(SEXP chrom, SEXP start, SEXP end, SEXP strand, SEXP seqlen, SEXP sfilter, SEXP dev) {
    rcp_reads_desc d = reads_of(chrom, start, end, strand, seqlen, sfilter);
    d.device = asInteger(dev);
    SEXP p = PROTECT(new_guard(readset_finalizer));
    rcp_readset* rs = NULL;
    int rc = rcp_readset_create(&d, NULL, &rs);
    R_SetExternalPtrAddr(p, rs);
    check(rc);
    UNPROTECT(1);
    return p;
}

/* .Call("rcp_R_readsets", <as rcp_R_readset>, devices) -> list of readsets, one per GPU */
SEXP rcp_R_readsets(SEXP chrom, SEXP start, SEXP end, SEXP strand, SEXP seqlen, SEXP sfilter, SEXP devs) {
    rcp_reads_desc d = reads_of(chrom, start, end, strand, seqlen, sfilter);
    int nd = LENGTH(devs);
    rcp_readset** rs = (rcp_readset**)R_alloc(nd > 0 ? nd : 1, sizeof(rcp_readset*));
    SEXP res = PROTECT(allocVector(VECSXP, nd));
    for (int i = 0; i < nd; ++i) {
        rs[i] = NULL;
        SET_VECTOR_ELT(res, i, new_guard(readset_finalizer));
    }
    int rc = rcp_readset_create_multi(&d, INTEGER(devs), nd, rs);
    for (int i = 0; i < nd; ++i) R_SetExternalPtrAddr(VECTOR_ELT(res, i), rc == RCP_OK ? rs[i] : NULL);
    check(rc);
    UNPROTECT(1);
    return res;
}

/* .Call("rcp_R_free", readset) releases a readset's device arrays now (the finalizer then finds
 * nothing to do) */
SEXP rcp_R_free(SEXP p) {
    readset_finalizer(p);
    return R_NilValue;
}

/* ------------------------------------------------------------------ rows / bins */
/* rows: segOff (numeric, n_rows + 1), chrom (0-based, NA = absent chromosome), start, end,
 * strand, group (0..3 per segment), isList (logical[4]), ignoreStrand (logical) */
static rcp_rows_desc rows_of(SEXP segOff, SEXP chrom, SEXP start, SEXP end, SEXP strand, SEXP group,
                             SEXP isList, SEXP ignoreStrand) {
    int nseg = LENGTH(start), nrow = LENGTH(segOff) - 1;
    int64_t* off = (int64_t*)R_alloc(nrow + 1, sizeof(int64_t));
    for (int r = 0; r <= nrow; ++r) off[r] = (int64_t)REAL(segOff)[r];
    int8_t* st = (int8_t*)R_alloc(nseg > 0 ? nseg : 1, 1);
    int8_t* gr = (int8_t*)R_alloc(nseg > 0 ? nseg : 1, 1);
    int32_t* ch = (int32_t*)R_alloc(nseg > 0 ? nseg : 1, sizeof(int32_t));
    for (int i = 0; i < nseg; ++i) {
        st[i] = (int8_t)INTEGER(strand)[i];
        gr[i] = (int8_t)INTEGER(group)[i];
        ch[i] = INTEGER(chrom)[i] == NA_INTEGER ? -1 : INTEGER(chrom)[i];
    }
    uint8_t* il = (uint8_t*)R_alloc(4, 1);
    for (int g = 0; g < 4; ++g) il[g] = (uint8_t)(g < LENGTH(isList) ? LOGICAL(isList)[g] : 0);
    rcp_rows_desc rd;
    memset(&rd, 0, sizeof rd);
    rd.n_rows = nrow;
    rd.seg_off = off;
    rd.seg_chrom = ch;
    rd.seg_start = INTEGER(start);
    rd.seg_end = INTEGER(end);
    rd.seg_strand = st;
    rd.seg_group = gr;
    rd.group_is_list = il;
    rd.ignore_strand = asLogical(ignoreStrand);
    return rd;
}

/* .Call("rcp_R_shards", <reads: 6 args as rcp_R_readset>, <rows: 8 args>, devices) -> the reads
 * split over several GPUs for ONE row table (rcp_shards_create): each GPU keeps only the reads
 * its block of the rows can overlap -- what cmclapply over the regions parallelises
 * (R/coverage.R:147-154, R/profile.R:198-199) */
SEXP rcp_R_shards(SEXP chrom, SEXP start, SEXP end, SEXP strand, SEXP seqlen, SEXP sfilter, SEXP segOff,
                  SEXP rchrom, SEXP rstart, SEXP rend, SEXP rstrand, SEXP group, SEXP isList, SEXP ignoreStrand,
                  SEXP devs) {
    rcp_reads_desc d = reads_of(chrom, start, end, strand, seqlen, sfilter);
    rcp_rows_desc rd = rows_of(segOff, rchrom, rstart, rend, rstrand, group, isList, ignoreStrand);
    SEXP p = PROTECT(new_guard(shards_finalizer));
    rcp_shards* sh = NULL;
    int rc = rcp_shards_create(&d, &rd, INTEGER(devs), LENGTH(devs), &sh);
    R_SetExternalPtrAddr(p, sh);
    check(rc);
    UNPROTECT(1);
    return p;
}

/* .Call("rcp_R_shards_free", shards) releases a shard set's device arrays now */
SEXP rcp_R_shards_free(SEXP p) {
    shards_finalizer(p);
    return R_NilValue;
}

/* bins: where (RCP_WHERE_* per part), flank (2 ints), nBins (per part, 0 = per base),
 * perBaseWidth (per part), stat (0 mean / 1 median), interp (0 auto .. 3 neighborhood),
 * rngKind (0 Rejection / 1 Rounding: RNGkind()[3]), scale (linear factor) */
static rcp_bins_desc bins_of(SEXP where, SEXP flank, SEXP nBins, SEXP pbw, SEXP stat, SEXP interp, SEXP rng,
                             SEXP scale, int* ncol) {
    rcp_bins_desc bd;
    memset(&bd, 0, sizeof bd);
    bd.n_parts = LENGTH(where);
    bd.where = INTEGER(where);
    bd.flank[0] = INTEGER(flank)[0];
    bd.flank[1] = INTEGER(flank)[1];
    bd.n_bins = INTEGER(nBins);
    bd.per_base_width = INTEGER(pbw);
    bd.stat = asInteger(stat);
    bd.interp = asInteger(interp);
    bd.rng_kind = asInteger(rng);
    bd.scale = asReal(scale);
    *ncol = 0;
    for (int p = 0; p < bd.n_parts; ++p) *ncol += INTEGER(nBins)[p] ? INTEGER(nBins)[p] : INTEGER(pbw)[p];
    return bd;
}

/* The dimnames the reference's profile matrices carry (R/profile.R:112-115,150,159-162,198-208):
 * rbind of a NAMED list gives rownames = the list's names (the caller passes names(cvrg), or NULL
 * where the reference's cmclapply runs over 1:length(cvrg) and the rows come back unnamed);
 * a binned row is unlist(llply(split(x, f), stat)), whose names are "<bin>.<stat>" -- llply
 * names each bin by its factor level "1".."n", and plyr::each, which llply applies to a
 * function given by name, names a length-1 result by that name -- while a per-base row
 * (as.numeric of an Rle) has none.  cbind of the parts (R/profile.R:78) keeps each part's
 * colnames, "" for a part without them; no binned part -> no colnames at all. */
static void set_dimnames(SEXP mat, SEXP rowNames, const rcp_bins_desc* bd, int nrow, int ncol) {
    SEXP rn = R_NilValue, cn = R_NilValue;
    int nprot = 0;
    if (TYPEOF(rowNames) == STRSXP && XLENGTH(rowNames) == nrow) rn = rowNames;
    int binned = 0;
    for (int p = 0; p < bd->n_parts; ++p) binned |= bd->n_bins[p] != 0;
    if (binned) {
        const char* stat = bd->stat == RCP_STAT_MEDIAN ? "median" : "mean";
        cn = PROTECT(allocVector(STRSXP, ncol));
        ++nprot;
        int c = 0;
        char buf[64];
        for (int p = 0; p < bd->n_parts; ++p) {
            int nb = bd->n_bins[p], w = nb ? nb : bd->per_base_width[p];
            for (int k = 1; k <= w; ++k, ++c) {
                if (nb) snprintf(buf, sizeof buf, "%d.%s", k, stat);
                else buf[0] = 0;
                SET_STRING_ELT(cn, c, mkChar(buf));
            }
        }
    }
    if (rn != R_NilValue || cn != R_NilValue) {
        SEXP dn = PROTECT(allocVector(VECSXP, 2));
        ++nprot;
        SET_VECTOR_ELT(dn, 0, rn);
        SET_VECTOR_ELT(dn, 1, cn);
        setAttrib(mat, R_DimNamesSymbol, dn);
    }
    UNPROTECT(nprot);
}

static SEXP profile_result(SEXP mat, const uint8_t* valid, int nrow) {
    SEXP v = PROTECT(allocVector(LGLSXP, nrow));
    for (int r = 0; r < nrow; ++r) LOGICAL(v)[r] = valid[r];
    SEXP res = PROTECT(allocVector(VECSXP, 2));
    SET_VECTOR_ELT(res, 0, mat);
    SET_VECTOR_ELT(res, 1, v);
    SEXP nm = PROTECT(allocVector(STRSXP, 2));
    SET_STRING_ELT(nm, 0, mkChar("profile"));
    SET_STRING_ELT(nm, 1, mkChar("valid"));
    setAttrib(res, R_NamesSymbol, nm);
    UNPROTECT(3);
    return res;
}

/* ------------------------------------------------------------------ profiles */
/* .Call("rcp_R_profile", readset, <rows: 8 args>, <bins: 8 args>, rowNames)
 * -> list(profile = n_rows x n_cols double matrix with the reference's dimnames, valid = logical) */
SEXP rcp_R_profile(SEXP rsp, SEXP segOff, SEXP chrom, SEXP start, SEXP end, SEXP strand, SEXP group,
                   SEXP isList, SEXP ignoreStrand, SEXP where, SEXP flank, SEXP nBins, SEXP pbw, SEXP stat,
                   SEXP interp, SEXP rng, SEXP scale, SEXP rowNames) {
    rcp_rows_desc rd = rows_of(segOff, chrom, start, end, strand, group, isList, ignoreStrand);
    int ncol = 0;
    rcp_bins_desc bd = bins_of(where, flank, nBins, pbw, stat, interp, rng, scale, &ncol);
    SEXP out = PROTECT(allocMatrix(REALSXP, rd.n_rows, ncol)); /* R column-major, filled in place */
    uint8_t* valid = (uint8_t*)R_alloc(rd.n_rows ? rd.n_rows : 1, 1);
    int rc = rcp_profile((const rcp_readset*)R_ExternalPtrAddr(rsp), &rd, &bd, REAL(out), valid);
    if (rc != RCP_OK) {
        UNPROTECT(1);
        check(rc);
    }
    set_dimnames(out, rowNames, &bd, rd.n_rows, ncol);
    SEXP res = profile_result(out, valid, rd.n_rows);
    UNPROTECT(1);
    return res;
}

/* .Call("rcp_R_profile_samples", list of readsets (one per sample, one GPU), <rows: 8 args>,
 * <bins: 8 args>, inflight, rowNames) -> list (per sample) of list(profile, valid): profileMatrix's loop
 * over the samples of a recoup input list (R/profile.R:13-98) in one call, passes kept
 * `inflight` deep on separate HIP streams */
SEXP rcp_R_profile_samples(SEXP rsl, SEXP segOff, SEXP chrom, SEXP start, SEXP end, SEXP strand, SEXP group,
                           SEXP isList, SEXP ignoreStrand, SEXP where, SEXP flank, SEXP nBins, SEXP pbw,
                           SEXP stat, SEXP interp, SEXP rng, SEXP scale, SEXP inflight, SEXP rowNames) {
    rcp_rows_desc rd = rows_of(segOff, chrom, start, end, strand, group, isList, ignoreStrand);
    int ncol = 0;
    rcp_bins_desc bd = bins_of(where, flank, nBins, pbw, stat, interp, rng, scale, &ncol);
    int ns = LENGTH(rsl);
    rcp_readset** rs = (rcp_readset**)R_alloc(ns > 0 ? ns : 1, sizeof(rcp_readset*));
    double** outs = (double**)R_alloc(ns > 0 ? ns : 1, sizeof(double*));
    uint8_t** valid = (uint8_t**)R_alloc(ns > 0 ? ns : 1, sizeof(uint8_t*));
    SEXP mats = PROTECT(allocVector(VECSXP, ns));
    for (int i = 0; i < ns; ++i) {
        rs[i] = (rcp_readset*)R_ExternalPtrAddr(VECTOR_ELT(rsl, i));
        SET_VECTOR_ELT(mats, i, allocMatrix(REALSXP, rd.n_rows, ncol));
        outs[i] = REAL(VECTOR_ELT(mats, i));
        valid[i] = (uint8_t*)R_alloc(rd.n_rows ? rd.n_rows : 1, 1);
    }
    int rc = rcp_profile_samples(rs, ns, &rd, &bd, asInteger(inflight), outs, valid);
    if (rc != RCP_OK) {
        UNPROTECT(1);
        check(rc);
    }
    SEXP res = PROTECT(allocVector(VECSXP, ns));
    for (int i = 0; i < ns; ++i) {
        set_dimnames(VECTOR_ELT(mats, i), rowNames, &bd, rd.n_rows, ncol);
        SET_VECTOR_ELT(res, i, profile_result(VECTOR_ELT(mats, i), valid[i], rd.n_rows));
    }
    UNPROTECT(2);
    return res;
}

/* .Call("rcp_R_profile_reads", list of samples' read args (each list(<reads: 6 args as
 * rcp_R_readset>)), device, <rows: 8 args>, <bins: 8 args>, rowNames) -> list (per sample) of
 * list(profile, valid): profileMatrix straight from the reads of an input list on one GPU, sample
 * k + 1's reads uploaded while sample k's matrix comes down (rcp_profile_reads) */
SEXP rcp_R_profile_reads(SEXP readsList, SEXP dev, SEXP segOff, SEXP chrom, SEXP start, SEXP end, SEXP strand,
                         SEXP group, SEXP isList, SEXP ignoreStrand, SEXP where, SEXP flank, SEXP nBins, SEXP pbw,
                         SEXP stat, SEXP interp, SEXP rng, SEXP scale, SEXP rowNames) {
    rcp_rows_desc rd = rows_of(segOff, chrom, start, end, strand, group, isList, ignoreStrand);
    int ncol = 0;
    rcp_bins_desc bd = bins_of(where, flank, nBins, pbw, stat, interp, rng, scale, &ncol);
    int ns = LENGTH(readsList);
    rcp_reads_desc* rds = (rcp_reads_desc*)R_alloc(ns > 0 ? ns : 1, sizeof(rcp_reads_desc));
    double** outs = (double**)R_alloc(ns > 0 ? ns : 1, sizeof(double*));
    uint8_t** valid = (uint8_t**)R_alloc(ns > 0 ? ns : 1, sizeof(uint8_t*));
    SEXP mats = PROTECT(allocVector(VECSXP, ns));
    for (int i = 0; i < ns; ++i) {
        SEXP a = VECTOR_ELT(readsList, i);
        rds[i] = reads_of(VECTOR_ELT(a, 0), VECTOR_ELT(a, 1), VECTOR_ELT(a, 2), VECTOR_ELT(a, 3), VECTOR_ELT(a, 4),
                          VECTOR_ELT(a, 5));
        rds[i].device = asInteger(dev);
        SET_VECTOR_ELT(mats, i, allocMatrix(REALSXP, rd.n_rows, ncol));
        outs[i] = REAL(VECTOR_ELT(mats, i));
        valid[i] = (uint8_t*)R_alloc(rd.n_rows ? rd.n_rows : 1, 1);
    }
    int rc = rcp_profile_reads(rds, ns, &rd, &bd, outs, valid);
    if (rc != RCP_OK) {
        UNPROTECT(1);
        check(rc);
    }
    SEXP res = PROTECT(allocVector(VECSXP, ns));
    for (int i = 0; i < ns; ++i) {
        set_dimnames(VECTOR_ELT(mats, i), rowNames, &bd, rd.n_rows, ncol);
        SET_VECTOR_ELT(res, i, profile_result(VECTOR_ELT(mats, i), valid[i], rd.n_rows));
    }
    UNPROTECT(2);
    return res;
}

/* .Call("rcp_R_profile_multi", list of readsets (one per GPU, rcp_R_readsets), <rows>, <bins>, rowNames):
 * row blocks on every GPU at once (the reference's cmclapply over regions) */
SEXP rcp_R_profile_multi(SEXP rsl, SEXP segOff, SEXP chrom, SEXP start, SEXP end, SEXP strand, SEXP group,
                         SEXP isList, SEXP ignoreStrand, SEXP where, SEXP flank, SEXP nBins, SEXP pbw,
                         SEXP stat, SEXP interp, SEXP rng, SEXP scale, SEXP rowNames) {
    rcp_rows_desc rd = rows_of(segOff, chrom, start, end, strand, group, isList, ignoreStrand);
    int ncol = 0;
    rcp_bins_desc bd = bins_of(where, flank, nBins, pbw, stat, interp, rng, scale, &ncol);
    int nd = LENGTH(rsl);
    rcp_readset** rs = (rcp_readset**)R_alloc(nd > 0 ? nd : 1, sizeof(rcp_readset*));
    for (int i = 0; i < nd; ++i) rs[i] = (rcp_readset*)R_ExternalPtrAddr(VECTOR_ELT(rsl, i));
    SEXP out = PROTECT(allocMatrix(REALSXP, rd.n_rows, ncol));
    uint8_t* valid = (uint8_t*)R_alloc(rd.n_rows ? rd.n_rows : 1, 1);
    int rc = rcp_profile_multi(rs, nd, &rd, &bd, REAL(out), valid, NULL);
    if (rc != RCP_OK) {
        UNPROTECT(1);
        check(rc);
    }
    set_dimnames(out, rowNames, &bd, rd.n_rows, ncol);
    SEXP res = profile_result(out, valid, rd.n_rows);
    UNPROTECT(1);
    return res;
}

/* .Call("rcp_R_shards_profile", shards, <bins: 8 args>, rowNames) -> list(profile, valid): the
 * shard set's row table profiled on every GPU at once, each writing its rows of the matrix */
SEXP rcp_R_shards_profile(SEXP shp, SEXP where, SEXP flank, SEXP nBins, SEXP pbw, SEXP stat, SEXP interp, SEXP rng,
                          SEXP scale, SEXP rowNames) {
    rcp_shards* sh = (rcp_shards*)R_ExternalPtrAddr(shp);
    int ncol = 0;
    rcp_bins_desc bd = bins_of(where, flank, nBins, pbw, stat, interp, rng, scale, &ncol);
    int32_t nrow = 0;
    check(rcp_shards_info(sh, &nrow, NULL, NULL, NULL));
    SEXP out = PROTECT(allocMatrix(REALSXP, nrow, ncol));
    uint8_t* valid = (uint8_t*)R_alloc(nrow ? nrow : 1, 1);
    int rc = rcp_shards_profile(sh, &bd, REAL(out), valid);
    if (rc != RCP_OK) {
        UNPROTECT(1);
        check(rc);
    }
    set_dimnames(out, rowNames, &bd, nrow, ncol);
    SEXP res = profile_result(out, valid, nrow);
    UNPROTECT(1);
    return res;
}

/* .Call("rcp_R_profile_rle", runOff (numeric, n_rows + 1), values (integer or double),
 *       lengths (integer), isNull (logical), <bins: 8 args>, devices, rowNames): devices of
 *       length > 1 split the rows over several GPUs (rcp_profile_rle_multi)
 * binCoverageMatrix / baseCoverageMatrix of the stored coverage list (list of Rle flattened
 * by .rcpRleArrays); -> list(profile, valid) */
SEXP rcp_R_profile_rle(SEXP runOff, SEXP values, SEXP lengths, SEXP isNull, SEXP where, SEXP flank, SEXP nBins,
                       SEXP pbw, SEXP stat, SEXP interp, SEXP rng, SEXP scale, SEXP dev, SEXP rowNames) {
    int nrow = LENGTH(runOff) - 1;
    int64_t* off = (int64_t*)R_alloc(nrow + 1, sizeof(int64_t));
    for (int r = 0; r <= nrow; ++r) off[r] = (int64_t)REAL(runOff)[r];
    uint8_t* nul = (uint8_t*)R_alloc(nrow > 0 ? nrow : 1, 1);
    for (int r = 0; r < nrow; ++r) nul[r] = (uint8_t)(LOGICAL(isNull)[r] != 0);
    rcp_rle_desc cd;
    memset(&cd, 0, sizeof cd);
    cd.n_rows = nrow;
    cd.run_off = off;
    cd.lengths = INTEGER(lengths);
    if (TYPEOF(values) == INTSXP) cd.ivalues = INTEGER(values);
    else cd.dvalues = REAL(values);
    cd.is_null = nul;
    int ncol = 0;
    rcp_bins_desc bd = bins_of(where, flank, nBins, pbw, stat, interp, rng, scale, &ncol);
    SEXP out = PROTECT(allocMatrix(REALSXP, nrow, ncol));
    uint8_t* valid = (uint8_t*)R_alloc(nrow ? nrow : 1, 1);
    int rc = LENGTH(dev) > 1 ? rcp_profile_rle_multi(&cd, &bd, INTEGER(dev), LENGTH(dev), REAL(out), valid)
                             : rcp_profile_rle(&cd, &bd, asInteger(dev), REAL(out), valid);
    if (rc != RCP_OK) {
        UNPROTECT(1);
        check(rc);
    }
    set_dimnames(out, rowNames, &bd, nrow, ncol);
    SEXP res = profile_result(out, valid, nrow);
    UNPROTECT(1);
    return res;
}

/* ------------------------------------------------------------------ coverage */
/* .Call("rcp_R_coverage", readset, <rows: 8 args>)
 * -> list(runOff = numeric n_rows + 1, values = integer, lengths = integer, valid = logical,
 *         handle = external pointer): the pieces of calcCoverage's named list of Rle
 * (R/coverage.R:171-173), from which the R side builds S4Vectors::Rle(values, lengths) per valid
 * row without expanding it, and the handle that keeps the same runs on the device (released by
 * rcp_R_cov_free or the garbage collector): while the list is unchanged, profileMatrix profiles
 * them there (rcp_R_profile_cov) instead of uploading its Rle vectors again */
/* The Rle pieces of a coverage handle held by `guard` (kept: the result's `handle`) */
static SEXP coverage_result(SEXP guard, rcp_cov* cov) {
    int32_t nrow = 0;
    int64_t nruns = 0;
    check(rcp_cov_info(cov, &nrow, &nruns));
    SEXP off = PROTECT(allocVector(REALSXP, nrow + 1));
    SEXP val = PROTECT(allocVector(INTSXP, (R_xlen_t)nruns));
    SEXP len = PROTECT(allocVector(INTSXP, (R_xlen_t)nruns));
    SEXP ok = PROTECT(allocVector(LGLSXP, nrow));
    int64_t* o64 = (int64_t*)R_alloc(nrow + 1, sizeof(int64_t));
    uint8_t* v8 = (uint8_t*)R_alloc(nrow > 0 ? nrow : 1, 1);
    int rc = rcp_cov_copy(cov, o64, INTEGER(val), INTEGER(len), v8);
    if (rc != RCP_OK) cov_finalizer(guard); /* (nothing to keep) */
    check(rc);
    for (int r = 0; r <= nrow; ++r) REAL(off)[r] = (double)o64[r];
    for (int r = 0; r < nrow; ++r) LOGICAL(ok)[r] = v8[r];
    SEXP res = PROTECT(allocVector(VECSXP, 5));
    SET_VECTOR_ELT(res, 0, off);
    SET_VECTOR_ELT(res, 1, val);
    SET_VECTOR_ELT(res, 2, len);
    SET_VECTOR_ELT(res, 3, ok);
    SET_VECTOR_ELT(res, 4, guard);
    SEXP nm = PROTECT(allocVector(STRSXP, 5));
    SET_STRING_ELT(nm, 0, mkChar("runOff"));
    SET_STRING_ELT(nm, 1, mkChar("values"));
    SET_STRING_ELT(nm, 2, mkChar("lengths"));
    SET_STRING_ELT(nm, 3, mkChar("valid"));
    SET_STRING_ELT(nm, 4, mkChar("handle"));
    setAttrib(res, R_NamesSymbol, nm);
    UNPROTECT(6);
    return res;
}

/* .Call("rcp_R_rle_addresses", list) -> numeric 2 n: for element i, the addresses of its
 * "values" and "lengths" slot vectors when it is an S4 object with both (an S4Vectors::Rle), else
 * 0, 0.  R replaces a modified vector (copy on modify) and builds a new Rle for any operation on
 * one (runValue<-, arithmetic, a linear rescale), so equal addresses mean the list still holds
 * the runs it was built from -- read in C: runValue() per element would be an S4 dispatch each */
SEXP rcp_R_rle_addresses(SEXP list) {
    R_xlen_t n = TYPEOF(list) == VECSXP ? XLENGTH(list) : 0;
    SEXP out = PROTECT(allocVector(REALSXP, 2 * n));
    SEXP vs = PROTECT(install("values")), ls = PROTECT(install("lengths"));
    for (R_xlen_t i = 0; i < n; ++i) {
        SEXP x = VECTOR_ELT(list, i);
        double a = 0.0, b = 0.0;
        if (IS_S4_OBJECT(x) && R_has_slot(x, vs) && R_has_slot(x, ls)) {
            a = (double)(uintptr_t)R_do_slot(x, vs);
            b = (double)(uintptr_t)R_do_slot(x, ls);
        }
        REAL(out)[2 * i] = a;
        REAL(out)[2 * i + 1] = b;
    }
    UNPROTECT(3);
    return out;
}

/* .Call("rcp_R_cov_alive", handle) -> TRUE while the handle holds its device runs (FALSE once
 * freed, or after save() / load(): R restores an external pointer as NULL) */
SEXP rcp_R_cov_alive(SEXP p) {
    SEXP out = PROTECT(allocVector(LGLSXP, 1));
    LOGICAL(out)[0] = TYPEOF(p) == EXTPTRSXP && R_ExternalPtrAddr(p) != NULL;
    UNPROTECT(1);
    return out;
}

/* .Call("rcp_R_cov_free", handle): release the device runs now */
SEXP rcp_R_cov_free(SEXP p) {
    cov_finalizer(p);
    return R_NilValue;
}

/* .Call("rcp_R_profile_cov", handle, <bins: 8 args>, rowNames) -> list(profile, valid):
 * rcp_R_profile_rle of the runs the handle keeps on the device(s) (rcp_profile_cov) */
SEXP rcp_R_profile_cov(SEXP p, SEXP where, SEXP flank, SEXP nBins, SEXP pbw, SEXP stat, SEXP interp, SEXP rng,
                       SEXP scale, SEXP rowNames) {
    rcp_cov* cov = (rcp_cov*)R_ExternalPtrAddr(p);
    if (!cov) Rf_error("recoup_amd: the coverage handle was released");
    int32_t nrow = 0;
    check(rcp_cov_info(cov, &nrow, NULL));
    int ncol = 0;
    rcp_bins_desc bd = bins_of(where, flank, nBins, pbw, stat, interp, rng, scale, &ncol);
    SEXP out = PROTECT(allocMatrix(REALSXP, nrow, ncol));
    uint8_t* valid = (uint8_t*)R_alloc(nrow ? nrow : 1, 1);
    int rc = rcp_profile_cov(cov, &bd, REAL(out), valid);
    if (rc != RCP_OK) {
        UNPROTECT(1);
        check(rc);
    }
    set_dimnames(out, rowNames, &bd, nrow, ncol);
    SEXP res = profile_result(out, valid, nrow);
    UNPROTECT(1);
    return res;
}

SEXP rcp_R_coverage(SEXP rsp, SEXP segOff, SEXP chrom, SEXP start, SEXP end, SEXP strand, SEXP group,
                    SEXP isList, SEXP ignoreStrand) {
    rcp_rows_desc rd = rows_of(segOff, chrom, start, end, strand, group, isList, ignoreStrand);
    SEXP guard = PROTECT(new_guard(cov_finalizer));
    rcp_cov* cov = NULL;
    int rc = rcp_coverage_rle((const rcp_readset*)R_ExternalPtrAddr(rsp), &rd, &cov);
    R_SetExternalPtrAddr(guard, cov);
    check(rc);
    SEXP res = coverage_result(guard, cov);
    UNPROTECT(1);
    return res;
}

/* .Call("rcp_R_shards_coverage", shards) -> as rcp_R_coverage, for the shard set's row table:
 * every GPU's block of rows at once (calcCoverage's cmclapply over regions, R/coverage.R:147-154) */
SEXP rcp_R_shards_coverage(SEXP shp) {
    SEXP guard = PROTECT(new_guard(cov_finalizer));
    rcp_cov* cov = NULL;
    int rc = rcp_shards_coverage((rcp_shards*)R_ExternalPtrAddr(shp), &cov);
    R_SetExternalPtrAddr(guard, cov);
    check(rc);
    SEXP res = coverage_result(guard, cov);
    UNPROTECT(1);
    return res;
}

/* ------------------------------------------------------------------ BAM, RNG */
/* .Call("rcp_R_read_bam", path, spliceAction (0 keep / 1 remove / 2 split), removeQ, threads)
 * -> list(seqnames = character, seqlengths = numeric, chrom = integer (0-based), start, end,
 *         strand = integer (0 '+', 1 '-')) */
SEXP rcp_R_read_bam(SEXP path, SEXP splice, SEXP q, SEXP threads) {
    SEXP guard = PROTECT(new_guard(bam_finalizer));
    rcp_bam* bam = NULL;
    int rc = rcp_bam_read(CHAR(STRING_ELT(path, 0)), asInteger(splice), asReal(q), asInteger(threads), &bam);
    R_SetExternalPtrAddr(guard, bam);
    check(rc);
    int64_t n = 0, nal = 0;
    int32_t nref = 0;
    check(rcp_bam_info(bam, &n, &nref, &nal));
    SEXP nm = PROTECT(allocVector(STRSXP, nref));
    for (int32_t i = 0; i < nref; ++i) SET_STRING_ELT(nm, i, mkChar(rcp_bam_ref_name(bam, i)));
    SEXP sl = PROTECT(allocVector(REALSXP, nref));
    SEXP ch = PROTECT(allocVector(INTSXP, (R_xlen_t)n));
    SEXP st = PROTECT(allocVector(INTSXP, (R_xlen_t)n));
    SEXP en = PROTECT(allocVector(INTSXP, (R_xlen_t)n));
    SEXP sd = PROTECT(allocVector(INTSXP, (R_xlen_t)n));
    int64_t* rl = (int64_t*)R_alloc(nref > 0 ? nref : 1, sizeof(int64_t));
    int8_t* s8 = (int8_t*)R_alloc(n > 0 ? (size_t)n : 1, 1);
    rc = rcp_bam_copy(bam, rl, INTEGER(ch), INTEGER(st), INTEGER(en), s8);
    bam_finalizer(guard);
    check(rc);
    for (int32_t i = 0; i < nref; ++i) REAL(sl)[i] = (double)rl[i];
    for (int64_t i = 0; i < n; ++i) INTEGER(sd)[i] = s8[i];
    SEXP res = PROTECT(allocVector(VECSXP, 6));
    SEXP names = PROTECT(allocVector(STRSXP, 6));
    const char* keys[6] = {"seqnames", "seqlengths", "chrom", "start", "end", "strand"};
    SEXP vals[6] = {nm, sl, ch, st, en, sd};
    for (int k = 0; k < 6; ++k) {
        SET_VECTOR_ELT(res, k, vals[k]);
        SET_STRING_ELT(names, k, mkChar(keys[k]));
    }
    setAttrib(res, R_NamesSymbol, names);
    UNPROTECT(9);
    return res;
}

/* .Call("rcp_R_sample_sorted", seed, kind, libSizes (numeric), size)
 * set.seed(seed); lapply(libSizes, function(x) sort(sample(x, size))) in R's RNG stream order
 * (R/ranges.R:32-62) -> list of 1-based read indices (numeric) */
SEXP rcp_R_sample_sorted(SEXP seed, SEXP kind, SEXP libSizes, SEXP size) {
    SEXP guard = PROTECT(new_guard(rng_finalizer));
    rcp_rng* g = NULL;
    int rc = rcp_rng_create((uint32_t)asInteger(seed), asInteger(kind), &g);
    R_SetExternalPtrAddr(guard, g);
    check(rc);
    int ns = LENGTH(libSizes);
    int64_t k = (int64_t)asReal(size);
    SEXP res = PROTECT(allocVector(VECSXP, ns));
    int64_t* idx = (int64_t*)R_alloc(k > 0 ? (size_t)k : 1, sizeof(int64_t));
    for (int i = 0; i < ns; ++i) {
        check(rcp_rng_sample_sorted(g, (int64_t)REAL(libSizes)[i], k, idx));
        SEXP v = PROTECT(allocVector(REALSXP, (R_xlen_t)k));
        for (int64_t j = 0; j < k; ++j) REAL(v)[j] = (double)idx[j];
        SET_VECTOR_ELT(res, i, v);
        UNPROTECT(1);
    }
    rng_finalizer(guard);
    UNPROTECT(2);
    return res;
}

/* ------------------------------------------------------------------ registration */
static const R_CallMethodDef call_methods[] = {
    {"rcp_R_readset", (DL_FUNC)&rcp_R_readset, 7},
    {"rcp_R_readsets", (DL_FUNC)&rcp_R_readsets, 7},
    {"rcp_R_profile", (DL_FUNC)&rcp_R_profile, 18},
    {"rcp_R_profile_multi", (DL_FUNC)&rcp_R_profile_multi, 18},
    {"rcp_R_profile_samples", (DL_FUNC)&rcp_R_profile_samples, 19},
    {"rcp_R_profile_reads", (DL_FUNC)&rcp_R_profile_reads, 19},
    {"rcp_R_profile_rle", (DL_FUNC)&rcp_R_profile_rle, 14},
    {"rcp_R_coverage", (DL_FUNC)&rcp_R_coverage, 9},
    {"rcp_R_read_bam", (DL_FUNC)&rcp_R_read_bam, 4},
    {"rcp_R_sample_sorted", (DL_FUNC)&rcp_R_sample_sorted, 4},
    {"rcp_R_free", (DL_FUNC)&rcp_R_free, 1},
    {"rcp_R_shards", (DL_FUNC)&rcp_R_shards, 15},
    {"rcp_R_shards_profile", (DL_FUNC)&rcp_R_shards_profile, 10},
    {"rcp_R_shards_coverage", (DL_FUNC)&rcp_R_shards_coverage, 1},
    {"rcp_R_shards_free", (DL_FUNC)&rcp_R_shards_free, 1},
    {"rcp_R_rle_addresses", (DL_FUNC)&rcp_R_rle_addresses, 1},
    {"rcp_R_cov_alive", (DL_FUNC)&rcp_R_cov_alive, 1},
    {"rcp_R_cov_free", (DL_FUNC)&rcp_R_cov_free, 1},
    {"rcp_R_profile_cov", (DL_FUNC)&rcp_R_profile_cov, 10},
    {NULL, NULL, 0}};

void R_init_recoup(DllInfo* dll) {
    R_registerRoutines(dll, NULL, call_methods, NULL, NULL);
    R_useDynamicSymbols(dll, FALSE);
}
