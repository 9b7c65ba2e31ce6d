/*
 * rcp_oracle.h -- CPU ORACLE for the recoup coverage -> profile hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product (recoup_amd/, librecoup_amd.so) never links or calls it.
 *
 * It is a plain-C restatement of the reference's algorithm, following:
 *   R/coverage.R:126-174   calcCoverage (strand filter, split by seqname, per-region map)
 *   R/coverage.R:176-226   coverageFromRanges (findOverlaps -> coverage -> [i2k] -> rev)
 *   R/profile.R:100-212    baseCoverageMatrix / binCoverageMatrix (slices, NULL -> zeros)
 *   R/util.R:15-85         splitVector (interpolation, R-RNG bin layout, stat)
 *   R/util.R:364-382       cmclapply (here: a pthread pool over regions)
 * plus the un-vendored upstream semantics it relies on (GenomicRanges findOverlaps /
 * coverage, S4Vectors Rle subsetting, base R set.seed/sample/mean/median,
 * stats::spline "fmm"), restated in SURVEY.md Appendix A/B.
 *
 * Parity pinning: R is not installed in this image, so no output of executed R
 * exists.  The oracle is pinned by (i) R's published RNG known answers
 * (set.seed(42); runif / sample), (ii) exactness properties of the fmm spline, and
 * (iii) SURVEY Appendix B sanity numbers on the reference's own fixture
 * data/recoup_test_data.rda.  See DESIGN.md §2.
 */
#ifndef RCP_ORACLE_H
#define RCP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_index orc_index;

/* Reads as a flat GRanges: 1-based closed [start,end]; strand 0 '+', 1 '-', 2 '*'. */
typedef struct {
    int64_t n;
    const int32_t* chrom;
    const int32_t* start;
    const int32_t* end;
    const int8_t* strand;
    int32_t n_chrom;
    const int64_t* seqlen; /* per chromosome, -1 = NA */
} orc_reads_in;

/* Mask elements (one GRanges element, or one GRangesList element = several ranges). */
typedef struct {
    int32_t n;
    const int64_t* seg_off;    /* n+1 */
    const int32_t* seg_chrom;
    const int32_t* seg_start;
    const int32_t* seg_end;
    const int8_t* seg_strand;
} orc_mask_in;

enum { ORC_WHERE_WHOLE = 0, ORC_WHERE_CENTER = 1, ORC_WHERE_UPSTREAM = 2, ORC_WHERE_DOWNSTREAM = 3 };
enum { ORC_INTERP_AUTO = 0, ORC_INTERP_SPLINE = 1, ORC_INTERP_LINEAR = 2, ORC_INTERP_NEIGHBORHOOD = 3 };
enum { ORC_STAT_MEAN = 0, ORC_STAT_MEDIAN = 1 };
enum { ORC_RNG_REJECTION = 0, ORC_RNG_ROUNDING = 1 };

/* splitBySeqname + optional strand filter (coverage.R:141-146): strand_filter -1 = none. */
orc_index* orc_index_build(const orc_reads_in* reads, int strand_filter);
void orc_index_free(orc_index* ix);

/* calcCoverage.  First call with out_cov == NULL fills out_len with the nominal
 * (valid-row) coverage length of every region; the caller then builds out_off
 * (prefix sums of out_len) and calls again to fill out_cov / valid.  A region the
 * reference maps to NULL gets valid = 0 and nothing written. */
int orc_coverage(const orc_index* ix, const orc_mask_in* mask, int ignore_strand, int nthreads,
                 const int64_t* out_off, int32_t* out_cov, uint8_t* valid, int64_t* out_len);

/* splitVector(x, n, interp, stat) (util.R:15-85).  out must hold max(n, L) doubles.
 * Returns 0, or a negative code where R would raise an error. */
int orc_split_vector(const double* x, int64_t L, int n, int interp, int stat, int rng_kind,
                     double* out, int64_t* out_len);

/* One fused pass per region, as the reference's dataflow does it: coverageFromRanges
 * -> as.numeric(x) * scale -> slice(where, f1, f2) -> splitVector (n > 0) or per-base
 * (n == 0) -> row of the R x ncol column-major matrix (rows shorter than ncol are
 * recycled, as rbind does).  Multithreaded over regions with nthreads threads. */
int orc_profile(const orc_index* ix, const orc_mask_in* mask, int ignore_strand, double scale,
                int where, int f1, int f2, int n, int interp, int stat, int rng_kind,
                int nthreads, double* out, int64_t ncol, uint8_t* valid);

/* Rows of several mask elements ("groups"; coverageRnaRef: left flank, exon list, right
 * flank, R/coverage.R:79-124) profiled over several column parts (R/profile.R:13-81). */
typedef struct {
    int32_t n;
    const int64_t* seg_off;     /* n+1 */
    const int32_t* seg_chrom;
    const int32_t* seg_start;
    const int32_t* seg_end;
    const int8_t* seg_strand;
    const int8_t* seg_group;    /* NULL = one group */
    const uint8_t* group_is_list; /* [4]; NULL = no lists */
} orc_rows_in;

typedef struct {
    int32_t n_parts;
    const int32_t* where;
    const int32_t* n_bins;      /* 0 = per base */
    const int32_t* per_base_width;
    int32_t f1, f2;
    int32_t stat, interp, rng_kind;
    double scale;
} orc_parts_in;

int orc_profile_rows(const orc_index* ix, const orc_rows_in* rows, const orc_parts_in* parts, int ignore_strand,
                     int nthreads, double* out, uint8_t* valid);

/* R RNG restatement, exposed for known-answer tests. */
void orc_set_seed(uint32_t seed);
double orc_unif_rand(void);
int orc_sample(int n, int k, int rng_kind, int* out); /* sample.int(n, k), 1-based */
/* spline(x, n=n) with method fmm on x = 1..L (stats::spline), no clipping. */
int orc_spline(const double* y, int64_t L, int n, double* out);

#ifdef __cplusplus
}
#endif
#endif
