/*
 * recoup_amd.h -- C ABI of the MI355X coverage-profile engine (librecoup_amd.so).
 *
 * Drop-in boundary for recoup's hot path
 *   calcCoverage / coverageRef / coverageRnaRef  ->  profileMatrix
 * The reference is pure R with no FFI; these entry points are what
 * a thin `.Call` shim replacing the R functions below would bind (INTEGRATION.md shows
 * that shim and the R-side wrappers):
 *
 *   rcp_readset_create   replaces splitBySeqname()            R/util.R:1-13
 *                        (+ the strand filter of calcCoverage R/coverage.R:141-144)
 *   rcp_calc_coverage    replaces calcCoverage()              R/coverage.R:126-174
 *   rcp_rle_encode       the Rle values / lengths of each coverage (R/coverage.R:171-173)
 *   rcp_bam_read         readBam() -> the read arrays      R/ranges.R:111-146 (next row)
 *   rcp_rng_*            set.seed + sort(sample(n, k)) of downsample / sampleto  R/ranges.R:32-62
 *                        and its per-region coverageFromRanges R/coverage.R:176-226
 *   rcp_plan_create /    replace the coverage -> profile pass:
 *   rcp_plan_execute /     coverageFromRanges                 R/coverage.R:176-226
 *   rcp_profile            binCoverageMatrix                  R/profile.R:153-212
 *                          baseCoverageMatrix                 R/profile.R:100-151
 *                          splitVector                        R/util.R:15-85
 *                        fused into one device pass; the caller (profileMatrix,
 *                        R/profile.R:1-98) describes the column parts it needs.
 *
 * Conventions
 *  - Coordinates are 1-based closed [start, end], as in GRanges.
 *  - Strand codes: 0 '+', 1 '-', 2 '*'.
 *  - Matrices are R column-major doubles (element (r, c) at out[c * n_rows + r]).
 *  - Every function returns RCP_OK (0) or a negative RCP_E* code; the message is
 *    available from rcp_last_error() (thread-local).  Nothing longjmps.
 *  - A region the reference maps to NULL (no overlapping reads, chromosome absent,
 *    subscript out of bounds: R/coverage.R:189-225) is NOT an error: row_valid = 0 and
 *    the row is zero-filled, as profile.R:116-122 / :191-197 do.
 *  - The library owns the device buffers it allocates (RAII inside handles); inputs are
 *    never modified.  Not fork-safe: call it outside mclapply (R/util.R:364-382).
 */
#ifndef RECOUP_AMD_H
#define RECOUP_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define RCP_API __attribute__((visibility("default")))
#else
#define RCP_API
#endif

#define RCP_OK 0
#define RCP_EINVAL (-1)       /* bad argument / shape */
#define RCP_EHIP (-2)         /* HIP runtime failure */
#define RCP_ENOMEM (-3)       /* device allocation failed */
#define RCP_EUNSUPPORTED (-4) /* valid R input outside what this build implements */
#define RCP_ESEMANTIC (-5)    /* the reference itself would raise an R error here */
#define RCP_ENODEVICE (-6)    /* no GPU visible */

enum { RCP_STRAND_PLUS = 0, RCP_STRAND_MINUS = 1, RCP_STRAND_ANY = 2 };
enum { RCP_STAT_MEAN = 0, RCP_STAT_MEDIAN = 1 };                    /* binParams$sumStat */
enum { RCP_INTERP_AUTO = 0, RCP_INTERP_SPLINE = 1,                  /* binParams$interpolation */
       RCP_INTERP_LINEAR = 2, RCP_INTERP_NEIGHBORHOOD = 3 };
enum { RCP_RNG_REJECTION = 0, RCP_RNG_ROUNDING = 1 };               /* RNGkind(sample.kind=) */

RCP_API const char* rcp_version(void);
RCP_API const char* rcp_last_error(void);
RCP_API int rcp_device_count(int* n);

/* ------------------------------------------------------------------ reads */
typedef struct rcp_readset rcp_readset;

typedef struct {
    int64_t n;              /* number of reads (< 2^31) */
    const int32_t* chrom;   /* [n] chromosome code 0..n_chrom-1 (seqnames); NULL: runs below.
                             * A code outside [0, n_chrom) (R's NA from match()) or a strand
                             * code outside 0..2 drops the read (it joins no stream), as a
                             * read on a seqlevel the mask never names is never a hit. */
    const int32_t* start;   /* [n] 1-based start                                       */
    const int32_t* end;     /* [n] 1-based end (inclusive); NULL: width runs below     */
    const int8_t* strand;   /* [n] strand code                                         */
    int32_t n_chrom;        /* seqlevels                                               */
    const int64_t* seqlen;  /* [n_chrom] host pointer; -1 = NA seqlength               */
    int32_t device;         /* HIP device ordinal                                      */
    int32_t on_device;      /* 1: chrom/start/end/strand are device pointers           */
    int32_t strand_filter;  /* -1 none, else keep only reads of that strand (calcCoverage strand=) */
    /* seqnames as runs, GRanges' own Rle (runValue / runLength of seqnames(x)), used when
     * chrom is NULL: a coordinate-sorted BAM's reads are a few dozen runs, so the 4 bytes per
     * read of an expanded chromosome vector never cross PCIe.  Host pointers in both modes. */
    int32_t n_chrom_runs;
    const int32_t* chrom_run_value;   /* [n_chrom_runs] chromosome code of each run          */
    const int64_t* chrom_run_length;  /* [n_chrom_runs] > 0, summing to n                    */
    /* widths as runs (IRanges holds start and width; width(x) as an Rle), used when end is
     * NULL: end = start + width - 1 is formed on the device, so reads of one length (a
     * sequencing run's fixed read length) send no end vector over PCIe.  Host pointers in
     * both modes. */
    int32_t n_width_runs;
    const int32_t* width_run_value;   /* [n_width_runs] >= 0                                  */
    const int64_t* width_run_length;  /* [n_width_runs] > 0, summing to n                    */
} rcp_reads_desc;

/* Upload (or adopt device arrays), sort by (chrom, strand, start) on the GPU, and build
 * the per-(chrom, strand) stream offsets plus the prefix-max-of-end search index. */
RCP_API int rcp_readset_create(const rcp_reads_desc* desc, void* hip_stream, rcp_readset** out);
RCP_API int rcp_readset_destroy(rcp_readset* rs);
/* The library's device memory (readset and plan arrays, build and encode temporaries) comes from
 * a caching allocator: freed blocks are kept, keyed by size class, for the next build of that
 * size (no hipMalloc / hipFree -- each a device-wide synchronisation, and now and then a
 * multi-second stall on the box -- once warm).  This returns every cached block to the runtime;
 * blocks are also released when a device allocation fails. */
RCP_API int rcp_release_pool(int device);
/* n_reads kept, and stream offsets (host array of n_chrom*3+1, may be NULL) of the strand-split
 * layout.  A readset made from host arrays builds that layout at its first use -- here when
 * stream_off != NULL, or in a plan with ignore_strand == 0 -- a device build of the same size as
 * rcp_readset_create's, which can fail with RCP_ENOMEM / RCP_EHIP; a failed build leaves the
 * readset as it was (the next use tries again). */
RCP_API int rcp_readset_info(const rcp_readset* rs, int64_t* n_reads, int64_t* stream_off);

/* ------------------------------------------------------------------ rows */
/* A coverage row is c(cov(g0), cov(g1), ...) over the mask elements ("groups") listed for
 * that row, each cov(g) being coverageFromRanges() of that mask element (ranges in list
 * order, reversed when the element's first range is on '-').  A ChIP-seq row has one group
 * (one GRanges element); a coverageRnaRef row has three: upstream flank, the gene's exon
 * list (a GRangesList element, reads counted once per exon they overlap), downstream flank
 * (R/coverage.R:84-121).  The row is NULL when any of its groups is NULL. */
typedef struct {
    int32_t n_rows;
    const int64_t* seg_off;     /* [n_rows+1] segments of each row, groups contiguous      */
    const int32_t* seg_chrom;   /* [n_seg]                                                 */
    const int32_t* seg_start;   /* [n_seg]                                                 */
    const int32_t* seg_end;     /* [n_seg]                                                 */
    const int8_t* seg_strand;   /* [n_seg]                                                 */
    const int8_t* seg_group;    /* [n_seg] group index inside the row (0..3); NULL = all 0  */
    const uint8_t* group_is_list; /* [4] 1 = the group is a GRangesList element; NULL = none */
    int32_t ignore_strand;      /* findOverlaps(ignore.strand=) (strandedParams$ignoreStrand) */
} rcp_rows_desc;

/* ------------------------------------------------------------------ bins */
/* The profile row is cbind over parts (R/profile.R:13-81); part p takes the slice of the
 * row named by where[p] (profile.R / binCoverageMatrix `where`, with flank = (f1, f2)):
 *   RCP_WHERE_WHOLE       1:nr             (equal-length branch, profile.R:83-96)
 *   RCP_WHERE_CENTER      (f1+1):(nr-f2)   (profile.R:166-173)
 *   RCP_WHERE_UPSTREAM    1:f1             (profile.R:175-181)
 *   RCP_WHERE_DOWNSTREAM  (nr-f2+1):nr     (profile.R:182-188)
 * and summarises it with n_bins[p] bins through splitVector (R/util.R:15-85), or per base
 * when n_bins[p] == 0 (baseCoverageMatrix; the part then has per_base_width[p] columns). */
enum { RCP_WHERE_WHOLE = 0, RCP_WHERE_CENTER = 1, RCP_WHERE_UPSTREAM = 2, RCP_WHERE_DOWNSTREAM = 3 };

typedef struct {
    int32_t n_parts;            /* 1..8 */
    const int32_t* where;       /* [n_parts] RCP_WHERE_* */
    int32_t flank[2];           /* (f1, f2) */
    const int32_t* n_bins;      /* [n_parts] 0 = per base */
    const int32_t* per_base_width; /* [n_parts] columns of a per-base part (else ignored) */
    int32_t stat;               /* RCP_STAT_* */
    int32_t interp;             /* RCP_INTERP_* */
    int32_t rng_kind;           /* RCP_RNG_* */
    double scale;               /* linear normalization factor (recoup.R:559-577); 1 = none */
} rcp_bins_desc;

typedef struct rcp_plan rcp_plan;

typedef struct {
    int64_t n_cols;             /* total matrix columns */
    int64_t n_segments;
    int64_t n_interp_rows;      /* (row, part) pairs with fewer positions than bins */
    int64_t lds_bytes;          /* dynamic LDS of the pileup kernel */
    int64_t grid;               /* workgroups of the pileup kernel */
    int32_t tile_rows;
    int32_t chunk_positions;
    int32_t pileup_kernel;   /* 0: general pileup kernel; 1: lean kernel (pile + store waves);
                              * 2: lean kernel, general bins; 3: row-wave kernel; 4: bin-difference kernel */
    int32_t read_bytes;      /* bytes per candidate read the pileup kernel streams: 4 (the starts alone,
                              * reads of one width) or 8 ((start, end) pairs) */
    int64_t out_ld;          /* column stride of d_out / d_binsum (rcp_plan_opts.out_ld resolved):
                              * both must hold out_ld * (n_cols - 1) + n_rows elements */
    int32_t fold;            /* 1: the pileup kernel searches its rows' read ranges itself (no locate or
                              * heavy-slice launch; skewed rows piled by whole workgroups): bin-difference
                              * and row-wave plans, and general-kernel plans of <= 65536 single-range rows
                              * in the merged layout, unless a heavy_threshold > 0 was asked for */
    int32_t reserved;
} rcp_plan_info;

/* Host work: orientation of segments, R-RNG bin layouts (set.seed(42); sample(1:n, dif)),
 * interpolation plans, chunking; uploads the tables to the readset's device.  bins may be
 * NULL for a calcCoverage-only plan.  The readset must outlive the plan. */
RCP_API int rcp_plan_create(const rcp_readset* rs, const rcp_rows_desc* rows, const rcp_bins_desc* bins,
                    rcp_plan** out);
/* Plan options (NULL = defaults).  pileup_kernel: RCP_KERNEL_AUTO picks the lean kernel
 * (pile + store waves) where every row is one plain range with uniform power-of-two bins
 * (binned plans: from 36000 rows up; fewer rows, e.g. one GPU's 1/8 of a region table, run
 * faster on the general kernel's smaller workgroup tiles), else the general kernel;
 * RCP_KERNEL_LEAN takes the lean kernel wherever AUTO's shape rule allows, at any row count;
 * RCP_KERNEL_GENERAL forces the general kernel; RCP_KERNEL_LEAN_ANY
 * also routes other mean plans whose chunks fit one wave pass through the lean kernel's
 * general-bins mode; RCP_KERNEL_ROWS forces the row-wave kernel (whole rows per wave: AUTO takes
 * it for mean plans with multi-range rows); RCP_KERNEL_BINS the bin-difference kernel (a read adds to
 * the bins it overlaps, not to positions: AUTO takes it for mean plans of one binned part whose
 * single-range rows are all cut into whole bins of >= 4 positions, <= 512 bins, e.g. TSS
 * windows in 200 bins).  All choices give bit-identical results.  heavy_threshold: candidate
 * reads per column chunk above which a skewed row is piled by many workgroups first
 * (-1 = default 4096, 0 = never; row-wave and bin-difference plans without an explicit
 * threshold search their rows' read ranges in the pileup kernel itself and have no heavy path).
 * out_ld: see the field. */
enum { RCP_KERNEL_AUTO = 0, RCP_KERNEL_GENERAL = 1, RCP_KERNEL_LEAN_ANY = 2, RCP_KERNEL_ROWS = 3, RCP_KERNEL_LEAN = 4,
       RCP_KERNEL_BINS = 5 };
typedef struct {
    int32_t pileup_kernel;
    int32_t heavy_threshold;
    int64_t out_ld;             /* column stride (leading dimension) of d_out / d_binsum in elements:
                                 * 0 = n_rows (plain R column-major); >= n_rows otherwise.  A multiple
                                 * of 16 keeps every 16-row column segment on whole 128-B lines
                                 * (RCP_OUT_LD_PADDED picks the next multiple of 16) */
    int32_t min_col_chunks;     /* lean plans and one-part general plans: cut each part into at least
                                 * this many column chunks (<= 16; 0 = auto: lean plans take enough
                                 * (row tile, chunk) work items for the persistent grid -- small row
                                 * tables, e.g. one GPU's shard, get more chunks so the last items do
                                 * not leave most workgroups idle; general plans keep <= 1023
                                 * positions a chunk -- more measured slower on the C4 shard) */
    int32_t concurrent;         /* plans the caller keeps in flight on other streams (0 / 1 = this one
                                 * alone, e.g. one profileMatrix pass per sample of an input list run
                                 * on D streams): > 1 makes the persistent pileup grids (lean,
                                 * row-wave) leave 1/8 of the CUs' workgroup slots free, so another
                                 * sample's locate and heavy
                                 * launches run beside this pileup (C4, 2 samples in flight:
                                 * 0.600-0.627 -> 0.580-0.596 ms per pass; alone 0.61 -> 0.67) */
    int32_t reserved[2];        /* zero */
} rcp_plan_opts;
#define RCP_OUT_LD_PADDED (-1)
RCP_API int rcp_plan_create_ex(const rcp_readset* rs, const rcp_rows_desc* rows, const rcp_bins_desc* bins,
                               const rcp_plan_opts* opts, rcp_plan** out);
RCP_API int rcp_plan_destroy(rcp_plan* plan);
RCP_API int rcp_plan_info_get(const rcp_plan* plan, rcp_plan_info* info);

/* Device work only (stream-ordered, no host sync, capturable in a hipGraph):
 *   locate kernel (per segment/stream read ranges + NULL semantics; writes d_valid; also
 *     clears the skewed-row state the previous execution of this plan left),
 *   skewed-row slice kernel,
 *   pileup-bin kernel (LDS difference array -> scans -> bins -> column-major out),
 *   interpolation kernel for rows with fewer positions than bins.
 * d_out: device doubles, column c of the R matrix at d_out + c * out_ld (out_ld =
 * rcp_plan_info.out_ld: n_rows unless the plan was created with a wider stride), so it holds
 * out_ld * (n_cols - 1) + n_rows elements -- [n_rows * n_cols] for the default stride.
 * d_valid (device, n_rows) and d_binsum (device int64 numerators, same shape and stride as
 * d_out; median rows hold 2x the median) may be NULL.  A device-side status word reports numerator overflow; rcp_plan_status() reads it. */
RCP_API int rcp_plan_execute(rcp_plan* plan, double* d_out, uint8_t* d_valid, int64_t* d_binsum,
                     void* hip_stream);
/* The same pass split into its launches (for per-kernel timing with events between them):
 * stages is a mask of RCP_STAGE_*; stages must be enqueued in order on one stream. */
enum { RCP_STAGE_LOCATE = 1, RCP_STAGE_PILEUP = 2, RCP_STAGE_INTERP = 4, RCP_STAGE_ALL = 7 };
RCP_API int rcp_plan_execute_stages(rcp_plan* plan, double* d_out, uint8_t* d_valid, int64_t* d_binsum,
                                    void* hip_stream, int stages);
/* Synchronises the stream and returns RCP_OK or the error the last execute raised. */
RCP_API int rcp_plan_status(rcp_plan* plan, void* hip_stream);
/* Rows the last execution sent through the skewed-row (heavy slice) path; synchronises the
 * stream.  Diagnostics / tests: the count is cleared by the next execution's first kernel. */
RCP_API int rcp_plan_heavy_rows(rcp_plan* plan, void* hip_stream, int32_t* n_rows);
/* Only the locate kernel: row validity (device pointer), e.g. for profileMatrix's
 * equal-length test on sample 1 (R/profile.R:6-10). */
RCP_API int rcp_plan_validity(rcp_plan* plan, uint8_t* d_valid, void* hip_stream);
/* Nominal (valid-row) coverage length of every row, host array [n_rows]. */
RCP_API int rcp_plan_row_lengths(const rcp_plan* plan, int64_t* out_len);

/* One-shot host-pointer entry point (what the R .Call shim binds): create plan, execute,
 * copy out (host, R column-major n_rows x n_cols), copy row_valid (host, may be NULL),
 * destroy. */
RCP_API int rcp_profile(const rcp_readset* rs, const rcp_rows_desc* rows, const rcp_bins_desc* bins,
                double* out, uint8_t* row_valid);

/* Several GPUs in one call: the reference parallelises the per-region
 * work over host cores with cmclapply (R/util.R:364-382, used by R/coverage.R:147-154 and
 * R/profile.R:84-96); here the rows are cut into n_devices contiguous blocks and one host thread
 * per GPU builds the plan for its block, executes it and copies its rows of every column straight
 * into the caller's R column-major n_rows x n_cols matrix -- no collective, no host reassembly.
 *
 * Two ways to hold the reads:
 *  - rcp_shards_create (below): the reads split for ONE row table -- each GPU holds only the reads
 *    its block's regions can overlap.  What recoup()'s own path uses (r/R/rcp.R).
 *  - rcp_readset_create_multi: REPLICAS -- one readset of all the reads on each listed device (in
 *    parallel, one thread per device), reusable with any row table (rcp_profile_multi), as R keeps
 *    input$ranges.  n_devices x the upload and the device memory of one readset.
 * rcp_profile_multi balances its blocks by each row's candidate reads (counted on readsets[0]'s
 * GPU) plus its length / 8, in the caller's row order; row_split (may be NULL) receives the
 * n_devices + 1 block boundaries.  The result is bit-identical to rcp_profile on one device. */
RCP_API int rcp_readset_create_multi(const rcp_reads_desc* desc, const int32_t* device_ids, int32_t n_devices,
                                     rcp_readset** out);
RCP_API int rcp_profile_multi(rcp_readset* const* readsets, int32_t n_devices, const rcp_rows_desc* rows,
                              const rcp_bins_desc* bins, double* out, uint8_t* row_valid, int32_t* row_split);

/* One sample's reads split over several GPUs for ONE row table (what cmclapply over the regions
 * of calcCoverage, R/coverage.R:147-154, and over the rows of binCoverageMatrix, R/profile.R:198-199,
 * parallelise).  The rows, taken in (chromosome, start) order whatever the caller's order (rows on
 * an absent chromosome last), are cut into n_devices contiguous blocks of that order of
 * near-equal weight -- each row's candidate reads, counted on the GPUs, plus its length / 8 -- and
 * device i keeps ONLY the reads block i's rows can overlap:
 *   the reads are uploaded in n_devices slices, one per GPU (all PCIe links at once; device input:
 *   one slice on its device); each GPU sorts its slice and counts every row range's candidates;
 *   each GPU gathers, for every block, its slice's reads inside the block's candidate ranges and
 *   copies them device to device (xGMI, hipMemcpyPeer) to the block's GPU, which builds the
 *   block's readset (the layout rows->ignore_strand searches).
 * A read that several blocks' regions overlap goes to each of them.  The row table is copied;
 * bins come per call.  device_ids may repeat a device.  Every result is bit-identical to the
 * same call on one device (a region sees exactly the reads findOverlaps hits). */
typedef struct rcp_shards rcp_shards;
typedef struct rcp_cov rcp_cov;  /* (calcCoverage results: see rcp_coverage_rle) */
RCP_API int rcp_shards_create(const rcp_reads_desc* reads, const rcp_rows_desc* rows, const int32_t* device_ids,
                              int32_t n_devices, rcp_shards** out);
/* n_rows, n_devices; row_split [n_devices + 1]: the row blocks, as positions of the order
 * rcp_shards_rows gives; n_reads [n_devices]: the reads each device holds (any may be NULL) */
RCP_API int rcp_shards_info(const rcp_shards* sh, int32_t* n_rows, int32_t* n_devices, int32_t* row_split,
                            int64_t* n_reads);
/* order [n_rows]: the caller's row at each position of the blocks' (chromosome, start) order --
 * block b holds rows order[row_split[b]] .. order[row_split[b + 1] - 1].  Results (profiles,
 * coverage lists) are always in the caller's row order. */
RCP_API int rcp_shards_rows(const rcp_shards* sh, int32_t* order);
/* profileMatrix of the row table (as rcp_profile: out = host R column-major n_rows x n_cols,
 * row_valid may be NULL): one plan per device, each writing its rows of the caller's matrix */
RCP_API int rcp_shards_profile(rcp_shards* sh, const rcp_bins_desc* bins, double* out, uint8_t* row_valid);
/* calcCoverage of the row table as run-length encoded lists (as rcp_coverage_rle): one handle
 * over the devices' blocks; rcp_cov_info / rcp_cov_copy / rcp_cov_free as for one device */
RCP_API int rcp_shards_coverage(rcp_shards* sh, rcp_cov** out);
RCP_API int rcp_shards_destroy(rcp_shards* sh);

/* Several samples over one region table -- profileMatrix's loop over the samples of a recoup
 * input list (R/profile.R:13-98, `for (n in names(input))`) -- in one call: one plan per sample
 * (all readsets on one device), passes kept `inflight` deep on as many HIP streams (1..3; 0 =
 * 2), so one sample's locate / heavy launches and the tail of its persistent pileup grid overlap
 * another's pileup, and each finished sample's matrix is copied (staged) into outs[s] -- the
 * caller's R column-major n_rows x n_cols matrix -- while later samples compute.  row_valid may
 * be NULL, or hold n_samples pointers (each may be NULL).  Bit-identical to rcp_profile per
 * sample. */
RCP_API int rcp_profile_samples(rcp_readset* const* readsets, int32_t n_samples, const rcp_rows_desc* rows,
                                const rcp_bins_desc* bins, int32_t inflight, double* const* outs,
                                uint8_t* const* row_valid);

/* profileMatrix straight from the reads of several samples over one region table, reads on the
 * host (R's vectors): samples[k] describes sample k's reads (all for one device, host arrays),
 * outs[k] its R column-major n_rows x n_cols matrix (row_valid may be NULL or hold per-sample
 * pointers).  A sample of >= 4 M coordinate-sorted reads given as chromosome runs (each
 * chromosome one run) and width runs -- a sorted BAM's GAlignments -- over >= 2048 rows streams
 * through the GPU in row blocks: block b's slice of the reads (found by bisection of the host
 * starts; the slices' order is checked on the device and a sample that proves unsorted is redone
 * whole) goes up while block b - 1's rows of the matrix come down; any other sample goes up whole
 * while the previous one's matrix comes down.  Both PCIe directions at once (the one-shot
 * rcp_readset_create + rcp_profile uses one direction at a time); at most four readsets are on
 * the device.  Bit-identical to rcp_profile per sample. */
RCP_API int rcp_profile_reads(const rcp_reads_desc* samples, int32_t n_samples, const rcp_rows_desc* rows,
                              const rcp_bins_desc* bins, double* const* outs, uint8_t* const* row_valid);

/* Profiles of a coverage list the caller holds as run-length encoded vectors -- the reference's
 * own `$coverage` object, a named list of S4Vectors::Rle (R/coverage.R:171-173) -- as
 * binCoverageMatrix / baseCoverageMatrix consume it (R/profile.R:100-212) when recoup() reuses a
 * stored or sliced coverage (R/recoup.R:126-135, R/util.R:209-210, :311-320).  Row r's runs are
 * run_off[r] .. run_off[r+1]-1 (runValue / runLength of the Rle); exactly one of ivalues (an
 * integer Rle, as calcCoverage returns it) and dvalues (a numeric Rle, e.g. after
 * normalize = "linear", R/recoup.R:559-577) is given.  is_null[r] = 1 marks a NULL list element
 * (a zero row, row_valid = 0).  bins as for rcp_profile (parts, stat, interpolation, R-RNG bin
 * layouts, scale); out: host R column-major n_rows x n_cols.  Integer Rle rows give the same
 * bits as the read path (numerators in int64, mean = numerator * scale / width); numeric Rle
 * means are the exact sum (double-double of value x overlap) divided once with a remainder
 * correction -- R's long-double mean of the same values except at double-rounding ties. */
typedef struct {
    int32_t n_rows;
    const int64_t* run_off;     /* [n_rows + 1], run_off[0] = 0 */
    const int32_t* lengths;     /* [n_runs] > 0 */
    const int32_t* ivalues;     /* [n_runs] or NULL */
    const double* dvalues;      /* [n_runs] or NULL */
    const uint8_t* is_null;     /* [n_rows] or NULL (no NULL elements) */
} rcp_rle_desc;
RCP_API int rcp_profile_rle(const rcp_rle_desc* cov, const rcp_bins_desc* bins, int device, double* out,
                            uint8_t* row_valid);
/* rcp_profile_rle over several GPUs: the rows cut into n_devices contiguous blocks balanced by
 * their runs (+ a constant per row: the output), each block's runs uploaded to its GPU and its
 * rows of every column copied into `out` (binCoverageMatrix's per-row cmclapply,
 * R/profile.R:198-199).  Bit-identical to rcp_profile_rle. */
RCP_API int rcp_profile_rle_multi(const rcp_rle_desc* cov, const rcp_bins_desc* bins, const int32_t* device_ids,
                                  int32_t n_devices, double* out, uint8_t* row_valid);

/* rcp_profile_rle of a calcCoverage result still held on the device (rcp_coverage_rle /
 * rcp_shards_coverage): the profile of exactly the runs rcp_cov_copy gives, without them crossing
 * PCIe again -- recoup() profiles the list coverageRef just returned (R/recoup.R:551-597, and the
 * forced heatmap binning :659-714); the R wrappers use it while the list's Rle vectors are the ones
 * copied out (r/R/rcp.R).  bins, out (host R column-major n_rows x n_cols) and row_valid as for
 * rcp_profile_rle; NULL rows are the invalid ones.  Bit-identical to rcp_profile_rle of the copied
 * runs. */
RCP_API int rcp_profile_cov(const rcp_cov* cov, const rcp_bins_desc* bins, double* out, uint8_t* row_valid);

/* calcCoverage: per-row integer depth vectors (CSR).  out_off is the host prefix sum of
 * rcp_plan_row_lengths(); d_cov (device int32 [out_off[n_rows]]) receives each valid row's
 * depth at its offset; d_valid (device) the NULL mask.  Rows are in the row's own
 * orientation (reversed for '-'), i.e. exactly the values of the reference's Rle. */
RCP_API int rcp_calc_coverage(rcp_plan* plan, const int64_t* out_off, int32_t* d_cov, uint8_t* d_valid,
                      void* hip_stream);

/* calcCoverage one-shot for host callers (the R .Call shim): the coverage of every row of
 * `rows` over the readset (R/coverage.R:126-226), run-length encoded on the GPU and held in
 * device memory by the handle -- exactly the values / lengths of the reference's named list of
 * Rle (NULL rows: valid[r] = 0 and no runs).  rcp_cov_info gives the sizes; rcp_cov_copy copies
 * them straight into caller arrays (run_off [n_rows + 1]: runs of row r are run_off[r] ..
 * run_off[r+1]-1; values / lengths [n_runs]; valid [n_rows]; any may be NULL; may be called
 * again); rcp_cov_free releases the device memory. */
typedef struct rcp_cov rcp_cov;
RCP_API int rcp_coverage_rle(const rcp_readset* rs, const rcp_rows_desc* rows, rcp_cov** out);
RCP_API int rcp_cov_info(const rcp_cov* c, int32_t* n_rows, int64_t* n_runs);
RCP_API int rcp_cov_copy(const rcp_cov* c, int64_t* run_off, int32_t* values, int32_t* lengths, uint8_t* valid);
RCP_API int rcp_cov_free(rcp_cov* c);

/* ------------------------------------------------------------------ BAM ingest */
/* readBam (R/ranges.R:111-146) on the host: BGZF blocks inflated by n_threads threads, mapped
 * alignments (readGAlignments) turned into 1-based ranges on their reference and strand:
 *   RCP_SPLICE_KEEP    the reference span (as(GAlignments, "GRanges"))
 *   RCP_SPLICE_SPLIT   one range per block between N-skips (unlist(grglist(.)))
 *   RCP_SPLICE_REMOVE  spans, minus those wider than quantile(width, remove_q) (type 7)
 * all clipped to [1, seqlength] (trim()).  The arrays feed rcp_readset_create (chrom = BAM
 * reference index, seqlen = the header's lengths). */
enum { RCP_SPLICE_KEEP = 0, RCP_SPLICE_REMOVE = 1, RCP_SPLICE_SPLIT = 2 };
typedef struct rcp_bam rcp_bam;
RCP_API int rcp_bam_read(const char* path, int splice_action, double remove_q, int n_threads, rcp_bam** out);
RCP_API int rcp_bam_info(const rcp_bam* bam, int64_t* n_reads, int32_t* n_ref, int64_t* n_alignments);
RCP_API const char* rcp_bam_ref_name(const rcp_bam* bam, int32_t i);
/* Copy out: ref_len [n_ref]; chrom / start / end / strand [n_reads] (any may be NULL). */
RCP_API int rcp_bam_copy(const rcp_bam* bam, int64_t* ref_len, int32_t* chrom, int32_t* start, int32_t* end,
                         int8_t* strand);
RCP_API int rcp_bam_free(rcp_bam* bam);

/* ------------------------------------------------------------------ R RNG */
/* The preprocessing steps normalize = "downsample" / "sampleto" (R/ranges.R:32-62):
 * set.seed(seed) once, then per sample sort(sample(libsize, size)) -- written to `out` as
 * 1-based read indices, in the RNG state order R uses (sample.int's hash variant when
 * n > 1e7 and k <= n/2).  k > n is the R error "cannot take a sample larger than the
 * population" (RCP_ESEMANTIC).  kind: RCP_RNG_*. */
typedef struct rcp_rng rcp_rng;
RCP_API int rcp_rng_create(uint32_t seed, int kind, rcp_rng** out);
RCP_API int rcp_rng_unif(rcp_rng* rng, int64_t k, double* out);
RCP_API int rcp_rng_sample_sorted(rcp_rng* rng, int64_t n, int64_t k, int64_t* out);
RCP_API int rcp_rng_free(rcp_rng* rng);

/* Run-length encoding of a CSR coverage (the output of rcp_calc_coverage): the values and
 * lengths of each row's Rle, as S4Vectors::Rle(values, lengths) holds them
 * (R/coverage.R:171-173 returns a list of Rle; the R shim rebuilds them without expanding).
 * out_off: host [n_rows + 1] offsets of d_cov (device int32).  d_values / d_lengths: device
 * int32 arrays of at least out_off[n_rows] entries.  run_off: host [n_rows + 1] (runs of row r
 * are run_off[r] .. run_off[r+1]); n_runs: total runs.  Blocks until done. */
RCP_API int rcp_rle_encode(int32_t n_rows, const int64_t* out_off, const int32_t* d_cov, int device,
                           int32_t* d_values, int32_t* d_lengths, int64_t* run_off, int64_t* n_runs,
                           void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* RECOUP_AMD_H */
