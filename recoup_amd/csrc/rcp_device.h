// rcp_device.h -- device-side plan layout shared by rcp_kernels.hip and rcp_host.cpp.
//
// All tables are built on the host (rcp_host.cpp) and uploaded once per plan; the
// kernels only read them.  Names follow the reference's domain: reads, streams
// (a (chromosome, strand) run of start-sorted reads), rows (one mask element, or the
// c(left, exons, right) of coverageRnaRef), segments (the ranges of a row, in output
// order), parts (the profile.R slices: upstream / center / downstream) and bins.
#pragma once
#include <stdint.h>

#define RCP_MAX_PARTS 8
#define RCP_BLOCK 256

// One oriented segment of a row: genomic run [lo, hi] written to row positions
// [off, off + hi - lo] forward (rev = 0) or reversed (rev = 1).
struct RcpSeg {
    int32_t lo, hi;      // genomic run (1-based, inclusive)
    int32_t off;         // first row position (0-based)
    int32_t gfirst;      // first segment of this segment's group (in the row's table)
    int16_t gcount;      // number of segments in the group
    uint8_t rev;         // 1 = reversed in the row
    uint8_t streams;     // bit s set = query stream s ('+', '-', '*')
    uint8_t multi;       // 1 = group is a GRangesList element (count reads once per range hit)
    uint8_t group;       // group index inside the row (0..3)
    uint8_t query_ok;    // 0 = zero-width query (hits nothing)
    uint8_t pad;
    // multi groups: a read [x, y] of this range overlaps no other range of its group when
    // nb_lo < x and y < nb_hi (nb_lo = INT32_MAX when the group's ranges intersect this one)
    int32_t nb_lo, nb_hi;
};

// Per-row locate input, built with the plan from the row table and the bound readset's stream
// directory offsets: one 80-byte load per row instead of a chain of dependent table loads
// (row_seg -> segs, row_chrom -> dir_off / seqlen).
struct RcpRowInfo {
    int32_t j0, j1;    // segments [j0, j1)
    int32_t chrom;     // chromosome index
    int32_t row_len;   // nominal coverage length nr
    int64_t seqlen;    // seqlengths[chrom] (-1 = NA)
    int64_t d0;        // first directory entry of stream chrom*3 in the plan's layout
    int32_t nb;        // its bucket count
    int32_t stat;      // row_static
    int32_t pad[2];
    RcpSeg seg0;       // segment j0
};
static_assert(sizeof(RcpSeg) == 32 && sizeof(RcpRowInfo) == 80, "RcpRowInfo is five 16-byte words");

// Per-row record the locate kernel leaves for the pileup kernel (one 64-byte load per row
// instead of a chain of dependent loads).  lo/hi are the row's candidate reads per strand
// stream when the row is a single range (flags & RCP_REC_FAST).
struct RcpRowRec {
    int32_t flags;       // RCP_REC_*
    int32_t row_len;     // nominal coverage length nr
    int32_t heavy;       // heavy slot or -1
    int32_t off, slo, shi, rev;  // the single range: row offset, genomic run, reversed
    uint32_t lo[3], hi[3];
    int32_t pad[3];
};
#define RCP_REC_VALID 1
#define RCP_REC_FAST 2
#define RCP_REC_CRANGE 4  // crange holds this row's per-chunk read ranges
#define RCP_MAX_CRANGE_CHUNKS 16

struct RcpPart {
    // slice [lo, hi) of the row (0-based): lo = (lo_end ? nr : 0) + lo_off, same for hi
    int32_t lo_off, hi_off;
    int32_t lo_end, hi_end;
    int32_t n_bins;      // bins (per-base parts: the column count)
    int32_t per_base;    // 1 = per base (bins of one position, no layout)
    int32_t col_off;     // first output column
    int32_t chunk_bins;  // bins per workgroup chunk
    int32_t n_chunks;    // ceil(n_bins / chunk_bins)
    int32_t lay_base;    // offset of this part's dif -> layout index table (n_bins entries)
};

struct RcpPlanDev {
    // reads
    const int2* se;            // sorted (start, end) pairs
    // reads of one width (ChIP-seq fragments extended to fragLen, fixed read lengths): their
    // starts alone, end = start + st_w (the lean kernel streams these; null = not uniform)
    const int32_t* st;
    int32_t st_w;
    const int32_t* pmax;       // prefix max of end inside each stream
    const int64_t* stream_off; // [n_chrom*3 + 1]
    const int64_t* seqlen;     // [n_chrom] (-1 = NA)
    int32_t n_chrom;
    // bucket directory of each stream (buckets of 2^dir_shift bp): for a position v in
    // bucket b, lower_bound(pmax >= v) lies in [dir_l[b], dir_l[b+1]] and
    // upper_bound(start > v) in [dir_u[b], dir_u[b+1]] (entries at dir_off[stream] ..; the two
    // arrays are interleaved, entry e at word 2e of each pointer, dir_u = dir_l + 1)
    const int32_t* dir_l;
    const int32_t* dir_u;
    const int64_t* dir_off;    // [n_chrom*3 + 1]
    // the same directory with each bucket's first keys inline, one 128-byte line per entry e:
    // words 0..15 = dir_l[e], dir_l[e+1], pmax[dir_l[e] + i] (i < 14); words 16..31 = dir_u[e],
    // dir_u[e+1], start[dir_u[e] + i] -- a bound search whose answer lies among a bucket's first
    // 14 reads reads this one line (null = not built)
    const int32_t* dir_k;
    int32_t dir_shift;
    int32_t merged;            // 1: the strand-merged layout (all reads in stream chrom*3)
    // rows
    int32_t n_rows;
    const int32_t* row_chrom;   // [n_rows]
    const int32_t* row_seg;     // [n_rows + 1] into segs
    const int32_t* row_len;     // [n_rows] nominal coverage length nr
    const uint8_t* row_static;  // [n_rows] 1 = statically NULL (negative index, bad chrom)
    const RcpSeg* segs;
    const RcpRowInfo* row_info; // [n_rows]
    // locate outputs
    uint32_t* seg_lo;           // [n_seg * 3]
    uint32_t* seg_hi;           // [n_seg * 3]
    uint8_t* valid;             // [n_rows]
    uint8_t* valid_out;         // [n_rows] or NULL: the caller's validity vector, written by
                                //    locate next to `valid` (no separate device copy per call)
    // bins
    int32_t n_parts;
    RcpPart part[RCP_MAX_PARTS];
    int32_t n_chunks_total;     // sum over parts (workgroups per row tile)
    const int32_t* lay_index;   // per part: [n_bins] dif -> offset into lay_cnt (-1 = none)
    const int32_t* lay_cnt;     // prefix counts of enlarged bins (n_bins + 1 per layout)
    const uint32_t* lay_bit;    // the same as bit masks, word lay + j = bins 32 j .. 32 j + 31 (plans only)
    int32_t stat;               // 0 mean, 1 median
    double scale;
    int64_t n_cols;
    int64_t out_ld;             // column stride of out / binsum in doubles (>= n_rows; rcp_plan_opts.out_ld)
    // interpolation rows
    int32_t n_interp;
    const int32_t* interp_row;  // [n_interp]
    const int32_t* interp_part; // [n_interp]
    const int32_t* interp_mode; // [n_interp] 1 spline, 2 linear (no-op), 3 neighborhood
    const int32_t* interp_pos;  // [n_interp] offset into nb_pos (neighborhood) or -1
    const int32_t* nb_pos;      // orig.pos tables (1-based, sorted)
    // fmm spline elimination on unit knot spacing (R splines.c fmm_spline): the pivots do not
    // depend on the data, so spl_tb[2i] = t_i = 1 / b_{i-1} and spl_tb[2i+1] = b_i (b_0 = -1,
    // b_i = 4 - t_i) are tabulated once on the host, in R's operation order (exact IEEE ops)
    const double* spl_tb;       // [2 * (interp_cap + 1)]
    double* interp_scratch;     // per interp row: 5 * max_interp_len doubles
    int32_t interp_stride;
    int32_t interp_lds;         // byte offset of the row's doubles in LDS, -1 = global scratch (launcher)
    int32_t interp_lds_budget;  // LDS bytes an interpolation block may take so that it runs beside the
                                // persistent pileup workgroups (the rest of a CU's 160 KB); 0 = all
    int32_t interp_stage;       // per execution: the row-wave kernel (HBM stage) piles the interpolated
                                // parts and interpolates them itself (interp_of) -- or, without that
                                // table, stages them in rm32 for rcp_interp_kernel launched after it
    const int32_t* interp_of;   // row-wave plans: [n_rows][n_parts] interpolation entry or -1
    const int32_t* tile_perm;   // row-wave plans with interp_of: the order 16-row tiles are claimed in
    // geometry
    int32_t chunk_cap;          // max positions per chunk (one wave's difference array)
    int32_t wave_words;         // LDS words per wave difference array (multiple of 256)
    int32_t stage_cap;          // max bins per chunk
    int32_t interp_cap;         // max positions of an interpolated slice
    // chunk windows of rows of nominal length cw_len (-1: none), tabulated by the plan:
    // chunk c piles row positions [cw[2c], cw[2c] + cw[2c+1]); cw[2c+1] < 0: not piled
    int32_t cw_len;
    int32_t cw[2 * RCP_MAX_CRANGE_CHUNKS];
    int32_t n_cus;              // compute units of the plan's device (persistent grid sizing)
    int32_t rounds;             // general pileup kernel: rounds of kTile rows per workgroup (1..4;
                                //    fewer for small row tables, so more workgroups fill the chip)
    int32_t lean;               // 1: every row is one plain range with uniform power-of-two bins
                                //    of one wave chunk -> rcp_pileup_lean_kernel
    int32_t lean_rounds;        // lean kernel: rounds of 16 rows per work item (2; else kRounds)
    int32_t fold;               // 1: the pileup kernel searches its rows' read ranges itself and applies
                                //    the NULL rules (no locate / heavy launches; bin-difference plans)
    int32_t coop_min;           // fold plans (general kernel): a fused-bins chunk of a row with more
                                //    candidate reads than this is piled by the whole workgroup
    // lean kernel, heaviest items first (per-base plans of few work items, e.g. one GPU's shard):
    // locate sums each (32-row tile, column chunk) item's candidate reads, files the item code in
    // item_order under its class floor(log2(reads)) (counts in status[kLptClass + class]), and
    // the lean kernel claims items from one counter, highest class first.  0: per-XCD order.
    int32_t lpt;
    int32_t multi_rows;         // 1: some row is a list of ranges (locate's pair loop does the work)
    int32_t grid_fill;          // eighths of the per-CU workgroup slots persistent pileup grids take
    int32_t lpt_cap;            // items per class list (>= the plan's item count)
    int32_t* item_order;        // [RCP_LPT_CLASSES][lpt_cap]
    // row-wave kernel (lean == 3): the bin numerators of its rows are staged (uint32, whole
    // rows) and the last wave to finish a 16-row tile divides them and writes the tile's rows of
    // every column into the R column-major output as whole 128-B lines (a row-wave store
    // straight into the column-major matrix is 8 bytes per 128-B line).  The stage is
    // row-major in HBM: rm32 [n_rows][n_cols] with the rows' part info rinfo [n_rows][8]
    // ({bin width, layout}; width 0: zeros, -1: left to the interpolation kernel)
    uint32_t* rm32;
    int2* rinfo;
    // coverage (CSR) mode
    const int64_t* csr_off;     // non-null: write per-row depth into csr (calcCoverage)
    int32_t* csr_out;
    // non-null (calcCoverage's Rle list without a dense depth array): each (row, column chunk)
    // writes its run starts -- the chunk's first position always, then every position whose
    // depth differs from the one before -- as (depth, row position) to csr_rs at the chunk's
    // dense offset (csr_off[row] + first position), and (starts, last depth) to
    // csr_sub[csr_sub_off[row] + column chunk]; rcp_cov_runs_* merge the seams and compact
    int2* csr_rs;
    int2* csr_sub;
    const int64_t* csr_sub_off;
    // skewed depth: rows with more than heavy_threshold candidate reads are piled up
    // first by many workgroups (heavy slices) into a global difference array
    uint32_t* ncand;            // [n_rows] candidate reads (locate output)
    RcpRowRec* rec;             // [n_rows] (locate output)
    // candidate reads of each (row, column chunk) of a single-range row, per strand stream:
    // [crange[((r * n_chunks_total + c) * 3 + s)].x, .y)  (locate output; null = not kept)
    uint2* crange;
    int32_t heavy_threshold;    // 0 = heavy path off
    int32_t heavy_cap;          // slots
    int32_t heavy_stride;       // ints per slot (>= max row length + 1 of eligible rows)
    int32_t heavy_max_len;      // rows longer than this never take the heavy path
    int32_t heavy_slice;        // candidate reads per heavy work item
    int32_t* heavy_rows;        // [heavy_cap]
    uint32_t* heavy_nslice;     // [heavy_cap] slices of each slot (locate output)
    int32_t* heavy_gdiff;       // [heavy_cap * heavy_stride]; the slots the last execution used
                                //    are cleared by the next one's locate kernel
    // Status words of this execution: status (status[0]), heavy slot counter (status[1]), locate
    // ticket (status[3]), lean work counters (status[8 .. 16]).  Executions alternate between
    // two sets of RCP_STATUS_WORDS words (the plan's epoch parity): an execution's locate kernel
    // reads the previous execution's slot count from status_prev[1], clears those slots, and its
    // last block zeroes status_prev -- the set the next execution uses.  No reset launch.
    uint32_t* status;           // bit 0: numerator overflow, bit 1: per-base width mismatch
    uint32_t* status_prev;
};
#define RCP_STATUS_WORDS 32
#define RCP_LPT_CLASSES 15      // item classes by log2 of their candidate reads (status words 17 ..)
#define RCP_LPT_STATUS 17

__host__ __device__ inline void rcp_part_slice(const RcpPart& p, int32_t nr, int32_t* lo, int32_t* len) {
    *lo = (p.lo_end ? nr : 0) + p.lo_off;
    *len = (p.hi_end ? nr : 0) + p.hi_off - *lo;
}

#define RCP_STATUS_OVERFLOW 1u
#define RCP_STATUS_WIDTH 2u
#define RCP_STATUS_INTERP 4u

#include "rcp_divrn.h"
