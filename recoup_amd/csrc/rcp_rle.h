// rcp_rle.h -- device tables of the Rle-input profile (rcp_rle.hip, rcp_profile_rle in
// rcp_host.cpp): one task per (row, column part), part-major.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rcp_device.h"

enum {
    RCP_RLE_ZERO = 0,    // NULL list element -> rep(0, ...) (profile.R:116-122, :191-197)
    RCP_RLE_BASE = 1,    // per-base part (baseCoverageMatrix)
    RCP_RLE_BINNED = 2,  // splitVector bins (uniform or R-RNG layout)
    RCP_RLE_INTERP = 3   // + 1 spline, + 2 "inear" (no-op), + 3 neighborhood (interp_finish modes)
};

struct RcpRleTask {
    int32_t row, part;
    int32_t head;    // first row position of the part's slice
    int32_t L;       // slice length
    int32_t mode;    // RCP_RLE_*
    int32_t bs;      // floor(L / n)
    int32_t lay;     // offset of the R-RNG layout prefix counts in lay_cnt, -1 = uniform bins
    int32_t nbpos;   // neighborhood positions (offset in nb_pos), -1 = none
    int32_t scratch; // interpolation scratch slot (global scratch), -1 = none
    int32_t pad;
};

struct RcpRleDev {
    const int64_t* run_off;    // [n_rows + 1]
    const int64_t* gstart;     // [n_runs + 1] exclusive scan of the run lengths (row r's
                               // positions start at gstart[run_off[r]]); null: starts are formed
                               // from the lengths in the tile kernel (slices start at position 0)
    const int32_t* lengths;    // [n_runs] run lengths
    const int32_t* ivals;      // integer Rle values or null
    const double* dvals;       // numeric Rle values or null
    const RcpRleTask* tasks;   // [n_parts][n_rows]
    int32_t n_rows, n_parts;
    const RcpRleTask* itasks;  // the interpolation tasks (rcp_rle_interp_kernel)
    int64_t n_itasks;
    const int32_t* lay_cnt;
    const int32_t* nb_pos;
    const double* spl_tb;      // fmm pivots (rcp_splitvector.h)
    double* out;               // column-major, stride ld
    int64_t ld;
    int32_t part_col0[RCP_MAX_PARTS];
    int32_t part_cols[RCP_MAX_PARTS];
    int32_t part_dense[RCP_MAX_PARTS];  // 1: every row of the part takes the dense-window tile path
    int32_t stat;              // 0 mean, 1 median
    double scale;
    double* scratch;           // interpolation rows whose working set exceeds LDS
    int64_t interp_stride;     // doubles per scratch slot
    int32_t interp_lds;        // 1: interpolation working set in dynamic LDS
};

extern "C" {
hipError_t rcp_rle_scan(const int32_t* lengths, int64_t n_runs, int64_t* gstart, void* temp, size_t* temp_bytes,
                        hipStream_t stream);
hipError_t rcp_rle_profile_launch(const RcpRleDev* P, int dbl, size_t lds, hipStream_t stream);
// the profile's means as uint32 numerators + per-row bin widths (flag set: not expressible)
hipError_t rcp_rle_pack(const RcpRleDev* P, int64_t n_cols, uint32_t* q_out, uint32_t* div, uint32_t* flag,
                        hipStream_t stream);
// row lengths and run-length checks of an Rle list (bad[2]: first row with a length <= 0 / with
// 2^31 or more positions, preset to INT32_MAX)
hipError_t rcp_rle_rowlen(int32_t R, const int64_t* run_off, const int32_t* lengths, int32_t* row_len, int32_t* bad,
                          hipStream_t stream);
}
