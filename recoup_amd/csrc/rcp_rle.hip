// rcp_rle.hip -- profiles of a coverage list given as run-length encoded vectors: the
// reference's own `$coverage` object (a named list of S4Vectors::Rle, R/coverage.R:171-173),
// as binCoverageMatrix / baseCoverageMatrix consume it (R/profile.R:100-212) when recoup()
// reuses a stored coverage (R/recoup.R:126-135) or a sliced object (R/util.R:209-210), and as
// recoup()'s own profileMatrix step reads the coverage calcCoverage just returned
// (R/recoup.R:551-597; saveParams$coverage = TRUE by default, R/util.R:459-461).
//
// Tile kernel (rcp_rle_tile_kernel): one workgroup of 4 waves per (column part, 16-row tile);
// the part's columns are walked in chunks of 128.  Each wave owns 4 of the tile's rows and
// streams the runs that cover a chunk's positions in batches of 128 (coalesced (start, value)
// loads into the wave's LDS); every lane then takes two of the chunk's columns and adds, for
// each run its bin overlaps, value x overlap (integer Rle: exact int64 numerator, mean =
// (numerator * scale) / width as the read kernels write it; numeric Rle -- a coverage already
// multiplied by a linear normalisation factor, R/recoup.R:559-577 -- the exact sum as a
// double-double, divided once with a remainder correction) or, per base, takes the value of
// the one run covering its position.  A run cursor per row carries over from chunk to chunk,
// so each run is loaded about once.  Results go to an LDS stage [16 rows][128 columns] that
// the whole workgroup writes as 128-B column segments (16 rows x 8 B) of the R column-major
// matrix.  Median bins: per-bin bisection over the order-preserving 64-bit keys of the bin's
// run values (count of positions <= a key from the runs), R's (a + b) / 2 for even widths.
// Slices shorter than their bin count (interpolation, R/util.R:17-73) are finished by a
// second launch (rcp_rle_interp_kernel): the values are expanded and interp_finish
// (rcp_splitvector.h) runs the same spline / neighborhood / "inear" code as the read path.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>

#include <type_traits>

#include "rcp_rle.h"
#include "rcp_splitvector.h"

namespace {

constexpr int kRleBlock = 256;

template <bool DBL>
__device__ __forceinline__ double run_value(const RcpRleDev& P, int64_t j) {
    return DBL ? P.dvals[j] : (double)P.ivals[j];
}

// row-relative start of run j (base = gstart[run_off[r]]); run j1 "starts" at the row length
__device__ __forceinline__ int32_t rstart(const RcpRleDev& P, int64_t j, int64_t base) {
    return (int32_t)(P.gstart[j] - base);
}

// last run of row r starting at or before row position pos (runs j0 .. j1 - 1, j1 > j0)
__device__ __forceinline__ int64_t run_at(const RcpRleDev& P, int64_t j0, int64_t j1, int32_t pos) {
    const int64_t base = P.gstart[j0];
    int64_t lo = j0, hi = j1;  // first run with start > pos is in (lo, hi]
    while (hi - lo > 1) {
        const int64_t m = lo + ((hi - lo) >> 1);
        if (rstart(P, m, base) <= pos) lo = m; else hi = m;
    }
    return lo;
}

__device__ __forceinline__ uint64_t okey(double v) {  // order-preserving key of a double
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double okey_value(uint64_t k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
}

// positions of [a, b) (row coordinates) whose value's key is <= kk
template <bool DBL>
__device__ uint64_t count_le(const RcpRleDev& P, int64_t j, int64_t j1, int64_t base, int32_t a, int32_t b,
                             uint64_t kk, double sc) {
    uint64_t c = 0;
    for (; j < j1; ++j) {
        const int32_t s = rstart(P, j, base);
        if (s >= b) break;
        const int32_t e = rstart(P, j + 1, base);
        const int32_t lo = max(s, a), hi = min(e, b);
        if (hi > lo && okey(DBL ? run_value<true>(P, j) * sc : run_value<false>(P, j)) <= kk) c += (uint64_t)(hi - lo);
    }
    return c;
}

// k-th smallest (1-based) value of positions [a, b)
template <bool DBL>
__device__ double kth_value(const RcpRleDev& P, int64_t j, int64_t j1, int64_t base, int32_t a, int32_t b, uint64_t k,
                            double sc) {
    uint64_t lo = ~0ull, hi = 0;
    for (int64_t q = j; q < j1; ++q) {
        const int32_t s = rstart(P, q, base);
        if (s >= b) break;
        const int32_t e = rstart(P, q + 1, base);
        if (min(e, b) <= max(s, a)) continue;
        const uint64_t kk = okey(DBL ? run_value<true>(P, q) * sc : run_value<false>(P, q));
        lo = min(lo, kk);
        hi = max(hi, kk);
    }
    while (lo < hi) {  // smallest key with count(<= key) >= k
        const uint64_t m = lo + ((hi - lo) >> 1);
        if (count_le<DBL>(P, j, j1, base, a, b, m, sc) >= k) hi = m; else lo = m + 1;
    }
    return okey_value(lo);
}

// interpolation tasks (length(x) < n): expand x = as.numeric(slice) * scale, then splitVector.
// Runs after the tile kernel, which leaves these rows' columns to it.
template <bool DBL>
__global__ void __launch_bounds__(kRleBlock) rcp_rle_interp_kernel(RcpRleDev P) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const RcpRleTask t = P.itasks[blockIdx.x];
    const int r = t.row;
    double* o = P.out + (size_t)P.part_col0[t.part] * (size_t)P.ld + (size_t)r;
    const size_t ld = (size_t)P.ld;
    const double sc = P.scale;
    const int64_t j0 = P.run_off[r], j1 = P.run_off[r + 1];
    const int L = t.L, n = P.part_cols[t.part];
    double* x = P.interp_lds ? reinterpret_cast<double*>(smem) : P.scratch + (size_t)t.scratch * (size_t)P.interp_stride;
    for (int i = threadIdx.x; i < L; i += kRleBlock) {
        const int64_t j = run_at(P, j0, j1, t.head + i);
        x[i] = DBL ? run_value<true>(P, j) * sc : run_value<false>(P, j) * sc;
    }
    __syncthreads();
    interp_finish(t.mode - RCP_RLE_INTERP, L, n, x, t.nbpos >= 0 ? P.nb_pos + t.nbpos : nullptr, P.spl_tb, o, ld);
}

constexpr int kRleWpe = 8;  // 8 waves per SIMD: two 16-wave workgroups per CU (<= 64 VGPRs)
constexpr int kTRows = 16;                 // rows per tile: one 128-B line of every column; one wave per row
constexpr int kTBlock = 64 * kTRows;
constexpr int kTCols = 128;                // columns per chunk (2 per lane)
constexpr int kTStride = kTCols + 1;       // doubles per stage row
constexpr int kTBatch = 128;               // runs per batch (2 per lane)
constexpr int kTDense = 512;               // positions of a dense window (2 columns x <= 4 positions per lane)

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return (uint32_t)x;
}

// Workgroup barrier that orders LDS only: __syncthreads() would also wait for vmcnt(0) on gfx9,
// i.e. for the next chunk's prefetched runs and for every output store of the tile
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ void wave_lds_order() {
    // a wave's LDS operations complete in issue order; keep the compiler from moving them
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// last run j of [j0, j1) with start <= pos (run j0 starts at 0 <= pos): a 64-ary search, one
// load per lane per round (two rounds for up to 4096 runs)
__device__ __forceinline__ int64_t wave_run_search(const RcpRleDev& P, int64_t j0, int64_t j1, int64_t base,
                                                   int32_t pos) {
    const int lane = threadIdx.x & 63;
    int64_t lo = j0, n = j1 - j0;
    while (n > 1) {
        const int64_t step = (n + 63) >> 6;
        const int64_t idx = lo + (int64_t)lane * step;
        const bool f = idx < lo + n && rstart(P, idx, base) <= pos;
        const int c = __popcll(__ballot(f));  // a prefix of the lanes (lane 0 always)
        const int64_t nlo = lo + (int64_t)(c - 1) * step;
        n = min(step, lo + n - nlo);
        lo = nlo;
    }
    return lo;
}

// first row position of column c of a binned (RCP_RLE_BINNED) task
__device__ __forceinline__ int32_t bin_lo(const RcpRleTask& t, const int32_t* cnt, int32_t c) {
    return t.head + t.bs * c + (cnt ? cnt[c] : 0);
}

// double-double accumulation of x * m (exact product via its FMA error term)
__device__ __forceinline__ void dd_add_prod(double& hi, double& lo, double x, double m) {
    const double p = x * m, pe = __fma_rn(x, m, -p);
    const double s1 = hi + p, bb = s1 - hi, se = (hi - (s1 - bb)) + (p - bb);
    hi = s1;
    lo += se + pe;
}
// (hi + lo) / w with one remainder correction: the quotient of the exact sum, rounded once
// (R: long-double sum, / n, long-double correction, rounded to double -- equal but for
// double-rounding ties)
__device__ __forceinline__ double dd_div(double hi, double lo, double w) {
    const double s = hi + lo, se = lo - (s - hi);
    const double q = s / w;
    const double rr = __fma_rn(-q, w, s) + se;
    return q + rr / w;
}

// A batch of runs in registers: runs j + lane and j + 64 + lane (value, and the low word of
// their global start), and the low word of run j + 128's start.  Row-relative starts fit int32,
// so start = (int32)(low word - low word of the row's base): the subtraction waits until the
// batch is used, and the loads stay in flight meanwhile.  LEN (parts whose slices start at the
// row's first position, no interpolation or median rows: the host then skips the scan of the
// lengths): g0 / g1 are the runs' lengths (0 past the row) and the starts are a wave scan of
// them from the batch's first start, when the batch is used.
template <class VT>
struct RunBatch {
    uint32_t g0, g1, g2;
    VT v0, v1;
};

template <bool DBL, bool LEN, class VT>
__device__ __forceinline__ RunBatch<VT> load_batch(const RcpRleDev& P, int64_t j, int64_t j1) {
    // indices clamped instead of branched (no divergent loads): gstart[j1] - base is the row
    // length, and values past the row are never used
    const int lane = threadIdx.x & 63;
    RunBatch<VT> b;
    const int64_t i0 = min(j + lane, j1), i1 = min(j + 64 + lane, j1), i2 = min(j + kTBatch, j1);
    const int64_t c0 = min(i0, j1 - 1), c1 = min(i1, j1 - 1);
    if constexpr (LEN) {
        const uint32_t l0 = (uint32_t)P.lengths[c0], l1 = (uint32_t)P.lengths[c1];
        b.g0 = i0 < j1 ? l0 : 0u;
        b.g1 = i1 < j1 ? l1 : 0u;
        b.g2 = 0;
    } else {
        const uint32_t* g32 = reinterpret_cast<const uint32_t*>(P.gstart);
        b.g0 = g32[2 * i0];
        b.g1 = g32[2 * i1];
        b.g2 = g32[2 * i2];
    }
    if constexpr (DBL) {
        b.v0 = P.dvals[c0];
        b.v1 = P.dvals[c1];
    } else {
        b.v0 = P.ivals[c0];
        b.v1 = P.ivals[c1];
    }
    return b;
}

// the batch's starts into rs[0 .. 128] (row-relative); cst = start of its first run (LEN)
template <bool LEN, class VT>
__device__ __forceinline__ void batch_starts(const RunBatch<VT>& b, uint32_t gbl, int32_t cst, int32_t* rs,
                                             int32_t* s0, int32_t* s1) {
    const int lane = threadIdx.x & 63;
    if constexpr (LEN) {
        const uint32_t i0 = wave_incl_scan(b.g0), i1 = wave_incl_scan(b.g1);
        const int32_t t0 = __builtin_amdgcn_readlane((int)i0, 63), t1 = __builtin_amdgcn_readlane((int)i1, 63);
        *s0 = cst + (int32_t)(i0 - b.g0);
        *s1 = cst + t0 + (int32_t)(i1 - b.g1);
        if (lane == 0) rs[kTBatch] = cst + t0 + t1;
    } else {
        *s0 = (int32_t)(b.g0 - gbl);
        *s1 = (int32_t)(b.g1 - gbl);
        if (lane == 0) rs[kTBatch] = (int32_t)(b.g2 - gbl);
    }
    rs[lane] = *s0;
    rs[lane + 64] = *s1;
}

// KIND 0: means (binned or per base) by per-column searches of the run batch; 1: median bins;
// 2: dense windows (integer Rle; per base, or uniform bins of 1, 2 or 4 positions; the host
// picks it per part when every row of the part qualifies).  LEN: starts from the lengths
// (load_batch).
template <bool DBL, int KIND, bool LEN>
__global__ void __launch_bounds__(kTBlock) __attribute__((amdgpu_waves_per_eu(kRleWpe)))
rcp_rle_tile_kernel(RcpRleDev P, int p) {
    constexpr bool MEDIAN = KIND == 1, DENSE = !DBL && KIND == 2;
    using VT = typename std::conditional<DBL, double, int32_t>::type;
    __shared__ double stage[kTRows * kTStride];
    __shared__ int32_t rs_l[kTRows][kTBatch + 4];
    __shared__ VT rv_l[kTRows][kTBatch];
    // dense windows (integer Rle, per-base or uniform bins of 1, 2 or 4 positions)
    __shared__ __attribute__((aligned(16))) int32_t dn_l[DENSE ? kTRows : 1][DENSE ? kTDense + 4 : 4];
    const int R = P.n_rows;
    const int r0 = blockIdx.x * kTRows;
    const int q = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = r0 + q;
    const int32_t ncol = P.part_cols[p];
    const double sc = P.scale;
    double* obase = P.out + (size_t)P.part_col0[p] * (size_t)P.ld + (size_t)r0;
    double* srow = stage + q * kTStride;
    int32_t* rs = rs_l[q];
    VT* rv = rv_l[q];
    RcpRleTask t;
    if (r < R) {
        t = P.tasks[(size_t)p * R + r];
    } else {
        t = RcpRleTask{};
        t.mode = RCP_RLE_ZERO;
    }
    // ZERO: NULL list element; interpolated rows: the interp launch writes them afterwards
    const bool zero = t.mode == RCP_RLE_ZERO || t.mode >= RCP_RLE_INTERP;
    const bool base = t.mode == RCP_RLE_BASE;
    const bool median = MEDIAN && !base;
    const int64_t j0 = zero ? 0 : P.run_off[r], j1 = zero ? 0 : P.run_off[r + 1];
    const int64_t gb = (zero || LEN) ? 0 : P.gstart[j0];
    const uint32_t gbl = (uint32_t)gb;
    const int32_t* cnt = (!zero && !base && t.lay >= 0) ? P.lay_cnt + t.lay : nullptr;
    // the run containing the next chunk's first position, and its batch (prefetched during the
    // previous chunk's stores)
    // dense window: the runs' value steps scattered into a per-position array, one wave scan,
    // each lane's two adjacent columns summed from registers (no per-column search)
    const int32_t dbs = base ? 1 : t.bs;
    int32_t* dn = dn_l[DENSE ? q : 0];
    int64_t j = 0;
    int32_t cst = 0;  // LEN: start of run j
    RunBatch<VT> nb_regs{};
    const bool streamed = !zero && !median;
    if (streamed) {
        if constexpr (LEN) j = j0;  // every slice starts at position 0: run j0
        else j = wave_run_search(P, j0, j1, gb, base ? t.head : bin_lo(t, cnt, 0));
        nb_regs = load_batch<DBL, LEN, VT>(P, j, j1);
    }
    for (int32_t c0 = 0; c0 < ncol; c0 += kTCols) {
        const int32_t cc = min(kTCols, ncol - c0);
        if (zero) {
            for (int c = lane; c < cc; c += 64) srow[c] = 0.0;
        } else if (median) {  // per-bin bisection over the runs in global memory
            for (int c = lane; c < cc; c += 64) {
                const int32_t a = bin_lo(t, cnt, c0 + c), b = bin_lo(t, cnt, c0 + c + 1);
                const int32_t w = b - a;
                const int64_t js = run_at(P, j0, j1, a);
                const uint64_t h = (uint64_t)(w + 1) >> 1;
                const double x1 = kth_value<DBL>(P, js, j1, gb, a, b, h, sc);
                const double x2 = (w & 1) ? x1 : kth_value<DBL>(P, js, j1, gb, a, b, h + 1, sc);
                srow[c] = DBL ? (x1 + x2) / 2.0 : ((x1 + x2) * sc) / 2.0;
            }
        } else if constexpr (DENSE) {
            const int32_t pa = t.head + dbs * c0, W = dbs * cc, pb = pa + W;
            for (int i = lane; i < (W + 3) >> 2; i += 64) reinterpret_cast<int4*>(dn)[i] = make_int4(0, 0, 0, 0);
            uint32_t carry = 0;  // value of the run before the batch's first run (0 before the window)
            for (;;) {
                int32_t s0, s1;
                batch_starts<LEN>(nb_regs, gbl, cst, rs, &s0, &s1);
                rv[lane] = nb_regs.v0;
                rv[lane + 64] = nb_regs.v1;
                const int n = __popcll(__ballot(s0 < pb)) + __popcll(__ballot(s1 < pb));
                wave_lds_order();
                const int32_t be = min(pb, rs[n]);
                const bool more = be < pb;
                // the next batch: the rest of this window, or the next chunk's first (the run
                // containing pb); in flight while this one is added
                const bool at = more || rs[n] == pb;
                const int64_t jn = at ? j + n : j + n - 1;
                cst = at ? rs[n] : rs[n - 1];
                nb_regs = load_batch<DBL, LEN, VT>(P, jn, j1);
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int k = lane + 64 * u;
                    if (k < n) {
                        const uint32_t v = (uint32_t)rv[k], vp = k ? (uint32_t)rv[k - 1] : carry;
                        dn[max(rs[k], pa) - pa] = (int32_t)(v - vp);  // distinct run starts: plain stores
                    }
                }
                carry = (uint32_t)rv[n - 1];
                wave_lds_order();
                j = jn;
                if (!more) break;
            }
            // lane: positions [2 dbs lane, 2 dbs (lane + 1)) = columns 2 lane, 2 lane + 1
            uint32_t x[8];
            const int32_t* src = dn + 2 * dbs * lane;
            if (dbs == 4) {
                const int4 a = reinterpret_cast<const int4*>(src)[0], b = reinterpret_cast<const int4*>(src)[1];
                x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
            } else if (dbs == 2) {
                const int4 a = reinterpret_cast<const int4*>(src)[0];
                x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = x[5] = x[6] = x[7] = 0;
            } else {
                const int2 a = reinterpret_cast<const int2*>(src)[0];
                x[0] = a.x; x[1] = a.y; x[2] = x[3] = x[4] = x[5] = x[6] = x[7] = 0;
            }
            if (2 * lane >= cc) {  // beyond the window: nothing (the array holds stale steps there)
#pragma unroll
                for (int i = 0; i < 8; ++i) x[i] = 0;
            }
            uint32_t A = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) A += x[i];
            uint32_t d = wave_incl_scan(A) - A;  // value before the lane's first position
            int64_t s0 = 0, s1 = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                d += x[i];
                const int64_t val = (int64_t)(int32_t)d;
                if (i < dbs) s0 += val;
                else if (i < 2 * dbs) s1 += val;
            }
            const double inv = 1.0 / (double)dbs;  // a power of two: x * inv == x / dbs exactly
            if (2 * lane < cc) srow[2 * lane] = ((double)s0 * sc) * inv;
            if (2 * lane + 1 < cc) srow[2 * lane + 1] = ((double)s1 * sc) * inv;
            wave_lds_order();
        } else {
            const int32_t pa = base ? t.head + c0 : bin_lo(t, cnt, c0);
            const int32_t pb = base ? pa + cc : bin_lo(t, cnt, c0 + cc);
            int32_t ca[2], cb[2];  // this lane's columns lane, lane + 64: positions [ca, cb)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int32_t c = lane + 64 * u;
                ca[u] = c < cc ? (base ? pa + c : bin_lo(t, cnt, c0 + c)) : pb;
                cb[u] = c < cc ? (base ? ca[u] + 1 : bin_lo(t, cnt, c0 + c + 1)) : pb;
            }
            int64_t inum[2] = {0, 0};
            double dhi[2] = {0.0, 0.0}, dlo[2] = {0.0, 0.0}, bval[2] = {0.0, 0.0};
            int32_t pos = pa;
            for (;;) {
                // the batch: runs j .. j + 127 and the start of run j + 128
                int32_t s0, s1;
                batch_starts<LEN>(nb_regs, gbl, cst, rs, &s0, &s1);
                rv[lane] = nb_regs.v0;
                rv[lane + 64] = nb_regs.v1;
                const int n = __popcll(__ballot(s0 < pb)) + __popcll(__ballot(s1 < pb));
                wave_lds_order();
                const int32_t be = min(pb, rs[n]);  // this batch covers positions [pos, be)
                const bool more = be < pb;          // then n == 128 and run j + 128 starts at be
                const bool at = more || rs[n] == pb;
                const int64_t jn = at ? j + n : j + n - 1;  // next batch's first run
                cst = at ? rs[n] : rs[n - 1];
                nb_regs = load_batch<DBL, LEN, VT>(P, jn, j1);
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int32_t lo = max(ca[u], pos), hi = min(cb[u], be);
                    if (lo < hi) {
                        int k0 = 0, k1 = n;  // last k with rs[k] <= lo (rs[0] <= pos <= lo)
                        while (k1 - k0 > 1) {
                            const int m = (k0 + k1) >> 1;
                            if (rs[m] <= lo) k0 = m; else k1 = m;
                        }
                        if (base) {
                            bval[u] = (double)rv[k0] * sc;
                        } else {
                            for (int k = k0; k < n; ++k) {
                                const int32_t s = rs[k];
                                if (s >= hi) break;
                                const int32_t m = min(rs[k + 1], hi) - max(s, lo);
                                if constexpr (DBL) dd_add_prod(dhi[u], dlo[u], rv[k] * sc, (double)m);
                                else inum[u] += (int64_t)rv[k] * (int64_t)m;
                            }
                        }
                    }
                }
                wave_lds_order();
                j = jn;
                if (!more) break;
                pos = be;
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int32_t c = lane + 64 * u;
                if (c < cc) {
                    double v;
                    if (base) v = bval[u];
                    else if constexpr (DBL) v = dd_div(dhi[u], dlo[u], (double)(cb[u] - ca[u]));
                    else v = ((double)inum[u] * sc) / (double)(cb[u] - ca[u]);
                    srow[c] = v;
                }
            }
        }
        lds_barrier();
        // 16 lanes per column: 128-B segments of the R column-major matrix (rows r0 .. r0 + 15
        // lie inside the padded leading dimension)
        const int qq = threadIdx.x & (kTRows - 1);
        for (int c = threadIdx.x / kTRows; c < cc; c += kTBlock / kTRows)
            __builtin_nontemporal_store(stage[qq * kTStride + c], obase + (size_t)(c0 + c) * (size_t)P.ld + qq);
        lds_barrier();
    }
}

// Row lengths of an Rle list and its checks (rcp_profile_rle's host pass, on the device for a
// big list): one wave per row sums its run lengths (int64) and takes their minimum; row_len[r] =
// min(sum, INT32_MAX); bad[0] / bad[1] = the first row with a length <= 0 / with 2^31 or more
// positions (atomicMin over rows; the caller presets them to INT32_MAX)
__global__ void __launch_bounds__(256) rcp_rle_rowlen_kernel(int32_t R, const int64_t* __restrict__ run_off,
                                                             const int32_t* __restrict__ lengths,
                                                             int32_t* __restrict__ row_len, int32_t* bad) {
    const int lane = threadIdx.x & 63;
    const int32_t r = (int32_t)((blockIdx.x * 256 + threadIdx.x) >> 6);
    if (r >= R) return;
    int64_t acc = 0;
    int32_t mn = INT32_MAX;
    for (int64_t j = run_off[r] + lane; j < run_off[r + 1]; j += 64) {
        const int32_t v = lengths[j];
        acc += v;
        mn = min(mn, v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        acc += __shfl_xor(acc, o);
        mn = min(mn, __shfl_xor(mn, o));
    }
    if (lane == 0) {
        row_len[r] = (int32_t)min(acc, (int64_t)INT32_MAX);
        if (mn <= 0) atomicMin(&bad[0], r);
        if (acc >= (int64_t(1) << 31)) atomicMin(&bad[1], r);
    }
}

}  // namespace

extern "C" hipError_t rcp_rle_rowlen(int32_t R, const int64_t* run_off, const int32_t* lengths, int32_t* row_len,
                                     int32_t* bad, hipStream_t stream) {
    if (R <= 0) return hipSuccess;
    hipLaunchKernelGGL(rcp_rle_rowlen_kernel, dim3((unsigned)(((int64_t)R * 64 + 255) / 256)), dim3(256), 0, stream, R,
                       run_off, lengths, row_len, bad);
    return hipGetLastError();
}

extern "C" hipError_t rcp_rle_scan(const int32_t* lengths, int64_t n_runs, int64_t* gstart, void* temp,
                                   size_t* temp_bytes, hipStream_t stream) {
    // exclusive scan of n_runs + 1 entries (the last input is a 0 pad), int32 -> int64
    hipcub::TransformInputIterator<int64_t, hipcub::CastOp<int64_t>, const int32_t*> in(lengths, hipcub::CastOp<int64_t>());
    return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, in, gstart, (int)(n_runs + 1), stream);
}

template <bool DBL, int KIND, bool LEN>
static void launch_tiles(const RcpRleDev* P, int p, int64_t grid, hipStream_t stream) {
    hipLaunchKernelGGL((rcp_rle_tile_kernel<DBL, KIND, LEN>), dim3((unsigned)grid), dim3(kTBlock), 0, stream, *P, p);
}

// The numerator download of an integer Rle profile (rcp_pack_kernel's, rcp_kernels.hip): one
// part, mean bins; div[r] = the row's uniform bin width (1 per base, 0 NULL); rows of R-RNG
// layouts or interpolated ones are marked in flag[r] (their doubles are fetched apart)
constexpr int kPackCols = 8;
__global__ void __launch_bounds__(kRleBlock) rcp_rle_pack_kernel(RcpRleDev P, int64_t n_cols, uint32_t* __restrict__ q_out,
                                                               uint32_t* __restrict__ div, uint32_t* __restrict__ flag) {
    const int r = blockIdx.x * kRleBlock + threadIdx.x;
    if (r >= P.ld) return;
    if (r >= P.n_rows) {  // column padding: zeros
        for (int64_t k = (int64_t)blockIdx.y * kPackCols; k < min<int64_t>((int64_t)(blockIdx.y + 1) * kPackCols, n_cols); ++k)
            q_out[k * P.ld + r] = 0u;
        return;
    }
    const RcpRleTask t = P.tasks[r];
    uint32_t bs = 0;
    bool bad = false;
    if (t.mode == RCP_RLE_BASE) bs = 1;
    else if (t.mode == RCP_RLE_BINNED && t.lay < 0 && t.bs > 0) bs = (uint32_t)t.bs;
    else if (t.mode != RCP_RLE_ZERO) bad = true;
    if (blockIdx.y == 0) div[r] = bs;
    const double sc = P.scale;
    const double dd = (double)max(bs, 1u), rdd = 1.0 / dd;
    const bool pow2 = (bs & (bs - 1)) == 0;
    const size_t ld = (size_t)P.ld;
    const int64_t k0 = (int64_t)blockIdx.y * kPackCols;
    for (int64_t k = k0; k < min<int64_t>(k0 + kPackCols, n_cols); ++k) {
        const double v = P.out[k * ld + r];
        uint32_t q = 0;
        if (bs) {
            const double x = rint(v * dd / sc);
            q = (x >= 0.0 && x <= 4294967295.0) ? (uint32_t)x : 0u;
            const double back = pow2 ? ((double)q * sc) * rdd : ((double)q * sc) / dd;
            bad = bad || __double_as_longlong(back) != __double_as_longlong(v);
        } else {
            bad = bad || __double_as_longlong(v) != 0;
        }
        q_out[k * ld + r] = q;
    }
    if (bad) atomicOr(flag + r, 1u);  // (per row: bad_row, as rcp_pack_kernel)
}

extern "C" hipError_t rcp_rle_pack(const RcpRleDev* P, int64_t n_cols, uint32_t* q_out, uint32_t* div, uint32_t* flag,
                                   hipStream_t stream) {
    if (P->n_rows == 0 || n_cols == 0) return hipSuccess;
    const dim3 grid((unsigned)((P->ld + kRleBlock - 1) / kRleBlock), (unsigned)((n_cols + kPackCols - 1) / kPackCols));
    hipLaunchKernelGGL(rcp_rle_pack_kernel, grid, dim3(kRleBlock), 0, stream, *P, n_cols, q_out, div, flag);
    return hipGetLastError();
}

extern "C" hipError_t rcp_rle_profile_launch(const RcpRleDev* P, int dbl, size_t lds, hipStream_t stream) {
    // tiles of every part first (they also zero-fill the interpolated rows' columns), then the
    // interpolation tasks on the same stream
    if (P->n_rows > 0 && P->n_parts > 0) {
        if ((P->ld & (kTRows - 1)) != 0) return hipErrorInvalidValue;  // tiles write whole 16-row segments
        const int64_t grid = (P->n_rows + kTRows - 1) / kTRows;
        const bool len = P->gstart == nullptr;  // starts from the lengths (the host skipped the scan)
        for (int p = 0; p < P->n_parts; ++p) {
            const int kind = (!dbl && P->part_dense[p]) ? 2 : (P->stat == 1 ? 1 : 0);
            if (kind == 1 && len) return hipErrorInvalidValue;  // median bins search the scanned starts
            if (dbl) {
                if (kind == 1) launch_tiles<true, 1, false>(P, p, grid, stream);
                else if (len) launch_tiles<true, 0, true>(P, p, grid, stream);
                else launch_tiles<true, 0, false>(P, p, grid, stream);
            } else if (kind == 2) {
                if (len) launch_tiles<false, 2, true>(P, p, grid, stream);
                else launch_tiles<false, 2, false>(P, p, grid, stream);
            } else if (kind == 1) {
                launch_tiles<false, 1, false>(P, p, grid, stream);
            } else {
                if (len) launch_tiles<false, 0, true>(P, p, grid, stream);
                else launch_tiles<false, 0, false>(P, p, grid, stream);
            }
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    }
    if (P->n_itasks == 0) return hipSuccess;
    const void* fn = dbl ? reinterpret_cast<const void*>(rcp_rle_interp_kernel<true>)
                         : reinterpret_cast<const void*>(rcp_rle_interp_kernel<false>);
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    if (dbl)
        hipLaunchKernelGGL(rcp_rle_interp_kernel<true>, dim3((unsigned)P->n_itasks), dim3(kRleBlock), lds, stream, *P);
    else
        hipLaunchKernelGGL(rcp_rle_interp_kernel<false>, dim3((unsigned)P->n_itasks), dim3(kRleBlock), lds, stream, *P);
    return hipGetLastError();
}
