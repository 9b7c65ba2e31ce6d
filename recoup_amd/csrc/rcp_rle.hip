// rcp_rle.hip -- profiles of a coverage list given as run-length encoded vectors: the
// reference's own `$coverage` object (a named list of S4Vectors::Rle, R/coverage.R:171-173),
// as binCoverageMatrix / baseCoverageMatrix consume it (R/profile.R:100-212) when recoup()
// reuses a stored coverage (R/recoup.R:126-135) or a sliced object (R/util.R:209-210).
//
// One workgroup per (row, column part) task.  A row's runs are (start, value) pairs with
// row-relative starts from a device scan of the Rle lengths.  Binned parts: one thread per
// bin walks the runs its bin covers -- integer Rle: exact int64 numerator, mean =
// (numerator * scale) / width as the read kernels write it; numeric Rle (a coverage already
// multiplied by a linear normalisation factor, R/recoup.R:559-577): double-double sum of
// value x overlap, then / width; median: bisection over the order-preserving 64-bit keys of
// the bin's values (count of positions <= a key from the runs), R's (a + b) / 2 for even
// widths.  Per-base parts: one thread per column, binary search of its run.  Slices shorter
// than their bin count: the values are expanded and interp_finish (rcp_splitvector.h) runs
// the same spline / neighborhood / "inear" code as the read path.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>

#include "rcp_rle.h"
#include "rcp_splitvector.h"

namespace {

constexpr int kRleBlock = 256;

template <bool DBL>
__device__ __forceinline__ double run_value(const RcpRleDev& P, int64_t j) {
    return DBL ? P.dvals[j] : (double)P.ivals[j];
}

// last run of row r starting at or before row position pos (runs j0 .. j1 - 1, j1 > j0)
__device__ __forceinline__ int64_t run_at(const RcpRleDev& P, int64_t j0, int64_t j1, int32_t pos) {
    int64_t lo = j0, hi = j1;  // first run with start > pos is in (lo, hi]
    while (hi - lo > 1) {
        const int64_t m = lo + ((hi - lo) >> 1);
        if (P.run_start[m] <= pos) lo = m; else hi = m;
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
__device__ uint64_t count_le(const RcpRleDev& P, int64_t j, int64_t j1, int32_t rl, int32_t a, int32_t b, uint64_t kk,
                             double sc) {
    uint64_t c = 0;
    for (; j < j1; ++j) {
        const int32_t s = P.run_start[j];
        if (s >= b) break;
        const int32_t e = j + 1 < j1 ? P.run_start[j + 1] : rl;
        const int32_t lo = max(s, a), hi = min(e, b);
        if (hi > lo && okey(DBL ? run_value<true>(P, j) * sc : run_value<false>(P, j)) <= kk) c += (uint64_t)(hi - lo);
    }
    return c;
}

// k-th smallest (1-based) value of positions [a, b)
template <bool DBL>
__device__ double kth_value(const RcpRleDev& P, int64_t j, int64_t j1, int32_t rl, int32_t a, int32_t b, uint64_t k,
                            double sc) {
    uint64_t lo = ~0ull, hi = 0;
    for (int64_t q = j; q < j1; ++q) {
        const int32_t s = P.run_start[q];
        if (s >= b) break;
        const int32_t e = q + 1 < j1 ? P.run_start[q + 1] : rl;
        if (min(e, b) <= max(s, a)) continue;
        const uint64_t kk = okey(DBL ? run_value<true>(P, q) * sc : run_value<false>(P, q));
        lo = min(lo, kk);
        hi = max(hi, kk);
    }
    while (lo < hi) {  // smallest key with count(<= key) >= k
        const uint64_t m = lo + ((hi - lo) >> 1);
        if (count_le<DBL>(P, j, j1, rl, a, b, m, sc) >= k) hi = m; else lo = m + 1;
    }
    return okey_value(lo);
}

template <bool DBL>
__global__ void __launch_bounds__(kRleBlock) rcp_rle_profile_kernel(RcpRleDev P) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const RcpRleTask t = P.tasks[blockIdx.x];
    const int r = t.row;
    const int32_t ncol = P.part_cols[t.part];
    double* o = P.out + (size_t)P.part_col0[t.part] * (size_t)P.ld + (size_t)r;
    const size_t ld = (size_t)P.ld;
    const double sc = P.scale;
    if (t.mode == RCP_RLE_ZERO) {
        for (int k = threadIdx.x; k < ncol; k += kRleBlock) o[(size_t)k * ld] = 0.0;
        return;
    }
    const int64_t j0 = P.run_off[r], j1 = P.run_off[r + 1];
    const int32_t rl = P.row_len[r];
    if (t.mode == RCP_RLE_BASE) {
        for (int k = threadIdx.x; k < ncol; k += kRleBlock) {
            const int64_t j = run_at(P, j0, j1, t.head + k);
            o[(size_t)k * ld] = DBL ? run_value<true>(P, j) * sc : run_value<false>(P, j) * sc;
        }
        return;
    }
    if (t.mode == RCP_RLE_BINNED) {
        const int32_t* cnt = t.lay >= 0 ? P.lay_cnt + t.lay : nullptr;
        for (int k = threadIdx.x; k < ncol; k += kRleBlock) {
            const int32_t a = t.head + t.bs * k + (cnt ? cnt[k] : 0);
            const int32_t w = t.bs + (cnt ? cnt[k + 1] - cnt[k] : 0);
            const int32_t b = a + w;
            const int64_t js = run_at(P, j0, j1, a);
            double v;
            if (P.stat == 0) {  // mean
                if (DBL) {
                    double hi = 0.0, lo = 0.0;  // double-double sum of (value * scale) x overlap
                    for (int64_t j = js; j < j1; ++j) {
                        const int32_t s = P.run_start[j];
                        if (s >= b) break;
                        const int32_t e = j + 1 < j1 ? P.run_start[j + 1] : rl;
                        const double x = run_value<true>(P, j) * sc;
                        const double m = (double)(min(e, b) - max(s, a));
                        const double p = x * m, pe = __fma_rn(x, m, -p);
                        const double s1 = hi + p, bb = s1 - hi, se = (hi - (s1 - bb)) + (p - bb);
                        hi = s1;
                        lo += se + pe;
                    }
                    v = (hi + lo) / (double)w;
                } else {
                    int64_t num = 0;
                    for (int64_t j = js; j < j1; ++j) {
                        const int32_t s = P.run_start[j];
                        if (s >= b) break;
                        const int32_t e = j + 1 < j1 ? P.run_start[j + 1] : rl;
                        num += (int64_t)P.ivals[j] * (int64_t)(min(e, b) - max(s, a));
                    }
                    v = ((double)num * sc) / (double)w;
                }
            } else {  // median: the middle value, or the mean of the two middle values
                const uint64_t h = (uint64_t)(w + 1) >> 1;
                const double x1 = kth_value<DBL>(P, js, j1, rl, a, b, h, sc);
                const double x2 = (w & 1) ? x1 : kth_value<DBL>(P, js, j1, rl, a, b, h + 1, sc);
                v = DBL ? (x1 + x2) / 2.0 : ((x1 + x2) * sc) / 2.0;
            }
            o[(size_t)k * ld] = v;
        }
        return;
    }
    // interpolation (length(x) < n): expand x = as.numeric(slice) * scale, then splitVector
    const int L = t.L, n = ncol;
    double* x = P.interp_lds ? reinterpret_cast<double*>(smem) : P.scratch + (size_t)t.scratch * (size_t)P.interp_stride;
    for (int i = threadIdx.x; i < L; i += kRleBlock) {
        const int64_t j = run_at(P, j0, j1, t.head + i);
        x[i] = DBL ? run_value<true>(P, j) * sc : run_value<false>(P, j) * sc;
    }
    __syncthreads();
    interp_finish(t.mode - RCP_RLE_INTERP, L, n, x, t.nbpos >= 0 ? P.nb_pos + t.nbpos : nullptr, P.spl_tb, o, ld);
}

// run_start: row-relative starts from the global exclusive scan of the lengths; row_len: the
// sum of a row's lengths
__global__ void rcp_rle_starts_kernel(int32_t n_rows, const int64_t* __restrict__ run_off,
                                      const int64_t* __restrict__ gstart, int32_t* __restrict__ run_start,
                                      int32_t* __restrict__ row_len) {
    const int r = blockIdx.x;
    const int64_t j0 = run_off[r], j1 = run_off[r + 1];
    const int64_t base = gstart[j0];
    for (int64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) run_start[j] = (int32_t)(gstart[j] - base);
    if (threadIdx.x == 0) row_len[r] = (int32_t)(gstart[j1] - base);
}

}  // namespace

extern "C" hipError_t rcp_rle_scan(const int32_t* lengths, int64_t n_runs, int64_t* gstart, void* temp,
                                   size_t* temp_bytes, hipStream_t stream) {
    // exclusive scan of n_runs + 1 entries (the last input is a 0 pad), int32 -> int64
    hipcub::TransformInputIterator<int64_t, hipcub::CastOp<int64_t>, const int32_t*> in(lengths, hipcub::CastOp<int64_t>());
    return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, in, gstart, (int)(n_runs + 1), stream);
}

extern "C" hipError_t rcp_rle_starts(int32_t n_rows, const int64_t* run_off, const int64_t* gstart, int32_t* run_start,
                                     int32_t* row_len, hipStream_t stream) {
    if (n_rows == 0) return hipSuccess;
    hipLaunchKernelGGL(rcp_rle_starts_kernel, dim3((unsigned)n_rows), dim3(kRleBlock), 0, stream, n_rows, run_off,
                       gstart, run_start, row_len);
    return hipGetLastError();
}

extern "C" hipError_t rcp_rle_profile_launch(const RcpRleDev* P, int dbl, size_t lds, hipStream_t stream) {
    if (P->n_tasks == 0) return hipSuccess;
    const void* fn = dbl ? reinterpret_cast<const void*>(rcp_rle_profile_kernel<true>)
                         : reinterpret_cast<const void*>(rcp_rle_profile_kernel<false>);
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    if (dbl)
        hipLaunchKernelGGL(rcp_rle_profile_kernel<true>, dim3((unsigned)P->n_tasks), dim3(kRleBlock), lds, stream, *P);
    else
        hipLaunchKernelGGL(rcp_rle_profile_kernel<false>, dim3((unsigned)P->n_tasks), dim3(kRleBlock), lds, stream, *P);
    return hipGetLastError();
}
