// rcp_shard.hip -- gfx950 kernels of the multi-GPU read split (rcp_shard.cpp).
//
// The reference parallelises calcCoverage over regions with cmclapply (R/coverage.R:147-154,
// R/util.R:364-382); here the regions are cut into one row block per GPU and each GPU holds
// only the reads its block's regions can overlap.  Two kernels serve that split:
//   rcp_seg_bounds_kernel  per (mask range, strand stream): the candidate reads
//                          [lower_bound(prefix max of end >= start), upper_bound(start <= end))
//                          of a sorted layout -- the bounds the locate kernel searches, so every
//                          read findOverlaps would hit (R/coverage.R:189-192) lies inside
//   rcp_gather_kernel      the reads of a list of such index ranges, written out as the
//                          (chromosome, start, end, strand) arrays a readset is built from
// Both are integer work over sorted arrays: one thread per query / per output read, no LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kB = 256;

__device__ __forceinline__ uint32_t lb_pmax(const int32_t* __restrict__ pmax, uint32_t lo, uint32_t hi, int32_t v) {
    while (lo < hi) {  // first index with pmax >= v (pmax is non-decreasing inside a stream)
        const uint32_t m = lo + ((hi - lo) >> 1);
        if (pmax[m] < v) lo = m + 1; else hi = m;
    }
    return lo;
}

__device__ __forceinline__ uint32_t ub_start(const int2* __restrict__ se, uint32_t lo, uint32_t hi, int32_t v) {
    while (lo < hi) {  // first index with start > v
        const uint32_t m = lo + ((hi - lo) >> 1);
        if (se[m].x <= v) lo = m + 1; else hi = m;
    }
    return lo;
}

}  // namespace

// Thread t: mask range j = t / 3, stream slot k = t % 3 of its chromosome c (stream c * 3 + k).
// merged: every strand lives in slot 0; else slot k holds strand k and the range searches the
// slots findOverlaps' strand compatibility allows ('*' matches everything).  A range the locate
// kernel never searches (absent chromosome, end < start) gets [0, 0).  The range searched is
// [max(start, 1), end]: R drops index 0 (rcp_host.cpp build_rows).
__global__ void __launch_bounds__(kB) rcp_seg_bounds_kernel(int64_t n_seg, const int32_t* __restrict__ chrom,
                                                            const int32_t* __restrict__ start,
                                                            const int32_t* __restrict__ end,
                                                            const int8_t* __restrict__ strand, int merged,
                                                            int32_t n_chrom, const int64_t* __restrict__ stream_off,
                                                            const int32_t* __restrict__ pmax,
                                                            const int2* __restrict__ se, uint2* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (t >= 3 * n_seg) return;
    const int64_t j = t / 3;
    const int k = (int)(t - 3 * j);
    const int32_t c = chrom[j], s = max(start[j], 1), e = end[j];
    bool use = c >= 0 && c < n_chrom && e >= s;
    if (merged) {
        use = use && k == 0;
    } else {
        const int q = strand[j];
        const uint32_t mask = (q == 2 || q < 0 || q > 2) ? 7u : ((1u << q) | 4u);
        use = use && ((mask >> k) & 1u);
    }
    uint2 r = make_uint2(0u, 0u);
    if (use) {
        const int64_t sid = (int64_t)c * 3 + k;
        const uint32_t so = (uint32_t)stream_off[sid], eo = (uint32_t)stream_off[sid + 1];
        const uint32_t lo = lb_pmax(pmax, so, eo, s);
        r = make_uint2(lo, max(lo, ub_start(se, lo, eo, e)));
    }
    out[t] = r;
}

// Output read i of the range list: range k with out_off[k] <= i < out_off[k + 1] (bisection over
// the ranges), layout index lo[k] + (i - out_off[k]); its stream sid[k] gives the chromosome
// (sid / 3) and, in a strand-split layout, the strand (sid % 3).  strand_out may be null (merged
// layouts: the receiver marks every read '*', which ignore.strand = TRUE never reads).
__global__ void __launch_bounds__(kB) rcp_gather_kernel(int64_t n_out, int64_t n_ranges,
                                                        const int64_t* __restrict__ out_off,
                                                        const uint32_t* __restrict__ lo,
                                                        const int32_t* __restrict__ sid,
                                                        const int2* __restrict__ se, int32_t* __restrict__ chrom_out,
                                                        int32_t* __restrict__ start_out, int32_t* __restrict__ end_out,
                                                        int8_t* __restrict__ strand_out) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= n_out) return;
    int64_t a = 0, b = n_ranges;  // last range with out_off <= i
    while (b - a > 1) {
        const int64_t m = (a + b) >> 1;
        if (out_off[m] <= i) a = m; else b = m;
    }
    const int2 rd = se[(int64_t)lo[a] + (i - out_off[a])];
    const int32_t st = sid[a];
    chrom_out[i] = st / 3;
    start_out[i] = rd.x;
    end_out[i] = rd.y;
    if (strand_out) strand_out[i] = (int8_t)(st % 3);
}

extern "C" hipError_t rcp_launch_seg_bounds(int64_t n_seg, const int32_t* chrom, const int32_t* start,
                                            const int32_t* end, const int8_t* strand, int merged, int32_t n_chrom,
                                            const int64_t* stream_off, const int32_t* pmax, const int2* se, uint2* out,
                                            hipStream_t stream) {
    if (n_seg <= 0) return hipSuccess;
    const int64_t grid = (3 * n_seg + kB - 1) / kB;
    hipLaunchKernelGGL(rcp_seg_bounds_kernel, dim3((unsigned)grid), dim3(kB), 0, stream, n_seg, chrom, start, end,
                       strand, merged, n_chrom, stream_off, pmax, se, out);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_gather(int64_t n_out, int64_t n_ranges, const int64_t* out_off, const uint32_t* lo,
                                        const int32_t* sid, const int2* se, int32_t* chrom_out, int32_t* start_out,
                                        int32_t* end_out, int8_t* strand_out, hipStream_t stream) {
    if (n_out <= 0) return hipSuccess;
    const int64_t grid = (n_out + kB - 1) / kB;
    hipLaunchKernelGGL(rcp_gather_kernel, dim3((unsigned)grid), dim3(kB), 0, stream, n_out, n_ranges, out_off, lo, sid,
                       se, chrom_out, start_out, end_out, strand_out);
    return hipGetLastError();
}
