// rcp_kernels.hip -- gfx950 (CDNA4) kernels of the coverage -> profile hot path.
//
// What they compute (reference semantics):
//   rcp_locate_kernel   findOverlaps() per region / range / strand stream, plus the
//                       NULL rules of coverageFromRanges (R/coverage.R:189-225)
//   rcp_pileup_kernel   coverage(reads)[i2k] (+ rev for '-')  ->  splitVector bins ->
//                       mean / median (R/util.R:74-84) for a tile of rows, written as the
//                       R column-major profile matrix (R/profile.R:153-212, :100-151)
//   rcp_interp_kernel   rows with fewer positions than bins: stats::spline "fmm",
//                       neighborhood fill, or the "inear" no-op (R/util.R:17-73)
//   readset kernels     splitBySeqname as a (chromosome, strand) stream index with a
//                       prefix-max-of-end array for exact overlap search
//
// Design: integer interval counting, HBM-bound, no MFMA.  Each workgroup owns
// T consecutive rows x one column chunk.  Reads of a row are streamed coalesced as 8-byte
// (start, end) pairs from HBM into +w/-w LDS atomics on a difference array; a two-level
// block scan turns it into depth and cumulative depth (uint32, modular: any bin sum that
// fits 32 bits comes out exact), so each bin is two LDS reads; numerators are staged in
// LDS as [bin][row] so the epilogue writes 16 consecutive rows of a column (128 B) per
// 16 lanes of the R column-major matrix.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "rcp_device.h"

namespace {

constexpr int kBlock = RCP_BLOCK;
constexpr int kWaves = kBlock / 64;

__device__ __forceinline__ uint32_t lower_bound_pmax(const int32_t* __restrict__ pmax, uint32_t lo,
                                                     uint32_t hi, int32_t v) {
    // first index in [lo, hi) with pmax >= v (pmax is non-decreasing inside a stream)
    while (lo < hi) {
        uint32_t m = lo + ((hi - lo) >> 1);
        if (pmax[m] < v) lo = m + 1; else hi = m;
    }
    return lo;
}

__device__ __forceinline__ uint32_t upper_bound_start(const int2* __restrict__ se, uint32_t lo,
                                                      uint32_t hi, int32_t v) {
    // first index in [lo, hi) with start > v
    while (lo < hi) {
        uint32_t m = lo + ((hi - lo) >> 1);
        if (se[m].x <= v) lo = m + 1; else hi = m;
    }
    return lo;
}

// Block-wide exclusive scan of one uint32 per thread.  `scratch` holds kWaves words.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* scratch) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) scratch[wave] = x;
    __syncthreads();
    uint32_t off = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w)
        if (w < wave) off += scratch[w];
    return off + x - v;
}

// ---------------------------------------------------------------------------------
// Pile the candidate reads of row r over row positions [P0, P0 + npos) into the LDS
// difference array `diff` (npos + 1 used words, zeroed by the caller).  Returns the number
// of candidate reads seen (identical in every thread) for the overflow bound.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void pileup_rows_segments(const RcpPlanDev& P, int r, int32_t P0,
                                                     int32_t npos, int32_t* diff) {
    const int tid = threadIdx.x;
    const int32_t P1 = P0 + npos;
    const int j0 = P.row_seg[r], j1 = P.row_seg[r + 1];
    for (int j = j0; j < j1; ++j) {
        const RcpSeg sg = P.segs[j];
        const int32_t len = sg.hi - sg.lo + 1;
        const int32_t a = max(P0, sg.off);
        const int32_t b = min(P1, sg.off + len);
        if (a >= b || !sg.query_ok) continue;
        const bool full = (a == sg.off) && (b == sg.off + len);
        int32_t gps, gpe;  // genomic piece
        if (!sg.rev) {
            gps = sg.lo + (a - sg.off);
            gpe = sg.lo + (b - 1 - sg.off);
        } else {
            gpe = sg.hi - (a - sg.off);
            gps = sg.hi - (b - 1 - sg.off);
        }
        for (int s = 0; s < 3; ++s) {
            if (!((sg.streams >> s) & 1)) continue;
            uint32_t lo = P.seg_lo[j * 3 + s];
            uint32_t hi = P.seg_hi[j * 3 + s];
            if (lo >= hi) continue;
            if (!full) {
                lo = lower_bound_pmax(P.pmax, lo, hi, gps);
                hi = upper_bound_start(P.se, lo, hi, gpe);
            }
            for (uint32_t idx = lo + tid; idx < hi; idx += kBlock) {
                const int2 rd = P.se[idx];
                if (rd.y < gps) continue;
                int32_t w = 1;
                if (sg.multi) {
                    // subjectHits repeats a read once per range of the list it overlaps
                    // (R/coverage.R:190-192): weight = number of overlapped ranges.
                    w = 0;
                    for (int g = sg.gfirst; g < sg.gfirst + sg.gcount; ++g) {
                        const RcpSeg o = P.segs[g];
                        w += (o.query_ok && o.lo <= rd.y && o.hi >= rd.x) ? 1 : 0;
                    }
                }
                const int32_t x0 = max(rd.x, gps);
                const int32_t x1 = min(rd.y, gpe);
                int32_t o0, o1;
                if (!sg.rev) {
                    o0 = sg.off + (x0 - sg.lo);
                    o1 = sg.off + (x1 - sg.lo);
                } else {
                    o0 = sg.off + (sg.hi - x1);
                    o1 = sg.off + (sg.hi - x0);
                }
                atomicAdd(&diff[o0 - P0], w);
                atomicAdd(&diff[o1 - P0 + 1], -w);
            }
        }
    }
}

// Turn diff[0 .. 256*per) into depth (CUM = false) or cumulative depth (CUM = true).
// `per` is a multiple of 4.  scratch: 2*kWaves words.
template <bool CUM>
__device__ __forceinline__ void scan_chunk(int32_t* diff, int per, uint32_t* scratch) {
    const int tid = threadIdx.x;
    uint32_t* base = reinterpret_cast<uint32_t*>(diff) + tid * per;
    uint32_t A = 0, B = 0;  // sum of diff, sum of local depth prefix
    for (int q = 0; q < per; q += 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(base + q);
        A += v.x; B += A;
        A += v.y; B += A;
        A += v.z; B += A;
        A += v.w; B += A;
    }
    const uint32_t D = block_exclusive_scan(A, scratch);  // depth entering this thread
    uint32_t C = 0;
    if (CUM) C = block_exclusive_scan((uint32_t)per * D + B, scratch + kWaves);
    uint32_t l = D, c = C;
    for (int q = 0; q < per; q += 4) {
        uint4 v = *reinterpret_cast<const uint4*>(base + q);
        uint4 o;
        l += v.x; c += l; o.x = CUM ? c : l;
        l += v.y; c += l; o.y = CUM ? c : l;
        l += v.z; c += l; o.z = CUM ? c : l;
        l += v.w; c += l; o.w = CUM ? c : l;
        *reinterpret_cast<uint4*>(base + q) = o;
    }
}

__device__ __forceinline__ int32_t bin_edge(int32_t bs, int32_t lay, const int32_t* __restrict__ cnt,
                                            int32_t k) {
    return bs * k + (lay >= 0 ? cnt[lay + k] : 0);
}

// k-th smallest (1-based) of depth[a .. b) by bisection on the value (depth is >= 0).
__device__ __forceinline__ uint32_t kth_smallest(const int32_t* d, int32_t a, int32_t b, int32_t k,
                                                 int32_t vmin, int32_t vmax) {
    int32_t lo = vmin, hi = vmax;
    while (lo < hi) {
        const int32_t mid = lo + ((hi - lo) >> 1);
        int32_t c = 0;
        for (int32_t q = a; q < b; ++q) c += d[q] <= mid;
        if (c >= k) hi = mid; else lo = mid + 1;
    }
    return (uint32_t)lo;
}

}  // namespace

// =================================================================================
// readset construction
// =================================================================================
__global__ void rcp_make_keys_kernel(int64_t n, const int32_t* __restrict__ chrom,
                                     const int32_t* __restrict__ start, const int32_t* __restrict__ end,
                                     const int8_t* __restrict__ strand, int32_t n_chrom, int32_t strand_filter,
                                     uint64_t* __restrict__ keys, int32_t* __restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t st = strand[i];
    const int32_t c = chrom[i];
    uint32_t sid;
    if ((strand_filter >= 0 && st != strand_filter) || c < 0 || c >= n_chrom || st < 0 || st > 2)
        sid = (uint32_t)n_chrom * 3u;  // sentinel stream: dropped reads sort last
    else
        sid = (uint32_t)c * 3u + (uint32_t)st;
    keys[i] = ((uint64_t)sid << 32) | (uint64_t)((uint32_t)start[i] ^ 0x80000000u);
    vals[i] = end[i];
}

__global__ void rcp_fill_i64_kernel(int64_t* p, int64_t n, int64_t v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

__global__ void rcp_stream_bounds_kernel(int64_t n, const uint64_t* __restrict__ keys,
                                         int64_t* __restrict__ off) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t sid = (int64_t)(keys[i] >> 32);
    const int64_t prev = i ? (int64_t)(keys[i - 1] >> 32) : -1;
    for (int64_t s = prev + 1; s <= sid; ++s) off[s] = i;
}

__global__ void rcp_pack_kernel(int64_t n, const uint64_t* __restrict__ keys, const int32_t* __restrict__ vals,
                                int2* __restrict__ se, uint64_t* __restrict__ scan_in) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    const int32_t start = (int32_t)((uint32_t)k ^ 0x80000000u);
    const int32_t end = vals[i];
    se[i] = make_int2(start, end);
    scan_in[i] = (k & 0xFFFFFFFF00000000ull) | (uint64_t)((uint32_t)end ^ 0x80000000u);
}

__global__ void rcp_unpack_pmax_kernel(int64_t n, const uint64_t* __restrict__ scan_out,
                                       int32_t* __restrict__ pmax) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) pmax[i] = (int32_t)((uint32_t)scan_out[i] ^ 0x80000000u);
}

struct SegMaxOp {
    // segmented max: keys in the high word, biased ends in the low word
    __host__ __device__ __forceinline__ uint64_t operator()(const uint64_t& a, const uint64_t& b) const {
        if ((a >> 32) != (b >> 32)) return b;
        return ((uint32_t)a > (uint32_t)b) ? ((b & 0xFFFFFFFF00000000ull) | (uint32_t)a) : b;
    }
};

extern "C" hipError_t rcp_sort_pairs(void* temp, size_t* temp_bytes, const uint64_t* kin, uint64_t* kout,
                                     const int32_t* vin, int32_t* vout, int64_t n, int end_bit,
                                     hipStream_t stream) {
    return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, kin, kout, vin, vout, (int)n, 0, end_bit,
                                              stream);
}

extern "C" hipError_t rcp_segmax_scan(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out,
                                      int64_t n, hipStream_t stream) {
    return hipcub::DeviceScan::InclusiveScan(temp, *temp_bytes, in, out, SegMaxOp(), (int)n, stream);
}

// =================================================================================
// locate: per (row, segment, stream) read ranges and the NULL rules
// =================================================================================
__global__ void __launch_bounds__(kBlock) rcp_locate_kernel(RcpPlanDev P) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= P.n_rows) return;
    const int j0 = P.row_seg[r], j1 = P.row_seg[r + 1];
    const int32_t chrom = P.row_chrom[r];
    const bool ok = !P.row_static[r] && chrom >= 0 && chrom < P.n_chrom && j1 > j0;
    bool hit[4] = {false, false, false, false};
    bool present[4] = {false, false, false, false};
    int32_t maxend[4] = {INT32_MIN, INT32_MIN, INT32_MIN, INT32_MIN};
    int32_t maxpos[4] = {INT32_MIN, INT32_MIN, INT32_MIN, INT32_MIN};
    for (int j = j0; j < j1; ++j) {
        const RcpSeg sg = P.segs[j];
        const int g = sg.group & 3;
        present[g] = true;
        maxpos[g] = max(maxpos[g], sg.hi);
        for (int s = 0; s < 3; ++s) {
            uint32_t lo = 0, hi = 0;
            if (ok && sg.query_ok && ((sg.streams >> s) & 1)) {
                const uint32_t so = (uint32_t)P.stream_off[chrom * 3 + s];
                const uint32_t eo = (uint32_t)P.stream_off[chrom * 3 + s + 1];
                lo = lower_bound_pmax(P.pmax, so, eo, sg.lo);
                hi = upper_bound_start(P.se, lo, eo, sg.hi);
                if (lo < hi) {
                    hit[g] = true;
                    maxend[g] = max(maxend[g], P.pmax[hi - 1]);
                }
            }
            P.seg_lo[j * 3 + s] = lo;
            P.seg_hi[j * 3 + s] = hi;
        }
    }
    bool valid = ok;
    if (ok) {
        const int64_t sl = P.seqlen[chrom];
        for (int g = 0; g < 4; ++g) {
            if (!present[g]) continue;
            // no hits -> NULL (coverage.R:224-225); Rle[i2k] beyond the Rle -> error -> NULL
            // (coverage.R:217-222): the Rle spans seqlength, or the hits' max end when NA.
            valid = valid && hit[g] && (sl >= 0 ? (int64_t)maxpos[g] <= sl : maxpos[g] <= maxend[g]);
        }
    }
    P.valid[r] = valid ? 1 : 0;
}

// =================================================================================
// pileup -> bins -> column-major profile (or CSR coverage)
// =================================================================================
template <int T, bool MEDIAN, bool CSR>
__global__ void __launch_bounds__(kBlock) rcp_pileup_kernel(RcpPlanDev P, double* __restrict__ out,
                                                            int64_t* __restrict__ binsum) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
    // ---- decode (row tile, part, chunk)
    const int tile = blockIdx.x / P.n_chunks_total;
    int c = blockIdx.x - tile * P.n_chunks_total;
    int p = 0;
    while (p < P.n_parts - 1 && c >= P.part[p].n_chunks) {
        c -= P.part[p].n_chunks;
        ++p;
    }
    const RcpPart part = P.part[p];
    const int32_t k0 = c * part.chunk_bins;

    int32_t* diff = reinterpret_cast<int32_t*>(smem);
    const int diff_words = (P.chunk_cap + 8 + 1023) & ~1023;
    uint32_t* stage = reinterpret_cast<uint32_t*>(smem) + diff_words;
    int32_t* m_bs = reinterpret_cast<int32_t*>(stage + (CSR ? 0 : P.stage_cap * T));
    int32_t* m_lay = m_bs + T;
    int32_t* m_P0 = m_lay + T;
    int32_t* m_npos = m_P0 + T;
    int32_t* m_kend = m_npos + T;
    int32_t* m_flag = m_kend + T;
    uint32_t* scratch = reinterpret_cast<uint32_t*>(m_flag + T);

    if (tid < T) {
        const int r = tile * T + tid;
        int32_t flag = 2, bs = 0, lay = -1, P0 = 0, npos = 0, kend = k0;
        if (r < P.n_rows) {
            int32_t head, L;
            rcp_part_slice(part, P.row_len[r], &head, &L);
            const int32_t n = CSR ? L : part.n_bins;
            kend = min(k0 + part.chunk_bins, n);
            if (!P.valid[r]) {
                flag = CSR ? 2 : 1;  // NULL row -> zeros (profile.R:191-197)
            } else if (k0 >= n) {
                flag = 2;
            } else if (!part.per_base && L < n) {
                flag = 2;  // interpolation rows: rcp_interp_kernel
            } else if (part.per_base && !CSR && L != n) {
                atomicOr(P.status, RCP_STATUS_WIDTH);
                flag = 1;
            } else {
                if (part.per_base) {
                    bs = 1;
                } else {
                    bs = L / n;
                    const int32_t dif = L - bs * n;
                    if (dif) {
                        lay = P.lay_index[part.lay_base + dif];
                        if (lay < 0) {
                            atomicOr(P.status, RCP_STATUS_INTERP);
                            lay = -1;
                        }
                    }
                }
                const int32_t e0 = bin_edge(bs, lay, P.lay_cnt, k0);
                const int32_t e1 = bin_edge(bs, lay, P.lay_cnt, kend);
                P0 = head + e0;
                npos = e1 - e0;
                flag = 0;
                if (npos > P.chunk_cap) {
                    atomicOr(P.status, RCP_STATUS_INTERP);
                    flag = 1;
                }
            }
        }
        m_bs[tid] = bs;
        m_lay[tid] = lay;
        m_P0[tid] = P0;
        m_npos[tid] = npos;
        m_kend[tid] = kend;
        m_flag[tid] = flag;
    }
    __syncthreads();

    for (int i = 0; i < T; ++i) {
        if (m_flag[i] != 0) continue;  // uniform: read from LDS
        const int r = tile * T + i;
        const int32_t P0 = m_P0[i];
        const int32_t npos = m_npos[i];
        const int per = (((npos + 1 + kBlock - 1) / kBlock) + 3) & ~3;
        for (int q = tid; q < per * kBlock; q += kBlock) diff[q] = 0;
        __syncthreads();
        pileup_rows_segments(P, r, P0, npos, diff);
        __syncthreads();
        scan_chunk<!(MEDIAN || CSR)>(diff, per, scratch);
        __syncthreads();
        const int32_t bs = m_bs[i], lay = m_lay[i], kend = m_kend[i];
        const int32_t e0 = bin_edge(bs, lay, P.lay_cnt, k0);
        for (int32_t k = k0 + tid; k < kend; k += kBlock) {
            if (CSR) {
                P.csr_out[P.csr_off[r] + k] = diff[k - k0];
                continue;
            }
            const int32_t a = bin_edge(bs, lay, P.lay_cnt, k) - e0;
            const int32_t b = bin_edge(bs, lay, P.lay_cnt, k + 1) - e0;
            uint32_t num;
            if (MEDIAN) {
                const int32_t m = b - a;
                int32_t vmin = INT32_MAX, vmax = INT32_MIN;
                for (int32_t q = a; q < b; ++q) {
                    vmin = min(vmin, diff[q]);
                    vmax = max(vmax, diff[q]);
                }
                const int32_t h = (m + 1) >> 1;
                const uint32_t x1 = (vmin == vmax) ? (uint32_t)vmin : kth_smallest(diff, a, b, h, vmin, vmax);
                uint32_t x2 = x1;
                if (!(m & 1)) x2 = (vmin == vmax) ? (uint32_t)vmin : kth_smallest(diff, a, b, h + 1, vmin, vmax);
                num = x1 + x2;  // 2 x median
            } else {
                const uint32_t* cum = reinterpret_cast<const uint32_t*>(diff);
                num = cum[b - 1] - (a > 0 ? cum[a - 1] : 0u);
            }
            stage[(k - k0) * T + i] = num;
        }
        __syncthreads();
    }
    if (CSR) return;

    // ---- epilogue: stage[bin][row] -> out[(col) * n_rows + row], 16 rows contiguous
    const int nk = part.chunk_bins;
    for (int idx = tid; idx < nk * T; idx += kBlock) {
        const int kk = idx / T;
        const int i = idx - kk * T;
        const int r = tile * T + i;
        const int32_t flag = m_flag[i];
        const int32_t k = k0 + kk;
        if (r >= P.n_rows || flag == 2 || k >= m_kend[i]) continue;
        const size_t o = (size_t)(part.col_off + k) * (size_t)P.n_rows + (size_t)r;
        if (flag == 1) {
            out[o] = 0.0;
            if (binsum) binsum[o] = 0;
            continue;
        }
        const uint32_t num = stage[kk * T + i];
        double den;
        if (MEDIAN) {
            den = 2.0;
        } else {
            const int32_t lay = m_lay[i];
            den = (double)(m_bs[i] + (lay >= 0 ? P.lay_cnt[lay + k + 1] - P.lay_cnt[lay + k] : 0));
        }
        out[o] = ((double)num * P.scale) / den;
        if (binsum) binsum[o] = (int64_t)num;
    }
}

// =================================================================================
// interpolation rows (length(x) < n): spline "fmm", neighborhood, "inear" no-op
// =================================================================================
namespace {

#pragma clang fp contract(off)
__device__ void fmm_spline_dev(int n, const double* y, double* b, double* c, double* d) {
    // stats::spline method "fmm" coefficients on x = 1..n (R splines.c fmm_spline),
    // with 1-based indexing kept for readability.
    const double* Y = y - 1;
    double *B = b - 1, *Cc = c - 1, *D = d - 1;
    if (n < 2) {
        for (int i = 1; i <= n; ++i) B[i] = Cc[i] = D[i] = 0.0;
        return;
    }
    if (n < 3) {
        const double t = (Y[2] - Y[1]);
        B[1] = t / 1.0;
        B[2] = B[1];
        Cc[1] = Cc[2] = D[1] = D[2] = 0.0;
        return;
    }
    const int nm1 = n - 1;
    D[1] = 1.0;
    Cc[2] = (Y[2] - Y[1]) / D[1];
    for (int i = 2; i < n; i++) {
        D[i] = 1.0;
        B[i] = 2.0 * (D[i - 1] + D[i]);
        Cc[i + 1] = (Y[i + 1] - Y[i]) / D[i];
        Cc[i] = Cc[i + 1] - Cc[i];
    }
    B[1] = -D[1];
    B[n] = -D[nm1];
    Cc[1] = Cc[n] = 0.0;
    if (n > 3) {
        Cc[1] = Cc[3] / 2.0 - Cc[2] / 2.0;          // x[4]-x[2], x[3]-x[1]
        Cc[n] = Cc[nm1] / 2.0 - Cc[n - 2] / 2.0;    // x[n]-x[n-2], x[n-1]-x[n-3]
        Cc[1] = Cc[1] * D[1] * D[1] / 3.0;           // x[4]-x[1]
        Cc[n] = -Cc[n] * D[nm1] * D[nm1] / 3.0;      // x[n]-x[n-3]
    }
    for (int i = 2; i <= n; i++) {
        const double t = D[i - 1] / B[i - 1];
        B[i] = B[i] - t * D[i - 1];
        Cc[i] = Cc[i] - t * Cc[i - 1];
    }
    Cc[n] = Cc[n] / B[n];
    for (int i = nm1; i >= 1; i--) Cc[i] = (Cc[i] - D[i] * Cc[i + 1]) / B[i];
    B[n] = (Y[n] - Y[n - 1]) / D[n - 1] + D[n - 1] * (Cc[n - 1] + 2.0 * Cc[n]);
    for (int i = 1; i <= nm1; i++) {
        B[i] = (Y[i + 1] - Y[i]) / D[i] - D[i] * (Cc[i + 1] + 2.0 * Cc[i]);
        D[i] = (Cc[i + 1] - Cc[i]) / D[i];
        Cc[i] = 3.0 * Cc[i];
    }
    Cc[n] = 3.0 * Cc[n];
    D[n] = D[nm1];
}

__device__ double seq_point(int L, int n, int i) {
    // seq.int(1, L, length.out = n)[i] as do_seq computes it
    if (i == 0) return 1.0;
    if (i == n - 1) return (double)L;
    const double by = ((double)L - 1.0) / (double)(n - 1);
    return (i < n / 2) ? 1.0 + (double)i * by : (double)L - (double)(n - 1 - i) * by;
}

__device__ double spline_eval_dev(int n, const double* y, const double* b, const double* c, const double* d,
                                  double u, int& i) {
    // spline_eval (R splines.c): keep the previous interval while x[i] <= u <= x[i+1],
    // else bisect; knots are x = 1..n.
    const int n_1 = n - 1;
    if (u < (double)(i + 1) || (i < n_1 && (double)(i + 2) < u)) {
        i = 0;
        int j = n;
        do {
            const int k = (i + j) / 2;
            if (u < (double)(k + 1)) j = k; else i = k;
        } while (j > i + 1);
    }
    const double dx = u - (double)(i + 1);
    return y[i] + dx * (b[i] + dx * (c[i] + dx * d[i]));
}
#pragma clang fp contract(on)

}  // namespace

__global__ void __launch_bounds__(kBlock) rcp_interp_kernel(RcpPlanDev P, double* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int32_t* diff = reinterpret_cast<int32_t*>(smem);
    const int diff_words = (P.chunk_cap + 8 + 1023) & ~1023;
    uint32_t* scratch = reinterpret_cast<uint32_t*>(smem) + diff_words;
    const int e = blockIdx.x;
    const int r = P.interp_row[e];
    const RcpPart part = P.part[P.interp_part[e]];
    const int n = part.n_bins;
    const size_t R = (size_t)P.n_rows;
    if (!P.valid[r]) {
        for (int k = threadIdx.x; k < n; k += kBlock) out[(size_t)(part.col_off + k) * R + r] = 0.0;
        return;
    }
    int32_t head, L;
    rcp_part_slice(part, P.row_len[r], &head, &L);
    if (L > P.chunk_cap) {
        if (threadIdx.x == 0) atomicOr(P.status, RCP_STATUS_INTERP);
        return;
    }
    const int per = (((L + 1 + kBlock - 1) / kBlock) + 3) & ~3;
    for (int q = threadIdx.x; q < per * kBlock; q += kBlock) diff[q] = 0;
    __syncthreads();
    pileup_rows_segments(P, r, head, L, diff);
    __syncthreads();
    scan_chunk<false>(diff, per, scratch);
    __syncthreads();
    if (threadIdx.x != 0) return;
    double* x = P.interp_scratch + (size_t)e * P.interp_stride;
    double* y = x + L + 1;
    const int mode = P.interp_mode[e];
    for (int i = 0; i < L; ++i) x[i] = (double)diff[i] * P.scale;
    if (mode == 1) {  // spline(x, n = n)$y, then x[x < 0] <- 0
        double* b = y + n + 1;
        double* c = b + L + 1;
        double* d = c + L + 1;
        fmm_spline_dev(L, x, b, c, d);
        int iv = 0;
        for (int i = 0; i < n; ++i) {
            const double v = (L == 1) ? x[0] : spline_eval_dev(L, x, b, c, d, seq_point(L, n, i), iv);
            y[i] = v < 0 ? 0.0 : v;
        }
    } else if (mode == 3) {  // neighborhood fill (util.R:53-69)
        const int32_t* pos = P.nb_pos + P.interp_pos[e];
        double* pre = y + n + 1;
        for (int i = 0; i < n; ++i) pre[i] = __builtin_nan("");
        pre[0] = x[0];
        pre[1] = x[1];
        pre[n - 2] = x[L - 2];
        pre[n - 1] = x[L - 1];
        for (int i = 0; i < L - 4; ++i) pre[pos[i] - 1] = x[2 + i];
        for (int z = 0; z < n; ++z) {
            if (!isnan(pre[z])) {
                y[z] = pre[z];
                continue;
            }
            double s = 0.0;
            int m = 0;
            const int nb[4] = {z - 2, z - 1, z + 1, z + 2};
            for (int q = 0; q < 4; ++q)
                if (nb[q] >= 0 && nb[q] < n && !isnan(pre[nb[q]])) {
                    s += pre[nb[q]];
                    ++m;
                }
            y[z] = m ? s / m : __builtin_nan("");
        }
    } else {  // "linear": the switch arm is spelled "inear" -> x unchanged; rbind recycles
        for (int i = 0; i < n; ++i) y[i] = x[i % L];
    }
    for (int k = 0; k < n; ++k) out[(size_t)(part.col_off + k) * R + r] = y[k];
}

// =================================================================================
// host-callable launchers
// =================================================================================
extern "C" hipError_t rcp_launch_locate(const RcpPlanDev* P, hipStream_t stream) {
    if (P->n_rows == 0) return hipSuccess;
    const int grid = (P->n_rows + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(rcp_locate_kernel, dim3(grid), dim3(kBlock), 0, stream, *P);
    return hipGetLastError();
}

template <int T, bool MEDIAN, bool CSR>
static hipError_t launch_pileup_t(const RcpPlanDev* P, double* out, int64_t* binsum, size_t lds, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&rcp_pileup_kernel<T, MEDIAN, CSR>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const int tiles = (P->n_rows + T - 1) / T;
    const int64_t grid = (int64_t)tiles * P->n_chunks_total;
    hipLaunchKernelGGL((rcp_pileup_kernel<T, MEDIAN, CSR>), dim3((unsigned)grid), dim3(kBlock), lds, s, *P, out,
                       binsum);
    return hipGetLastError();
}

extern "C" size_t rcp_pileup_lds_bytes(const RcpPlanDev* P, int tile_rows, int csr) {
    const size_t diff_words = (size_t)((P->chunk_cap + 8 + 1023) & ~1023);
    const size_t stage_words = csr ? 0 : (size_t)P->stage_cap * tile_rows;
    return 4 * (diff_words + stage_words + 6 * (size_t)tile_rows + 2 * kWaves + 8);
}

extern "C" hipError_t rcp_launch_pileup(const RcpPlanDev* P, double* out, int64_t* binsum, int csr,
                                        hipStream_t stream) {
    if (P->n_rows == 0) return hipSuccess;
    constexpr int T = 16;
    const size_t lds = rcp_pileup_lds_bytes(P, T, csr);
    if (csr) return launch_pileup_t<T, false, true>(P, out, binsum, lds, stream);
    if (P->stat == 1) return launch_pileup_t<T, true, false>(P, out, binsum, lds, stream);
    return launch_pileup_t<T, false, false>(P, out, binsum, lds, stream);
}

extern "C" hipError_t rcp_launch_interp(const RcpPlanDev* P, double* out, hipStream_t stream) {
    if (P->n_interp == 0) return hipSuccess;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&rcp_interp_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const size_t lds = 4 * ((size_t)((P->chunk_cap + 8 + 1023) & ~1023) + 2 * kWaves + 8);
    hipLaunchKernelGGL(rcp_interp_kernel, dim3(P->n_interp), dim3(kBlock), lds, stream, *P, out);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_readset(int64_t n, const int32_t* chrom, const int32_t* start, const int32_t* end,
                                         const int8_t* strand, int32_t n_chrom, int32_t strand_filter,
                                         uint64_t* keys, int32_t* vals, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const int64_t grid = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(rcp_make_keys_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream, n, chrom, start, end,
                       strand, n_chrom, strand_filter, keys, vals);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_streams(int64_t n, const uint64_t* keys, const int32_t* vals, int64_t* off,
                                         int64_t n_off, int2* se, uint64_t* scan_in, hipStream_t stream) {
    hipLaunchKernelGGL(rcp_fill_i64_kernel, dim3((unsigned)((n_off + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                       off, n_off, n);
    if (n == 0) return hipGetLastError();
    const int64_t grid = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(rcp_stream_bounds_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream, n, keys, off);
    hipLaunchKernelGGL(rcp_pack_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream, n, keys, vals, se, scan_in);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_unpack_pmax(int64_t n, const uint64_t* scan_out, int32_t* pmax, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const int64_t grid = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(rcp_unpack_pmax_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream, n, scan_out, pmax);
    return hipGetLastError();
}
