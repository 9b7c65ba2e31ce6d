// rcp_kernels.hip -- gfx950 (CDNA4) kernels of the coverage -> profile hot path.
//
// What they compute (reference semantics):
//   rcp_locate_kernel   findOverlaps() per region / range / strand stream, plus the
//                       NULL rules of coverageFromRanges (R/coverage.R:189-225)
//   rcp_heavy_*         rows with skewed depth (hot peaks): their reads are split into
//                       slices piled up by many workgroups into a global difference array
//   rcp_pileup_kernel   coverage(reads)[i2k] (+ rev for '-')  ->  splitVector bins ->
//                       mean / median (R/util.R:74-84) for a tile of rows, written as the
//                       R column-major profile matrix (R/profile.R:153-212, :100-151)
//   rcp_interp_kernel   rows with fewer positions than bins: stats::spline "fmm",
//                       neighborhood fill, or the "inear" no-op (R/util.R:17-73)
//   readset kernels     splitBySeqname as a (chromosome, strand) stream index with a
//                       prefix-max-of-end array for exact overlap search
//
// Design: integer interval counting, HBM-bound, no MFMA.  A workgroup owns
// 32 consecutive rows x one column chunk; each of its 4 waves owns whole rows, so a
// row needs no block barrier: the wave streams the row's reads as coalesced 8-byte
// (start, end) pairs (4 loads in flight per lane), adds +w / -w into its own LDS
// difference array, turns it into depth / cumulative depth with a wave scan (uint32,
// modular: a bin sum that fits 32 bits comes out exact), and reads every bin with two LDS
// reads.  Numerators are staged as [bin][row] so the epilogue writes 16 consecutive rows of
// a column (128 B) per 16 lanes of the R column-major matrix (64-B segments write at ~60 %
// of the 128-B rate: tools/write_bench.hip).
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <type_traits>
#include <hipcub/hipcub.hpp>

#include <mutex>
#include <set>
#include <utility>

#include "rcp_device.h"

namespace {

constexpr int kBlock = RCP_BLOCK;  // 256 threads = 4 waves
constexpr int kWaves = kBlock / 64;
constexpr int kTile = 16;          // rows per output round (128 B column segments)

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

// Wave64 inclusive prefix sum with DPP (row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 across rows): six VALU ops, no LDS round trip.  (__shfl_up
// lowers to ds_bpermute + an lgkmcnt wait per step.)
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return (uint32_t)x;
}

__device__ __forceinline__ uint32_t wave_exclusive_scan(uint32_t v) { return wave_inclusive_scan(v) - v; }

__device__ __forceinline__ int32_t wave_sum(int32_t v) {
    return __builtin_amdgcn_readlane((int)wave_inclusive_scan((uint32_t)v), 63);
}

// Block-wide exclusive scan of one uint32 per thread.  `scratch` holds kWaves words.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* scratch) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint32_t x = wave_inclusive_scan(v);
    if (lane == 63) scratch[wave] = x;
    __syncthreads();
    uint32_t off = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w)
        if (w < wave) off += scratch[w];
    return off + x - v;
}


// ---------------------------------------------------------------------------------
// Add read `rd` of segment sg to the difference array of row positions [P0, P0 + npos)
// restricted to the genomic piece [gps, gpe] of the segment.
// ---------------------------------------------------------------------------------
// LDS word of row position p in a wave array whose lanes own 2^sh positions each, padded
// by 4 words per lane (bank-conflict-free b128 scans); sh = 30 leaves p unchanged.
__device__ __forceinline__ int32_t lp(int32_t p, int sh) { return p + ((p >> sh) << 2); }

// diff[key] += w * (length of the run of equal keys starting at this lane), once per run of
// consecutive lanes holding the same key; inactive lanes split runs and add nothing.  The
// reads of a wave are consecutive in start order, so the reads of a hot row pile onto a
// few positions per wave: one LDS atomic per run instead of one per read.
__device__ __forceinline__ void run_add(int32_t* diff, int32_t key, bool act, int32_t w) {
    const int lane = threadIdx.x & 63;
    const int32_t k = act ? key : -1;                                   // -1: never a position
    const int32_t prev = __builtin_amdgcn_update_dpp(-2, k, 0x138, 0xf, 0xf, false);  // wave_shr:1
    const bool head = lane == 0 || k != prev;
    const uint64_t heads = __ballot(head);
    const uint64_t above = lane == 63 ? 0ull : heads & (~0ull << (lane + 1));
    const int nxt = above ? __builtin_ctzll(above) : 64;
    if (head && act) atomicAdd(&diff[k], w * (nxt - lane));
}


__device__ __forceinline__ void add_read(const RcpPlanDev& P, const RcpSeg& sg, int2 rd, int32_t gps, int32_t gpe,
                                         int32_t P0, int32_t* diff, int sh) {
    if (rd.y < gps || rd.x > gpe) return;
    int32_t w = 1;
    if (sg.multi && !(rd.x > sg.nb_lo && rd.y < sg.nb_hi)) {
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
    atomicAdd(&diff[lp(o0 - P0, sh)], w);
    atomicAdd(&diff[lp(o1 - P0 + 1, sh)], -w);
}

// add_read for a read of segment sg with the row offset folded: window index of genomic
// position x is x + k (forward; k = off - lo - P0) or k - x (reversed; k = off + hi - P0)
template <bool REV>
__device__ __forceinline__ void add_read_k(const RcpPlanDev& P, const RcpSeg& sg, int32_t k, int2 rd, int32_t gps,
                                           int32_t gpe, int32_t* diff, int sh, bool act) {
    if (!act || rd.y < gps || rd.x > gpe) return;
    int32_t w = 1;
    if (sg.multi && !(rd.x > sg.nb_lo && rd.y < sg.nb_hi)) {
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
    const int32_t a = REV ? k - x1 : x0 + k;
    const int32_t b = REV ? k - x0 + 1 : x1 + k + 1;
    atomicAdd(&diff[lp(a, sh)], w);
    atomicSub(&diff[lp(b, sh)], w);
}

// The candidate reads of the (segment, stream) pairs held one per lane -- lane t: segment `sg`,
// genomic piece [gps, gpe] of a row window, candidate reads [lo, hi) (empty: lo == hi) -- as one
// stream: a wave scan lays the pairs' candidates end to end, and batches of 256 candidates
// cross pair boundaries, so a window costs one round trip per 256 candidates with the next
// batch in flight while the current one is added.  The per-pair data a candidate needs is
// picked by a scalar loop over the (few) pairs a batch spans.
struct PairStream {
    int32_t gps, gpe;
    uint32_t incl, start, delta;  // per lane: inclusive / exclusive candidate scan, lo - start
    uint32_t N;                   // candidates of the window (uniform)
    uint64_t nz;                  // lanes with candidates
    int pl, pa;                   // pair holding the next batch to load / to add
};

__device__ __forceinline__ void ps_prepare(PairStream& ps, int32_t gps, int32_t gpe, uint32_t lo, uint32_t hi) {
    ps.gps = gps;
    ps.gpe = gpe;
    const uint32_t cnt = hi - lo;
    ps.incl = wave_inclusive_scan(cnt);
    ps.start = ps.incl - cnt;
    ps.N = (uint32_t)__builtin_amdgcn_readlane((int)ps.incl, 63);
    ps.delta = lo - ps.start;  // candidate q of this pair is read lo + (q - start)
    ps.nz = __ballot(cnt > 0);
    ps.pl = ps.nz ? __builtin_ctzll(ps.nz) : 0;
    ps.pa = ps.pl;
}

// Candidate slot u of a lane in a batch: 4 lane + u, so the 64 adds of one instruction are 4
// reads apart (fewer same-bank / same-address LDS atomics on start-sorted reads than lane + 64 u:
// C3 pass 0.760-0.770 -> 0.753-0.755 ms, profiles/r03/pipeline/ps_interleave_ab.log)
__device__ __forceinline__ uint32_t ps_slot(int lane, int u) { return 4u * (uint32_t)lane + (uint32_t)u; }

// Issue the loads of batch [q0, q0 + 256) (q0 < N; lanes past N load the last candidate again).
__device__ __forceinline__ void ps_load(const RcpPlanDev& P, PairStream& ps, uint32_t q0, int2 (&dst)[4]) {
    const int lane = threadIdx.x & 63;
    while ((uint32_t)__builtin_amdgcn_readlane((int)ps.incl, ps.pl) <= q0) ++ps.pl;
    uint32_t qc[4], d[4];
    const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)ps.delta, ps.pl);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        qc[u] = min(q0 + ps_slot(lane, u), ps.N - 1);
        d[u] = d0;
    }
    const uint32_t qe = min(q0 + 256u, ps.N);
    uint64_t m = ps.pl < 63 ? ps.nz & (~0ull << (ps.pl + 1)) : 0ull;
    while (m) {
        const int p = __builtin_ctzll(m);
        const uint32_t sp = (uint32_t)__builtin_amdgcn_readlane((int)ps.start, p);
        if (sp >= qe) break;
        const uint32_t dp = (uint32_t)__builtin_amdgcn_readlane((int)ps.delta, p);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (qc[u] >= sp) d[u] = dp;
        m &= m - 1;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) dst[u] = P.se[qc[u] + d[u]];
}

// Add batch [q0, q0 + 256) (loaded by ps_load) to the difference array of the window at row
// position P0; lane t holds pair t's segment `sg`.  Candidate q belongs to the pair p with
// start_p <= q < incl_p.
__device__ __forceinline__ void ps_add(const RcpPlanDev& P, const RcpSeg& sg, PairStream& ps, uint32_t q0,
                                       const int2 (&rd)[4], int32_t P0, int32_t* diff, int sh) {
    const int lane = threadIdx.x & 63;
    while ((uint32_t)__builtin_amdgcn_readlane((int)ps.incl, ps.pa) <= q0) ++ps.pa;
    const uint32_t qe = min(q0 + 256u, ps.N);
    uint64_t m = ps.nz & (~0ull << ps.pa);
    while (m) {
        const int p = __builtin_ctzll(m);
        const uint32_t sp = (uint32_t)__builtin_amdgcn_readlane((int)ps.start, p);
        if (sp >= qe) break;
        const uint32_t ep = (uint32_t)__builtin_amdgcn_readlane((int)ps.incl, p);
        RcpSeg o;
        o.lo = __builtin_amdgcn_readlane(sg.lo, p);
        o.hi = __builtin_amdgcn_readlane(sg.hi, p);
        o.off = __builtin_amdgcn_readlane(sg.off, p);
        o.gfirst = __builtin_amdgcn_readlane(sg.gfirst, p);
        o.gcount = (int16_t)__builtin_amdgcn_readlane((int)sg.gcount, p);
        o.rev = (uint8_t)__builtin_amdgcn_readlane((int)sg.rev, p);
        o.multi = (uint8_t)__builtin_amdgcn_readlane((int)sg.multi, p);
        o.nb_lo = __builtin_amdgcn_readlane(sg.nb_lo, p);
        o.nb_hi = __builtin_amdgcn_readlane(sg.nb_hi, p);
        const int32_t gs = __builtin_amdgcn_readlane(ps.gps, p);
        const int32_t ge = __builtin_amdgcn_readlane(ps.gpe, p);
        // the pair's orientation and origin folded into one offset (SGPR): a read's two adds
        // take a clip (max / min), an add and the lane padding each
        if (o.rev) {
            const int32_t k = o.off + o.hi - P0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t q = q0 + ps_slot(lane, u);
                add_read_k<true>(P, o, k, rd[u], gs, ge, diff, sh, q >= sp && q < ep);
            }
        } else {
            const int32_t k = o.off - o.lo - P0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t q = q0 + ps_slot(lane, u);
                add_read_k<false>(P, o, k, rd[u], gs, ge, diff, sh, q >= sp && q < ep);
            }
        }
        m &= m - 1;
    }
}

// Pile a prepared stream whose batch `first` is in `cur` (loaded by ps_load(.., 256 first, ..)):
// batches first, first + step, ... (step > 1: the waves of a block share one stream)
__device__ __forceinline__ void ps_pile(const RcpPlanDev& P, const RcpSeg& sg, PairStream& ps, int2 (&cur)[4],
                                        int32_t P0, int32_t* diff, int sh, int first = 0, int step = 1) {
    const uint32_t st = 256u * (uint32_t)step;
    for (uint32_t q0 = 256u * (uint32_t)first; q0 < ps.N; q0 += st) {
        int2 nx[4];
        if (q0 + st < ps.N) ps_load(P, ps, q0 + st, nx);
        ps_add(P, sg, ps, q0, cur, P0, diff, sh);
#pragma unroll
        for (int u = 0; u < 4; ++u) cur[u] = nx[u];
    }
}

__device__ __forceinline__ void pile_pairs(const RcpPlanDev& P, const RcpSeg& sg, int32_t gps, int32_t gpe,
                                           uint32_t lo, uint32_t hi, int32_t P0, int32_t* diff, int sh,
                                           int first = 0, int step = 1) {
    PairStream ps;
    ps_prepare(ps, gps, gpe, lo, hi);
    if (256u * (uint32_t)first >= ps.N) return;  // wave-uniform
    int2 cur[4];
    ps_load(P, ps, 256u * (uint32_t)first, cur);
    ps_pile(P, sg, ps, cur, P0, diff, sh, first, step);
}

// One wave piles row r (any number of segments x strand streams, e.g. a coverageRnaRef
// c(flank, exons, flank) row) over row positions [P0, P0 + npos).  Walking the (segment,
// stream) pairs one after the other costs one HBM round trip per pair, a dozen per gene.
// Here lane t owns pair t (its candidate range, narrowed by its own binary searches
// in parallel with the other lanes'); a wave scan lays the pairs' candidates end to end, and
// batches of 256 candidates cross pair boundaries, so a row costs one round trip per 256
// candidates with the next batch in flight while the current one is added.  The per-pair
// data each candidate needs is picked by a scalar loop over the (few) pairs a batch spans.
// (first, step): this wave adds batches first, first + step, ... of each stream of 64 pairs
// (the waves of a block splitting one row: block_window_depth)
__device__ __forceinline__ void pileup_row_wave(const RcpPlanDev& P, int r, int32_t P0, int32_t npos, int32_t* diff,
                                                int sh, int first = 0, int step = 1) {
    const int lane = threadIdx.x & 63;
    const int32_t P1 = P0 + npos;
    const int j0 = P.row_seg[r], j1 = P.row_seg[r + 1];
    const int n_all = (j1 - j0) * 3;
    // directory of the row's chromosome stream c*3 (all pairs in the merged layout, pair
    // stream 0 in the stranded one)
    const int64_t d0 = P.row_info[r].d0;
    const int32_t dnb = P.row_info[r].nb;
    for (int t0 = 0; t0 < n_all; t0 += 64) {
        // ---- lane t: pair (segment j, stream s)
        const int t = t0 + lane;
        RcpSeg sg = {};
        int32_t gps = 0, gpe = -1;
        uint32_t lo = 0, hi = 0;
        if (t < n_all) {
            const int j = j0 + t / 3, s = t % 3;
            sg = P.segs[j];
            const int32_t len = sg.hi - sg.lo + 1;
            const int32_t a = max(P0, sg.off);
            const int32_t b = min(P1, sg.off + len);
            if (a < b && sg.query_ok && ((sg.streams >> s) & 1)) {
                if (!sg.rev) {
                    gps = sg.lo + (a - sg.off);
                    gpe = sg.lo + (b - 1 - sg.off);
                } else {
                    gpe = sg.hi - (a - sg.off);
                    gps = sg.hi - (b - 1 - sg.off);
                }
                lo = P.seg_lo[j * 3 + s];
                hi = P.seg_hi[j * 3 + s];
                const bool full = (a == sg.off) && (b == sg.off + len);
                // a piece of the segment (the chunk window cuts it): its reads lie inside the
                // directory buckets of its ends -- one load per bound, no bisection, at most a
                // bucket (~8 reads) of extra candidates at each end, which add_read drops
                if (lo < hi && !full && (P.merged || s == 0)) {
                    const int32_t bl = min(max(gps, 0) >> P.dir_shift, dnb - 1);
                    const int32_t bu = min(max(gpe, 0) >> P.dir_shift, dnb - 1);
                    lo = max(lo, (uint32_t)P.dir_l[2 * (d0 + bl)]);
                    hi = min(hi, (uint32_t)P.dir_u[2 * (d0 + bu + 1)]);
                } else if (lo < hi && !full && hi - lo > 1024) {
                    lo = lower_bound_pmax(P.pmax, lo, hi, gps);
                    hi = upper_bound_start(P.se, lo, hi, gpe);
                }
                if (hi < lo) hi = lo;
            }
        }
        pile_pairs(P, sg, gps, gpe, lo, hi, P0, diff, sh, first, step);
    }
}

// Wave scan of the 64*per positions of a padded wave array (lane l owns positions
// [l*per, (l+1)*per) at words l*(per+4) ..): depth (CUM = false) or cumulative depth.
template <bool CUM>
__device__ __forceinline__ void scan_wave(int32_t* diff, int per) {
    const int lane = threadIdx.x & 63;
    uint32_t* base = reinterpret_cast<uint32_t*>(diff) + lane * (per + 4);
    uint32_t A = 0, B = 0;  // sum of diff, sum of the local depth prefix
    for (int q = 0; q < per; q += 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(base + q);
        A += v.x; B += A;
        A += v.y; B += A;
        A += v.z; B += A;
        A += v.w; B += A;
    }
    const uint32_t D = wave_exclusive_scan(A);  // depth entering this lane
    uint32_t C = 0;
    if (CUM) C = wave_exclusive_scan((uint32_t)per * D + B);
    uint32_t l = D, c = C;
    for (int q = 0; q < per; q += 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(base + q);
        uint4 o;
        l += v.x; c += l; o.x = CUM ? c : l;
        l += v.y; c += l; o.y = CUM ? c : l;
        l += v.z; c += l; o.z = CUM ? c : l;
        l += v.w; c += l; o.w = CUM ? c : l;
        *reinterpret_cast<uint4*>(base + q) = o;
    }
}

// Block scan (interpolation kernel): diff[0 .. 256*per) -> depth.
__device__ __forceinline__ void scan_block_depth(int32_t* diff, int per, uint32_t* scratch) {
    const int tid = threadIdx.x;
    uint32_t* base = reinterpret_cast<uint32_t*>(diff) + tid * per;
    uint32_t A = 0;
    for (int q = 0; q < per; ++q) A += base[q];
    uint32_t l = block_exclusive_scan(A, scratch);
    for (int q = 0; q < per; ++q) {
        l += base[q];
        base[q] = l;
    }
}

__device__ __forceinline__ int32_t bin_edge(int32_t bs, int32_t lay, const int32_t* __restrict__ cnt, int32_t k) {
    return bs * k + (lay >= 0 ? cnt[lay + k] : 0);
}

// k-th smallest (1-based) of depth[a .. b) by bisection on the value (depth is >= 0).
__device__ __forceinline__ uint32_t kth_smallest(const int32_t* d, int32_t a, int32_t b, int32_t k, int32_t vmin,
                                                 int32_t vmax, int sh) {
    int32_t lo = vmin, hi = vmax;
    while (lo < hi) {
        const int32_t mid = lo + ((hi - lo) >> 1);
        int32_t c = 0;
        for (int32_t q = a; q < b; ++q) c += d[lp(q, sh)] <= mid;
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
                                     int merge, uint64_t* __restrict__ keys, int32_t* __restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t st = strand[i];
    const int32_t c = chrom[i];
    uint32_t sid;
    if ((strand_filter >= 0 && st != strand_filter) || c < 0 || c >= n_chrom || st < 0 || st > 2)
        sid = (uint32_t)n_chrom * 3u;  // sentinel stream: dropped reads sort last
    else
        sid = (uint32_t)c * 3u + (merge ? 0u : (uint32_t)st);
    keys[i] = ((uint64_t)sid << 32) | (uint64_t)((uint32_t)start[i] ^ 0x80000000u);
    vals[i] = end[i];
}

__global__ void rcp_fill_i64_kernel(int64_t* p, int64_t n, int64_t v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

__global__ void rcp_stream_bounds_kernel(int64_t n, const uint64_t* __restrict__ keys, int64_t* __restrict__ off) {
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
    if (scan_in) scan_in[i] = (k & 0xFFFFFFFF00000000ull) | (uint64_t)((uint32_t)end ^ 0x80000000u);
}

__global__ void rcp_unpack_pmax_kernel(int64_t n, const uint64_t* __restrict__ scan_out, int32_t* __restrict__ pmax) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) pmax[i] = (int32_t)((uint32_t)scan_out[i] ^ 0x80000000u);
}

struct SegMaxOp {
    // segmented max: stream id in the high word, biased ends in the low word
    __host__ __device__ __forceinline__ uint64_t operator()(const uint64_t& a, const uint64_t& b) const {
        if ((a >> 32) != (b >> 32)) return b;
        return ((uint32_t)a > (uint32_t)b) ? ((b & 0xFFFFFFFF00000000ull) | (uint32_t)a) : b;
    }
};

extern "C" hipError_t rcp_sort_pairs(void* temp, size_t* temp_bytes, const uint64_t* kin, uint64_t* kout,
                                     const int32_t* vin, int32_t* vout, int64_t n, int begin_bit, int end_bit,
                                     hipStream_t stream) {
    return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, kin, kout, vin, vout, (int)n, begin_bit, end_bit,
                                              stream);
}

// flag = 1 when some key is smaller than its predecessor
__global__ void rcp_unsorted_kernel(int64_t n, const uint64_t* __restrict__ keys, uint32_t* __restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (i < n && keys[i] < keys[i - 1]) *flag = 1u;
}

// end = start + width - 1 in place over the expanded widths (IRanges: width >= 0, end fits
// int32); an end past INT32_MAX sets *overflow (the host refuses the reads)
__global__ void rcp_width_end_kernel(int64_t n, const int32_t* __restrict__ start, int32_t* __restrict__ width_end,
                                     uint32_t* __restrict__ overflow) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t e = (int64_t)start[i] + (int64_t)width_end[i] - 1;
    if (e > INT32_MAX) *overflow = 1u;
    width_end[i] = (int32_t)e;
}

// flag = 1 when a read starts before the one in front of it on the same chromosome (the slices
// of a streamed sample must hold coordinate-sorted reads, rcp_profile_reads)
__global__ void rcp_order_kernel(int64_t n, const int32_t* __restrict__ chrom, const int32_t* __restrict__ start,
                                 uint32_t* __restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i + 1 >= n) return;
    if (chrom[i] == chrom[i + 1] && start[i] > start[i + 1]) *flag = 1u;
}

// chromosome code of read i from the seqnames runs (run_start: prefix sums, n_runs + 1 entries)
__global__ void rcp_expand_runs_kernel(int64_t n, int32_t n_runs, const int64_t* __restrict__ run_start,
                                       const int32_t* __restrict__ run_value, int32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t a = 0, b = n_runs;  // last run with run_start <= i
    while (b - a > 1) {
        const int32_t m = (a + b) >> 1;
        if (run_start[m] <= i) a = m; else b = m;
    }
    out[i] = run_value[a];
}

extern "C" hipError_t rcp_segmax_scan(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out, int64_t n,
                                      hipStream_t stream) {
    return hipcub::DeviceScan::InclusiveScan(temp, *temp_bytes, in, out, SegMaxOp(), (int)n, stream);
}

// Last prefix-max of every stream = its largest read end (-1 for an empty stream).
__global__ void rcp_stream_maxend_kernel(int64_t n_streams, const int64_t* __restrict__ off,
                                         const int32_t* __restrict__ pmax, int32_t* __restrict__ out) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_streams) return;
    out[s] = off[s + 1] > off[s] ? pmax[off[s + 1] - 1] : -1;
}

// Directory entry e (stream found by bisection on dir_off): bucket b = e - dir_off[s];
// dir_l = lower_bound(pmax >= b << shift), dir_u = upper_bound(start > (b << shift) - 1).
__global__ void rcp_dir_kernel(int64_t n_entries, int64_t n_streams, const int64_t* __restrict__ dir_off,
                               const int64_t* __restrict__ off, const int32_t* __restrict__ pmax,
                               const int2* __restrict__ se, int shift, int32_t* __restrict__ dir_l,
                               int32_t* __restrict__ dir_u) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_entries) return;
    int64_t a = 0, b = n_streams;  // last stream with dir_off[s] <= e
    while (b - a > 1) {
        const int64_t m = (a + b) >> 1;
        if (dir_off[m] <= e) a = m; else b = m;
    }
    const int64_t bucket = e - dir_off[a];
    const int64_t v = bucket << shift;
    const int32_t vc = (int32_t)min(v, (int64_t)INT32_MAX);
    const uint32_t so = (uint32_t)off[a], eo = (uint32_t)off[a + 1];
    // one 8-byte entry per bucket edge: a region's lower- and upper-bound searches at the
    // same position (the interior chunk edges) read one directory line
    dir_l[2 * e] = (int32_t)lower_bound_pmax(pmax, so, eo, vc);
    dir_u[2 * e] = (int32_t)upper_bound_start(se, so, eo, (int32_t)min(v - 1, (int64_t)INT32_MAX));
}

// Inline-key directory (rcp_device.h dir_k): thread t fills half t & 1 of entry t >> 1 from the
// interleaved (dir_l, dir_u) entries e and e + 1 of the same directory.  A bucket of n <= 14
// reads keeps its keys; a denser one (reads piled at a peak or a DNase site, far above the
// genome-average density the bucket width is sized for) keeps the keys at bucket offsets
// m_i = (i + 1) n / 15 (rcp_dirk_offset), so one line narrows any search to n / 15 reads.
constexpr int kDirKeys = 14;
__device__ __forceinline__ int32_t rcp_dirk_offset(int32_t n, int i) {
    return n <= kDirKeys ? i : (int32_t)(((int64_t)(i + 1) * n) / (kDirKeys + 1));
}
__global__ void rcp_dirk_kernel(int64_t n_entries, const int32_t* __restrict__ dir_lu, const int32_t* __restrict__ pmax,
                                const int2* __restrict__ se, int32_t* __restrict__ dir_k) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 2 * n_entries) return;
    const int64_t e = t >> 1;
    const int h = (int)(t & 1);
    const int32_t a = dir_lu[2 * e + h];
    // the last entry of a stream is never a bucket's first edge (its successor is the next
    // stream's): any count is fine there, but stay inside the arrays
    const int32_t b = e + 1 < n_entries ? max(dir_lu[2 * (e + 1) + h], a) : a;
    int32_t w[16];
    w[0] = a;
    w[1] = b;
#pragma unroll
    for (int i = 0; i < kDirKeys; ++i) {
        const int32_t k = a + rcp_dirk_offset(b - a, i);
        w[2 + i] = k < b ? (h ? se[k].x : pmax[k]) : 0;
    }
    int4* dst = reinterpret_cast<int4*>(dir_k + 32 * e + 16 * h);
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[q] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// =================================================================================
// locate: per (row, segment, stream) read ranges, the NULL rules, heavy-row slots
// =================================================================================
// Row positions [*p0, *p0 + *np) that column chunk (part, first bin k0) piles up for a
// valid row of nominal length nr, mirroring the pileup kernel's metadata stage; false when
// that stage would not pile the chunk (interpolated, wide median, width mismatch, empty).
__device__ __forceinline__ bool chunk_window(const RcpPlanDev& P, const RcpPart& part, int32_t k0, int32_t nr,
                                             int32_t* p0, int32_t* np) {
    int32_t head, L;
    rcp_part_slice(part, nr, &head, &L);
    const int32_t n = part.n_bins;
    if (k0 >= n) return false;
    if (part.per_base ? L != n : L < n) return false;
    const int32_t kend = min(k0 + part.chunk_bins, n);
    int32_t bs = 1, lay = -1;
    if (!part.per_base) {
        bs = L / n;
        const int32_t dif = L - bs * n;
        if (dif) lay = max(P.lay_index[part.lay_base + dif], -1);
    }
    if (P.stat == 1 && bs + (lay >= 0 ? 1 : 0) > P.chunk_cap) return false;
    const int32_t e0 = bs * k0 + (lay >= 0 ? P.lay_cnt[lay + k0] : 0);
    const int32_t e1 = bs * kend + (lay >= 0 ? P.lay_cnt[lay + kend] : 0);
    *p0 = head + e0;
    *np = e1 - e0;
    return true;
}

// DPP quad permutations (lanes 4k .. 4k+3): 0xB1 xor 1, 0x4E xor 2, 0x00 / 0x55 / 0xAA
// broadcast lane 0 / 1 / 2
template <int CTRL>
__device__ __forceinline__ int qperm(int x) { return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false); }

// Up to K searches of one lane bisecting in lockstep: search u is lower_bound(pmax >= v[u])
// or, when dst[u] == -1 or dst[u] is odd (the locate task numbering), upper_bound(start >
// v[u]), confined to the reads of v[u]'s bucket of the directory at entry d0[u] (nb[u]
// buckets; rcp_device.h).  Both bounds are one instruction stream (first index of the bucket
// with key >= thr, key = pmax or start), and each step issues the probes of all unfinished
// searches before using any, so they cost one chain of round trips together.  (An 8-ary
// variant -- 7 probes in flight per step -- measured slower on C4: 0.099 vs 0.082 ms.)
template <int K>
__device__ __forceinline__ void dir_bound_multi(const RcpPlanDev& P, const int64_t (&d0)[K], const int32_t (&nb)[K],
                                                const int32_t (&v)[K], const int (&dst)[K], int cnt,
                                                uint32_t (&res)[K]) {
    uint32_t lo[K], hi[K];
    int64_t thr[K];
    bool up[K];
#pragma unroll
    for (int u = 0; u < K; ++u) {
        up[u] = dst[u] == -1 || (dst[u] >= 0 && (dst[u] & 1));
        lo[u] = hi[u] = 0;
        thr[u] = (int64_t)v[u] + (up[u] ? 1 : 0);
        if (u < cnt && !P.dir_k) {
            const int32_t b = min(max(v[u], 0) >> P.dir_shift, nb[u] - 1);
            const int32_t* dir = up[u] ? P.dir_u : P.dir_l;  // interleaved: stride 2
            lo[u] = (uint32_t)dir[2 * (d0[u] + b)];
            hi[u] = (uint32_t)dir[2 * (d0[u] + b + 1)];
        }
    }
    if (P.dir_k) {
        // one line per search: the bucket's edges and 14 keys -- its first ones (n <= 14: the
        // answer is the number of keys below the threshold) or, in a denser bucket, the keys at
        // offsets m_i = (i + 1) n / 15: c keys below the threshold put the answer in
        // (m_{c-1}, m_c] (rcp_dirk_offset), searched below
        constexpr int kQ = 4, kKeys = 4 * kQ - 2;  // 16-byte words of the entry half read per search
        static_assert(kKeys == kDirKeys, "the search reads the keys rcp_dirk_kernel writes");
        int4 w[K][kQ];
#pragma unroll
        for (int u = 0; u < K; ++u) {
            if (u < cnt) {
                const int32_t b = min(max(v[u], 0) >> P.dir_shift, nb[u] - 1);
                const int4* src = reinterpret_cast<const int4*>(P.dir_k + 32 * (d0[u] + b) + (up[u] ? 16 : 0));
#pragma unroll
                for (int q = 0; q < kQ; ++q) w[u][q] = src[q];
            }
        }
#pragma unroll
        for (int u = 0; u < K; ++u) {
            if (u < cnt) {
                const int32_t* x = reinterpret_cast<const int32_t*>(w[u]);
                const int32_t n = x[1] - x[0];
                uint32_t c = 0;
#pragma unroll
                for (int i = 0; i < kKeys; ++i) c += (i < n && (int64_t)x[2 + i] < thr[u]) ? 1u : 0u;
                if (n <= kKeys) {
                    lo[u] = (uint32_t)x[0] + c;
                    hi[u] = c < (uint32_t)kKeys ? lo[u] : (uint32_t)x[1];
                } else {
                    lo[u] = (uint32_t)x[0] + (c ? (uint32_t)rcp_dirk_offset(n, (int)c - 1) + 1u : 0u);
                    hi[u] = c < (uint32_t)kKeys ? (uint32_t)x[0] + (uint32_t)rcp_dirk_offset(n, (int)c) : (uint32_t)x[1];
                }
            }
        }
    }
    const int32_t* se = reinterpret_cast<const int32_t*>(P.se);
    // bisection to the answer (an 8-ary step -- 7 probes per search in flight -- and a last
    // linear pass over <= 16 keys both measured slower on C4 / C5: profiles/r04/locate_ab.log,
    // locate_lin_ab.log)
    while (true) {
        uint32_t m[K];
        int32_t kv[K];
        bool any = false;
#pragma unroll
        for (int u = 0; u < K; ++u) {
            if (lo[u] < hi[u]) {
                m[u] = lo[u] + ((hi[u] - lo[u]) >> 1);
                kv[u] = up[u] ? se[(size_t)m[u] << 1] : P.pmax[m[u]];
                any = true;
            }
        }
        if (!any) break;
#pragma unroll
        for (int u = 0; u < K; ++u) {
            if (lo[u] < hi[u]) {
                if ((int64_t)kv[u] < thr[u]) lo[u] = m[u] + 1; else hi[u] = m[u];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < K; ++u) res[u] = lo[u];
}


// LPR = 4 lanes per row: the row's (segment, stream) searches are dealt round-robin to the
// quad's lanes (one stream per segment in the merged layout, three in the stranded one), so
// multi-range rows search in parallel; the quad then combines hits / max ends / candidate
// counts with DPP.  For a single-range row the lanes also split the per-chunk range searches.
// Every search is bounded by the bucket directory and independent of the others: the
// dependent chain per lane is one bucket search, not a sequence of them.
constexpr int kLocWpe = 1;   // waves per SIMD asked of the KS = 4 / 8 variants
constexpr int kLocWpe2 = 6;  // ... of the KS = 2 variant (<= 80 VGPRs)

// KS: searches of one lockstep round per lane of a single-range row (2: plans of <= 3 column
// chunks, 4: <= 7, 8: more, one round); KP: searches per round of the (segment, stream) pair
// loop (two per pair).  Fewer held dir_k lines = fewer VGPRs = more waves in flight.
template <int KS, int KP>
__device__ __forceinline__ void locate_rows(const RcpPlanDev& P, uint32_t (*xres)[2 * RCP_MAX_CRANGE_CHUNKS],
                                            uint32_t (*item_w)[RCP_MAX_CRANGE_CHUNKS]) {
    constexpr int LPR = 4;                 // lanes per row (a quad)
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = t / LPR;
    const int q = t % LPR;
    uint32_t* xr = xres[threadIdx.x / LPR];
    const bool in_row = r < P.n_rows;
    // the row's locate input: one 80-byte record (RcpRowInfo, built with the plan)
    RcpRowInfo ri;
    {
        uint4* d = reinterpret_cast<uint4*>(&ri);
        if (in_row) {
            const uint4* src = reinterpret_cast<const uint4*>(P.row_info + r);
#pragma unroll
            for (int u = 0; u < (int)(sizeof(RcpRowInfo) / 16); ++u) d[u] = src[u];
        } else {
#pragma unroll
            for (int u = 0; u < (int)(sizeof(RcpRowInfo) / 16); ++u) d[u] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
    const int j0 = ri.j0, j1 = ri.j1;
    const int32_t chrom = in_row ? ri.chrom : -1;
    const bool ok = in_row && !ri.stat && chrom >= 0 && chrom < P.n_chrom && j1 > j0;
    const int ns = P.merged ? 1 : 3;  // streams searched per segment
    const int npairs = (j1 - j0) * ns;
    uint32_t hit = 0, present = 0;  // bit g: group g
    int32_t maxend[4] = {INT32_MIN, INT32_MIN, INT32_MIN, INT32_MIN};
    int32_t maxpos[4] = {INT32_MIN, INT32_MIN, INT32_MIN, INT32_MIN};
    uint32_t ncand = 0, lo = 0, hi = 0;
    const int64_t sl = ok ? ri.seqlen : -1;
    // ---- single-range rows: the per-chunk candidate ranges (each column chunk streams only
    // the reads that reach its piece of the row) need bound searches at the interior chunk
    // edges; they do not depend on the row's own bounds, so they run in the same round
    RcpSeg sg0{};
    bool fast = false;
    if (in_row && j1 == j0 + 1) {
        sg0 = ri.seg0;
        fast = !sg0.multi && sg0.query_ok;
    }
    const int nc = P.n_chunks_total;
    const int32_t nr = in_row ? ri.row_len : 0;
    const int32_t len = sg0.hi - sg0.lo + 1;
    // genomic piece of chunk c (false: the chunk streams the whole range / nothing special)
    auto piece = [&](int c, int32_t* gps, int32_t* gpe, bool* empty) -> bool {
        int32_t p0, np;
        *empty = false;
        if (nr == P.cw_len) {  // the plan's common row length: windows tabulated on the host
            np = P.cw[2 * c + 1];
            if (np < 0) return false;
            p0 = P.cw[2 * c];
        } else
        {
            int p = 0, cp = c;
            while (p < P.n_parts - 1 && cp >= P.part[p].n_chunks) {
                cp -= P.part[p].n_chunks;
                ++p;
            }
            if (!chunk_window(P, P.part[p], cp * P.part[p].chunk_bins, nr, &p0, &np)) return false;
        }
        const int32_t a = max(p0, sg0.off), b = min(p0 + np, sg0.off + len);
        if (a >= b) {
            *empty = true;
            return false;
        }
        if (!sg0.rev) {
            *gps = sg0.lo + (a - sg0.off);
            *gpe = sg0.lo + (b - 1 - sg0.off);
        } else {
            *gpe = sg0.hi - (a - sg0.off);
            *gps = sg0.hi - (b - 1 - sg0.off);
        }
        return true;
    };
    // one search pair (a single-range row in the merged layout): searches [lower, upper,
    // interior chunk edges ...] are dealt to the quad's lanes and run in lockstep
    const bool split1 = ns == 1 && npairs == 1;
    const bool spec_cr = split1 && P.crange != nullptr && fast && ok;
    if (split1) {
        const RcpSeg sg = ri.seg0;
        const int g = sg.group & 3;
        present = 1u << g;
        maxpos[g] = sg.hi;
        const bool qok = ok && sg.query_ok && (sg.streams & 1);
        // the searches, tasks -2 (lower), -1 (upper), 0 .. 2 nc - 1 (chunk edges): lane q takes
        // tasks -2 + q, -2 + q + 4, ... (up to 9 of 2 + 2 * RCP_MAX_CRANGE_CHUNKS = 34; edges at
        // the row's ends are skipped) and evaluates only its own chunk windows
        int32_t sx[KS] = {};
        int sdst[KS] = {};  // -2 lower, -1 upper, >= 0 xr index (its parity = upper)
        int cnt = 0;
        uint32_t v = 0;
        // up to 4 searches bisect in lockstep (one chain of dependent loads for all of them:
        // C2 has 8 searches per row -> 2 per lane, C5 16 -> 4); a 5th starts a second round
        auto run = [&]() {
            uint32_t w[KS];
            int64_t dd[KS];
            int32_t dn[KS];
#pragma unroll
            for (int u = 0; u < KS; ++u) {
                dd[u] = ri.d0;
                dn[u] = ri.nb;
            }
            dir_bound_multi<KS>(P, dd, dn, sx, sdst, cnt, w);
#pragma unroll
            for (int u = 0; u < KS; ++u)
                if (u < cnt) {
                    if (sdst[u] == -2) v = w[u];
                    else if (sdst[u] == -1) v = w[u];
                    else xr[sdst[u]] = w[u];
                }
            cnt = 0;
        };
        for (int task = -2 + q; task < (spec_cr ? 2 * nc : 0); task += LPR) {
            int32_t x = 0;
            bool need = false;
            if (task < 0) {
                x = task == -1 ? sg.hi : sg.lo;
                need = qok;
            } else {
                int32_t gps = 0, gpe = 0;
                bool empty;
                if (piece(task >> 1, &gps, &gpe, &empty)) {
                    need = (task & 1) ? gpe < sg0.hi : gps > sg0.lo;  // a row end: the row's own bound
                    x = (task & 1) ? gpe : gps;
                }
            }
            if (!need) continue;
#pragma unroll
            for (int u = 0; u < KS; ++u)
                if (cnt == u) {
                    sx[u] = x;
                    sdst[u] = task;
                }
            if (++cnt == KS) run();
        }
        if (cnt) run();
        lo = (uint32_t)qperm<0x00>((int)v);
        hi = max(lo, (uint32_t)qperm<0x55>((int)v));
        if (lo < hi) {
            hit = 1u << g;
            if (sl < 0 && q == 0) maxend[g] = P.pmax[hi - 1];
            if (q == 0) ncand = hi - lo;
        }
        // (P.seg_lo / seg_hi of the row: written below, once the heavy slot is known -- the
        // lean and bin-difference kernels read fast rows' ranges from the record)
        if (q != 0) lo = hi = 0;  // the quad combine below reads (lo, hi) from lane 0
    }
    // (segment, stream) pairs dealt round-robin to the quad; a lane's two pairs of one round
    // (pi, pi + LPR) search their lower and upper bounds in lockstep: one chain of dependent
    // loads for four searches (an exon list of ~10 segments: 2 rounds instead of 6 chains)
    constexpr int kPairs = KP / 2;  // pairs per lane per round
    for (int pb = split1 ? npairs : q; pb < npairs; pb += kPairs * LPR) {
        int32_t sv[KP];
        int sd[KP];
        int64_t sd0[KP];
        int32_t snb[KP];
        bool use[kPairs];
#pragma unroll
        for (int u = 0; u < KP; ++u) {
            sv[u] = 0;
            sd[u] = (u & 1) ? -1 : -2;
            sd0[u] = 0;
            snb[u] = 1;
        }
#pragma unroll
        for (int k = 0; k < kPairs; ++k) use[k] = false;
        int cnt = 0;
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
            const int pi = pb + k * LPR;
            if (pi >= npairs) continue;
            const int j = j0 + pi / ns;
            const int s = pi % ns;
            const RcpSeg sg = P.segs[j];
            const int g = sg.group & 3;
            present |= 1u << g;
            maxpos[g] = max(maxpos[g], sg.hi);
            if (ok && sg.query_ok && ((sg.streams >> s) & 1)) {
                use[k] = true;
                int64_t d0 = ri.d0;
                int32_t nb = ri.nb;
                if (!P.merged) {
                    d0 = P.dir_off[chrom * 3 + s];
                    nb = (int32_t)(P.dir_off[chrom * 3 + s + 1] - d0) - 1;
                }
                sv[2 * k] = sg.lo;
                sv[2 * k + 1] = sg.hi;
                sd0[2 * k] = sd0[2 * k + 1] = d0;
                snb[2 * k] = snb[2 * k + 1] = nb;
                cnt = 2 * k + 2;
            }
        }
        uint32_t res[KP];
        dir_bound_multi<KP>(P, sd0, snb, sv, sd, cnt, res);
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
            const int pi = pb + k * LPR;
            if (pi >= npairs) continue;
            const int j = j0 + pi / ns;
            const int s = pi % ns;
            const int g = P.segs[j].group & 3;
            lo = 0;
            hi = 0;
            if (use[k]) {
                lo = res[2 * k];
                hi = max(lo, res[2 * k + 1]);
                if (lo < hi) {
                    hit |= 1u << g;
                    if (sl < 0) maxend[g] = max(maxend[g], P.pmax[hi - 1]);  // only NA seqlengths need it
                    ncand += hi - lo;
                }
            }
            P.seg_lo[j * 3 + s] = lo;
            P.seg_hi[j * 3 + s] = hi;
            // (merged layout: the entries of streams 1, 2 stay as
            // the plan zeroed them; no read lives there)
        }
    }
    // ---- combine the quad (all lanes active: DPP reads neighbours)
    {
        hit |= (uint32_t)qperm<0xB1>((int)hit);
        hit |= (uint32_t)qperm<0x4E>((int)hit);
        present |= (uint32_t)qperm<0xB1>((int)present);
        present |= (uint32_t)qperm<0x4E>((int)present);
        ncand += (uint32_t)qperm<0xB1>((int)ncand);
        ncand += (uint32_t)qperm<0x4E>((int)ncand);
    #pragma unroll
        for (int g = 0; g < 4; ++g) {
            maxend[g] = max(maxend[g], qperm<0xB1>(maxend[g]));
            maxend[g] = max(maxend[g], qperm<0x4E>(maxend[g]));
            maxpos[g] = max(maxpos[g], qperm<0xB1>(maxpos[g]));
            maxpos[g] = max(maxpos[g], qperm<0x4E>(maxpos[g]));
        }
    }
    // the single range of a fast row: (lo, hi) of pairs 0, 1, 2 sit in lanes 0, 1, 2 (LPR 1:
    // the merged layout's one pair, in the lane itself)
    const uint32_t lo0 = (uint32_t)qperm<0x00>((int)lo), hi0 = (uint32_t)qperm<0x00>((int)hi);
    const uint32_t lo1 = (uint32_t)qperm<0x55>((int)lo), hi1 = (uint32_t)qperm<0x55>((int)hi);
    const uint32_t lo2 = (uint32_t)qperm<0xAA>((int)lo), hi2 = (uint32_t)qperm<0xAA>((int)hi);
    bool valid = ok;
    if (ok) {
        for (int g = 0; g < 4; ++g) {
            if (!((present >> g) & 1)) continue;
            // no hits -> NULL (coverage.R:224-225); Rle[i2k] beyond the Rle -> error -> NULL
            // (coverage.R:217-222): the Rle spans seqlength, or the hits' max end when NA.
            valid = valid && ((hit >> g) & 1) && (sl >= 0 ? (int64_t)maxpos[g] <= sl : maxpos[g] <= maxend[g]);
        }
    }
    int32_t slot = -1;
    // side outputs a fast row needs only on the heavy path when the pileup is a lean or
    // bin-difference kernel (they read the record): its (lo, hi) in seg_lo / seg_hi and ncand,
    // for rcp_heavy_pileup_kernel (4 scattered stores per row fewer: C4 locate -14 us,
    // profiles/r04/r4j/ab.log l1).  Not when the plan interpolates rows: rcp_interp_kernel piles
    // an interpolated row from seg_lo / seg_hi (block_window_depth), and a lean plan may hold
    // such rows (a row shorter than its bins among power-of-two-binned ones)
    const bool rec_only = fast && P.n_interp == 0 && (P.lean == 1 || P.lean == 2 || P.lean == 4);
    if (in_row && q == 0) {
        P.valid[r] = valid ? 1 : 0;
        if (P.valid_out) P.valid_out[r] = valid ? 1 : 0;
        // skewed rows only: many candidates per column chunk (each chunk of a row is one
        // wave's work) AND a deep pileup (> 2 reads per position), so a long row with
        // proportionally many reads stays on the workgroup path
        const int32_t rl = nr;
        if (valid && P.heavy_threshold > 0 &&
            (uint64_t)ncand > (uint64_t)P.heavy_threshold * (uint64_t)max(P.n_chunks_total, 1) &&
            ncand > 2u * (uint32_t)max(rl, 0) && rl <= P.heavy_max_len) {
            const uint32_t u = atomicAdd(&P.status[1], 1u);
            if (u < (uint32_t)P.heavy_cap) {
                slot = (int32_t)u;
                P.heavy_rows[u] = r;
                P.heavy_nslice[u] = (ncand + (uint32_t)P.heavy_slice - 1) / (uint32_t)P.heavy_slice;
            }
        }
        if (!rec_only || slot >= 0) {
            P.ncand[r] = ncand;
            if (split1) {
                P.seg_lo[j0 * 3] = lo0;
                P.seg_hi[j0 * 3] = hi0;
            }
        }
    }
    slot = qperm<0x00>(slot);
    const bool cr = P.crange != nullptr && fast && valid && slot < 0;
    if (cr && ns == 1) {
        // merged layout: the interior edges were searched with the row's bounds (xr)
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // the quad's lanes take every LPR-th chunk (lo0 / hi0 are broadcast, xr is shared)
        for (int c = q; c < nc; c += LPR) {
            int32_t gps, gpe;
            bool empty;
            uint32_t clo = lo0, chi = hi0;
            if (piece(c, &gps, &gpe, &empty)) {
                clo = gps > sg0.lo ? max(lo0, xr[2 * c]) : lo0;
                chi = max(clo, gpe < sg0.hi ? min(hi0, xr[2 * c + 1]) : hi0);
            } else if (empty) {
                chi = clo;
            }
            // merged layout: one stream, so dense (row, chunk) words -- a wave's writes are
            // whole lines (stride 3, as the stranded layout below, measured ~1 us slower on C4)
            P.crange[(size_t)r * nc + c] = make_uint2(clo, chi);
            if (item_w && chi > clo) atomicAdd(&item_w[(threadIdx.x / LPR) >> 5][c], chi - clo);
        }
    } else if (cr && q < 3) {
        // stranded layout: lane q refines its own stream's range chunk by chunk
        for (int c = 0; c < nc; ++c) {
            int32_t gps, gpe;
            bool empty;
            uint32_t clo = lo, chi = hi;
            if (lo < hi && piece(c, &gps, &gpe, &empty)) {
                if (gps > sg0.lo) clo = lower_bound_pmax(P.pmax, lo, hi, gps);
                if (gpe < sg0.hi) chi = upper_bound_start(P.se, clo, hi, gpe);
                chi = max(clo, chi);
            } else if (lo < hi && empty) {
                chi = clo;
            }
            P.crange[((size_t)r * nc + c) * 3 + q] = make_uint2(clo, chi);
            if (item_w && chi > clo) atomicAdd(&item_w[(threadIdx.x / LPR) >> 5][c], chi - clo);
        }
    }
    if (!in_row || q != 0) return;
    // one record per row for the pileup kernel's metadata stage
    RcpRowRec rec;
    rec.flags = valid ? RCP_REC_VALID : 0;
    rec.row_len = nr;
    rec.heavy = slot;
    rec.off = rec.slo = rec.shi = rec.rev = 0;
    for (int u = 0; u < 3; ++u) rec.lo[u] = rec.hi[u] = 0;
    rec.pad[0] = rec.pad[1] = rec.pad[2] = 0;
    if (fast) {
        rec.flags |= RCP_REC_FAST | (cr ? RCP_REC_CRANGE : 0);
        rec.off = sg0.off; rec.slo = sg0.lo; rec.shi = sg0.hi; rec.rev = sg0.rev;
        rec.lo[0] = lo0; rec.hi[0] = hi0;
        if (ns == 3) {
            rec.lo[1] = lo1; rec.hi[1] = hi1;
            rec.lo[2] = lo2; rec.hi[2] = hi2;
        }
    }
    const uint4* src = reinterpret_cast<const uint4*>(&rec);
    uint4* dst = reinterpret_cast<uint4*>(P.rec + r);
#pragma unroll
    for (int u = 0; u < 4; ++u) dst[u] = src[u];
}

template <int KS, int KP>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KS == 2 ? kLocWpe2 : kLocWpe)))
rcp_locate_kernel(RcpPlanDev P) {
    constexpr int LPR = 4;                 // lanes per row (a quad)
    __shared__ uint32_t xres[kBlock / LPR][2 * RCP_MAX_CRANGE_CHUNKS];  // per row: chunk bounds
    // heaviest-first lean items (P.lpt): this block's 64 rows are two 32-row tiles; their
    // items' candidate reads are summed here and filed by class after the rows
    __shared__ uint32_t item_w[2][RCP_MAX_CRANGE_CHUNKS];
    if (P.lpt && threadIdx.x < 2 * RCP_MAX_CRANGE_CHUNKS)
        item_w[threadIdx.x / RCP_MAX_CRANGE_CHUNKS][threadIdx.x % RCP_MAX_CRANGE_CHUNKS] = 0u;
    if (P.lpt) __syncthreads();
    locate_rows<KS, KP>(P, xres, P.lpt ? item_w : nullptr);
    if (P.lpt) {
        __syncthreads();
        const int nc = P.n_chunks_total;
        const int t = threadIdx.x;
        const int tile = blockIdx.x * 2 + t / max(nc, 1);
        const int n_tiles = (P.n_rows + 31) / 32;
        if (t < 2 * nc && tile < n_tiles) {
            const uint32_t w = item_w[t / nc][t % nc];
            const int cls = w ? min(RCP_LPT_CLASSES - 1, 31 - __clz(w)) : 0;
            const uint32_t slot = atomicAdd(&P.status[RCP_LPT_STATUS + cls], 1u);
            if (slot < (uint32_t)P.lpt_cap) P.item_order[cls * P.lpt_cap + slot] = tile * nc + t % nc;
        }
    }
    // ---- the previous execution's heavy slots (its pileup kernels read them across column
    // chunks, so they are cleared here, before this execution's heavy kernel adds into them).
    // After the rows, each wave reading the count itself: no block-wide wait on that load
    // before the rows' own chains start (neutral on C4 / C2, profiles/r03/pipeline/locate_ablation_ab.log).
    const uint32_t n_prev = P.heavy_threshold > 0 ? min(P.status_prev[1], (uint32_t)P.heavy_cap) : 0u;
    for (uint32_t s = blockIdx.x; s < n_prev; s += gridDim.x) {
        int4* g4 = reinterpret_cast<int4*>(P.heavy_gdiff + (size_t)s * P.heavy_stride);  // stride: multiple of 64
        for (int i = threadIdx.x; i < (P.heavy_stride >> 2); i += blockDim.x) g4[i] = make_int4(0, 0, 0, 0);
    }
    // (status_prev is zeroed by the next launch, rcp_heavy_pileup_kernel, once every block here
    // has read it: a last-block ticket over this grid's thousands of blocks cost ~150 us)
}


// =================================================================================
// heavy rows: slice pileup
// =================================================================================
constexpr int kHeavyLoads = 16;  // = the heavy slice (4096 reads) / kBlock: one round trip per slice

__global__ void __launch_bounds__(kBlock) rcp_heavy_pileup_kernel(RcpPlanDev P) {
    // dynamic LDS only (a static array on top of the 160 KB dynamic limit fails the launch
    // attribute): 16 words of scan scratch, the row's difference array, the slice offsets
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint32_t* scratch = reinterpret_cast<uint32_t*>(smem);
    int32_t* diff = reinterpret_cast<int32_t*>(smem) + 16;
    uint32_t* offs = reinterpret_cast<uint32_t*>(diff) + (P.heavy_max_len + 1 + 64);  // [heavy_cap + 1]
    // every locate block has read the previous execution's status set: zero it for the next
    // execution (launched with one block when the plan has no heavy path)
    if (blockIdx.x == 0 && threadIdx.x < RCP_STATUS_WORDS) P.status_prev[threadIdx.x] = 0u;
    const uint32_t n = P.heavy_threshold > 0 ? min(P.status[1], (uint32_t)P.heavy_cap) : 0u;
    if (n == 0) return;
    // slice offsets of the slots: every block scans the per-slot slice counts locate stored
    // when it claimed them (no separate one-block planning kernel between the two)
    uint32_t total = 0;
    for (uint32_t b = 0; b < n; b += kBlock) {
        const uint32_t s = b + threadIdx.x;
        const uint32_t c = s < n ? P.heavy_nslice[s] : 0u;
        const uint32_t ex = block_exclusive_scan(c, scratch);
        if (s < n) offs[s] = total + ex;
        uint32_t round = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) round += scratch[w];
        total += round;
        __syncthreads();  // scratch is rewritten by the next round
    }
    __syncthreads();
    for (uint32_t w = blockIdx.x; w < total; w += gridDim.x) {
        // slot holding slice w
        uint32_t lo = 0, hi = n;
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (offs[m] <= w) lo = m; else hi = m;
        }
        const int slot = (int)lo;
        const int r = P.heavy_rows[slot];
        const int32_t nr = P.row_len[r];
        const uint32_t q0 = (w - offs[slot]) * (uint32_t)P.heavy_slice;
        const uint32_t q1 = min(q0 + (uint32_t)P.heavy_slice, P.ncand[r]);
        for (int q = threadIdx.x; q <= nr; q += kBlock) diff[q] = 0;
        __syncthreads();
        // walk the row's (segment, stream) read ranges in candidate order; the slice's part
        // of each range is streamed with kHeavyLoads loads in flight per thread (a whole
        // slice of one range is one round trip)
        const int j0 = P.row_seg[r], j1 = P.row_seg[r + 1];
        uint32_t base = 0;
        for (int j = j0; j < j1 && base < q1; ++j) {
            const RcpSeg sg = P.segs[j];
            for (int s = 0; s < 3 && base < q1; ++s) {
                const uint32_t lo = P.seg_lo[j * 3 + s], hi = P.seg_hi[j * 3 + s];
                const uint32_t c = hi > lo ? hi - lo : 0;
                const uint32_t a = max(q0, base), b = min(q1, base + c);
                if (a < b) {
                    const uint32_t i0 = lo + (a - base), i1 = lo + (b - base);
                    // wave-uniform trip count: run_add needs every lane of the wave
                    const uint32_t lane = threadIdx.x & 63;
                    for (uint32_t wb = i0 + (threadIdx.x & ~63u); wb < i1; wb += kHeavyLoads * kBlock) {
                        const uint32_t i = wb + lane;
                        int2 rd[kHeavyLoads];
#pragma unroll
                        for (int u = 0; u < kHeavyLoads; ++u) rd[u] = P.se[min(i + u * kBlock, i1 - 1)];
                        if (sg.multi) {
#pragma unroll
                            for (int u = 0; u < kHeavyLoads; ++u)
                                if (i + u * kBlock < i1) add_read(P, sg, rd[u], sg.lo, sg.hi, 0, diff, 30);
                        } else {
#pragma unroll
                            for (int u = 0; u < kHeavyLoads; ++u) {
                                // add_read with weight 1, the two atomics merged per run
                                const int2 x = rd[u];
                                const bool act = i + u * kBlock < i1 && !(x.y < sg.lo || x.x > sg.hi);
                                const int32_t x0 = max(x.x, sg.lo), x1 = min(x.y, sg.hi);
                                const int32_t o0 = sg.rev ? sg.off + (sg.hi - x1) : sg.off + (x0 - sg.lo);
                                const int32_t o1 = sg.rev ? sg.off + (sg.hi - x0) : sg.off + (x1 - sg.lo);
                                run_add(diff, o0, act, 1);
                                run_add(diff, o1 + 1, act, -1);
                            }
                        }
                    }
                }
                base += c;
            }
        }
        __syncthreads();
        int32_t* g = P.heavy_gdiff + (size_t)slot * P.heavy_stride;
        for (int q = threadIdx.x; q <= nr; q += kBlock) {
            const int32_t v = diff[q];
            if (v) atomicAdd(&g[q], v);
        }
        __syncthreads();
    }
}

// =================================================================================
// pileup -> bins -> column-major profile (or CSR coverage)
// =================================================================================
// A workgroup owns kRounds x kTile rows x one column chunk.  Per round, each of the 4 waves
// piles up 2 rows (one at a time) into its own LDS difference array and stages the bin
// numerators; the block then writes the round's kTile rows column by column.
//
// Latency: all per-row metadata (segment, read ranges per strand stream, refined for the
// chunk) is resolved once per workgroup by one thread per row (parallel binary searches),
// and each wave issues the loads of its NEXT row's first 256 candidate reads before
// working on the current row's LDS, so a row's HBM round trip overlaps the previous row.
constexpr int kPWaves = 8;  // waves per pileup workgroup (they share one stage)
constexpr int kPBlock = 64 * kPWaves;
constexpr int kRounds = 4;  // at most 4 rounds of kTile rows per workgroup (RcpPlanDev::rounds)
static_assert(kTile % kPWaves == 0, "a round's rows are split evenly over the waves");
constexpr int kRowsPerWave = kTile / kPWaves;  // rows a wave piles per round
constexpr int kAhead = 1;  // rows whose first reads are prefetched
constexpr int kRows = kTile * kRounds;  // rows per workgroup

struct RowMeta {  // [kRows] each, in LDS
    int32_t flag, bs, lay, P0, npos, kend, heavy;
    int32_t fast;                 // 1 = single range, reads resolved below
    int32_t off, slo, shi, rev;   // the range: row offset, genomic run, reversed
    int32_t gps, gpe;             // genomic piece covered by this chunk
    uint32_t lo[3], hi[3];        // candidate reads per strand stream (refined to the piece)
};
constexpr int kMetaWords = sizeof(RowMeta) / 4;

// Row metadata in SGPRs: every field is wave-uniform (read from LDS, made scalar)
__device__ __forceinline__ RowMeta uniform_meta(const RowMeta& src) {
    RowMeta m;
    const int32_t* s = reinterpret_cast<const int32_t*>(&src);
    int32_t* d = reinterpret_cast<int32_t*>(&m);
#pragma unroll
    for (int q = 0; q < kMetaWords; ++q) d[q] = __builtin_amdgcn_readfirstlane(s[q]);
    return m;
}

__device__ __forceinline__ uint32_t fast_candidates(const RowMeta& m) {
    return (m.hi[0] - m.lo[0]) + (m.hi[1] - m.lo[1]) + (m.hi[2] - m.lo[2]);
}

// index of candidate q of a fast row (q < fast_candidates)
__device__ __forceinline__ uint32_t fast_index(const RowMeta& m, uint32_t q) {
    // one stream (the merged layout, or a strand-specific row): a scalar test, no selects
    if (m.hi[1] == m.lo[1] && m.hi[2] == m.lo[2]) return m.lo[0] + q;
    const uint32_t c0 = m.hi[0] - m.lo[0];
    const uint32_t c1 = m.hi[1] - m.lo[1];
    return q < c0 ? m.lo[0] + q : (q < c0 + c1 ? m.lo[1] + (q - c0) : m.lo[2] + (q - c0 - c1));
}

// Same as add_read_fast with the orientation known at compile time: the chunk positions of
// the read's first covered base and of the base after its last are one add each.
template <bool REV>
__device__ __forceinline__ void add_read_fast_t(const RowMeta& m, int2 rd, int32_t* diff, int sh) {
    if (rd.y < m.gps || rd.x > m.gpe) return;
    const int32_t x0 = max(rd.x, m.gps);
    const int32_t x1 = min(rd.y, m.gpe);
    int32_t a, b;
    if (!REV) {
        const int32_t k = m.off - m.slo - m.P0;  // wave-uniform
        a = x0 + k;
        b = x1 + k + 1;
    } else {
        const int32_t k = m.off + m.shi - m.P0;
        a = k - x1;
        b = k - x0 + 1;
    }
    atomicAdd(&diff[lp(a, sh)], 1);
    atomicAdd(&diff[lp(b, sh)], -1);
}

__device__ __forceinline__ void add_read_fast(const RowMeta& m, int2 rd, int32_t* diff, int sh) {
    if (rd.y < m.gps || rd.x > m.gpe) return;
    const int32_t x0 = max(rd.x, m.gps);
    const int32_t x1 = min(rd.y, m.gpe);
    int32_t o0, o1;
    if (!m.rev) {
        o0 = m.off + (x0 - m.slo);
        o1 = m.off + (x1 - m.slo);
    } else {
        o0 = m.off + (m.shi - x1);
        o1 = m.off + (m.shi - x0);
    }
    atomicAdd(&diff[lp(o0 - m.P0, sh)], 1);
    atomicAdd(&diff[lp(o1 - m.P0 + 1, sh)], -1);
}

// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup-scope release of
// all address spaces, which on gfx9 waits for vmcnt(0): every global store of the previous
// epilogue (and every prefetched read) would have to land before the barrier.  The pileup
// kernel's waves share nothing through global memory, so LDS ordering is enough.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ void lds_order() {
    // a wave's LDS operations complete in issue order; keep the compiler from moving them
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// Words per stage row: >= cap and = 4 (mod 8), so a row's bins are consecutive (b128
// writes stay aligned) and 16 rows x 4 consecutive columns fall in 64 distinct banks.
__host__ __device__ __forceinline__ int stage_stride(int cap) { return ((cap + 3) >> 3 << 3) + 4; }

// Fused pass for uniform bins of 2^lbs positions with 2^lbs <= PER (every bin inside one
// lane's positions): read the lane's PER differences once, zero them for the next row, turn
// them into depth with one wave scan and write the lane's bin sums straight to the stage row.
// Replaces zeroing + two scan passes + the bin reads of the general path.
template <int PER>
__device__ __forceinline__ void scan_bins_fast(int32_t* diff, int lbs, uint32_t* srow, int32_t nbins) {
    const int lane = threadIdx.x & 63;
    uint4* base = reinterpret_cast<uint4*>(diff + lane * (PER + 4));
    uint32_t v[PER];
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
        const uint4 x = base[q];
        v[4 * q] = x.x;
        v[4 * q + 1] = x.y;
        v[4 * q + 2] = x.z;
        v[4 * q + 3] = x.w;
    }
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) base[q] = make_uint4(0u, 0u, 0u, 0u);
    uint32_t A = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) A += v[j];
    uint32_t d = wave_exclusive_scan(A);  // depth entering this lane
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        d += v[j];
        v[j] = d;
    }
    // bin sums by pairwise levels (uniform branches; register indices stay static)
#pragma unroll
    for (int L = 1; (1 << L) <= PER; ++L) {
        if (L <= lbs) {
#pragma unroll
            for (int i = 0; i < (PER >> L); ++i) v[i] = v[2 * i] + v[2 * i + 1];
        }
    }
    const int nb = PER >> lbs;
    const int b0 = lane * nb;
    if (nb >= 4) {
#pragma unroll
        for (int m = 0; m < PER; m += 4) {
            if (m < nb) {
                if (b0 + m + 3 < nbins) {
                    *reinterpret_cast<uint4*>(srow + b0 + m) = make_uint4(v[m], v[m + 1], v[m + 2], v[m + 3]);
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (b0 + m + u < nbins) srow[b0 + m + u] = v[m + u];
                }
            }
        }
    } else {
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if (m < nb && b0 + m < nbins) srow[b0 + m] = v[m];
    }
}

// write-once output: non-temporal stores keep the reads' lines in L2 / MALL
__device__ __forceinline__ void out_store(double x, double* p) {
    __builtin_nontemporal_store(x, p);
}

// Row metadata of row r for column chunk (part, k0, cidx), from the locate kernel's 64-byte
// record (one thread per row; the refine searches of all rows are in flight together).
// flag: 0 = pile up, 1 = NULL row (zeros), 2 = not this kernel's (interp / outside).
template <bool MEDIAN, bool CSR>
__device__ __forceinline__ RowMeta decode_row(const RcpPlanDev& P, const RcpPart& part, int32_t k0, int cidx, int r) {
    RowMeta m;
    m.flag = 2; m.bs = 0; m.lay = -1; m.P0 = 0; m.npos = 0; m.kend = k0; m.heavy = -1; m.fast = 0;
    m.off = m.slo = m.shi = m.rev = m.gps = m.gpe = 0;
    for (int s = 0; s < 3; ++s) m.lo[s] = m.hi[s] = 0;
    if (r < P.n_rows) {
        RcpRowRec rec;
        {
            const uint4* src = reinterpret_cast<const uint4*>(P.rec + r);
            uint4* dst = reinterpret_cast<uint4*>(&rec);
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[q] = src[q];
        }
        // the merged layout's chunk range: its address does not depend on the record, so it is
        // loaded with it (one round trip, not two); used only when the record says CRANGE
        uint2 cr_pre = make_uint2(0u, 0u);
        if (P.crange && P.merged) cr_pre = P.crange[(size_t)r * P.n_chunks_total + cidx];
        int32_t head, L;
        rcp_part_slice(part, rec.row_len, &head, &L);
        const int32_t n = CSR ? L : part.n_bins;
        m.kend = min(k0 + part.chunk_bins, n);
        if (!(rec.flags & RCP_REC_VALID)) {
            m.flag = CSR ? 2 : 1;  // NULL row -> zeros (profile.R:191-197)
        } else if (k0 >= n) {
            m.flag = 2;
        } else if (!part.per_base && L < n) {
            m.flag = 2;  // interpolation rows: rcp_interp_kernel
        } else if (part.per_base && !CSR && L != n) {
            atomicOr(P.status, RCP_STATUS_WIDTH);
            m.flag = 1;
        } else {
            if (part.per_base) {
                m.bs = 1;
            } else {
                m.bs = L / n;
                const int32_t dif = L - m.bs * n;
                if (dif) {
                    m.lay = P.lay_index[part.lay_base + dif];
                    if (m.lay < 0) {
                        atomicOr(P.status, RCP_STATUS_INTERP);
                        m.lay = -1;
                    }
                }
            }
            const int32_t e0 = bin_edge(m.bs, m.lay, P.lay_cnt, k0);
            const int32_t e1 = bin_edge(m.bs, m.lay, P.lay_cnt, m.kend);
            m.P0 = head + e0;
            m.npos = e1 - e0;
            m.flag = 0;
            // median bins wider than a wave chunk: rcp_interp_kernel (mode 4)
            if (MEDIAN && m.bs + (m.lay >= 0 ? 1 : 0) > P.chunk_cap) m.flag = 2;
            m.heavy = rec.heavy;
            if (m.heavy < 0 && m.npos <= P.chunk_cap && (rec.flags & RCP_REC_FAST)) {
                const int32_t len = rec.shi - rec.slo + 1;
                const int32_t a = max(m.P0, rec.off);
                const int32_t b = min(m.P0 + m.npos, rec.off + len);
                m.fast = 1;
                m.off = rec.off; m.slo = rec.slo; m.shi = rec.shi; m.rev = rec.rev;
                if (a < b) {
                    if (!rec.rev) {
                        m.gps = rec.slo + (a - rec.off);
                        m.gpe = rec.slo + (b - 1 - rec.off);
                    } else {
                        m.gpe = rec.shi - (a - rec.off);
                        m.gps = rec.shi - (b - 1 - rec.off);
                    }
                    const bool full = (a == rec.off) && (b == rec.off + len);
                    uint32_t all = 0;
                    for (int s = 0; s < 3; ++s) all += rec.hi[s] - rec.lo[s];
                    // a chunk of a modest row streams all the row's reads (the piece
                    // check drops the others; they are L2 hits for the sibling chunks);
                    // only big rows pay the dependent binary searches
                    const bool refine = !full && all > 4096;
                    if (rec.flags & RCP_REC_CRANGE) {
                        // exact ranges for this chunk from the locate kernel
                        if (P.merged) {  // one stream: dense (row, chunk) words
                            const uint2 v = cr_pre;
                            m.lo[0] = v.x;
                            m.hi[0] = v.y;
                            m.lo[1] = m.hi[1] = m.lo[2] = m.hi[2] = 0;
                        } else {
                            const uint2* cr = P.crange + ((size_t)r * P.n_chunks_total + cidx) * 3;
                            for (int s = 0; s < 3; ++s) {
                                const uint2 v = cr[s];
                                m.lo[s] = v.x;
                                m.hi[s] = v.y;
                            }
                        }
                    } else
                    for (int s = 0; s < 3; ++s) {
                        uint32_t lo = rec.lo[s], hi = rec.hi[s];
                        if (lo < hi && refine) {
                            lo = lower_bound_pmax(P.pmax, lo, hi, m.gps);
                            hi = upper_bound_start(P.se, lo, hi, m.gpe);
                        }
                        m.lo[s] = lo;
                        m.hi[s] = lo < hi ? hi : lo;
                    }
                }
            }
        }
    }
    return m;
}


// Fold plans (P.fold; rcp_host.cpp sets it for small single-range tables in the merged layout):
// the locate kernel's work for row r and one column chunk done by the pileup kernel itself --
// four bound searches per row: (0, 1) the row's lower / upper bound, for the row hit and the NULL
// rules (R/coverage.R:189-225), (2, 3) the chunk piece's, i.e. its candidate reads (the locate
// kernel's crange).  No locate launch and no 64-B record round trip.  fold_geom is the part before
// the searches (the chunk's slice of the row and its genomic piece), fold_finish the part after
// (validity, written by the row's first lane in chunk 0, and the row's metadata).
struct FoldRow {
    RcpRowInfo ri;
    RowMeta m;
    bool in, ok, pile, piece;
    int32_t L, n, gps, gpe;
};

__device__ __forceinline__ void fold_geom(const RcpPlanDev& P, const RcpPart& part, int32_t k0, int r, FoldRow& f) {
    RowMeta& m = f.m;
    m.flag = 2; m.bs = 0; m.lay = -1; m.P0 = 0; m.npos = 0; m.kend = k0; m.heavy = -1; m.fast = 0;
    m.off = m.slo = m.shi = m.rev = m.gps = m.gpe = 0;
    for (int s = 0; s < 3; ++s) m.lo[s] = m.hi[s] = 0;
    f.in = r < P.n_rows;
    {
        uint4* d = reinterpret_cast<uint4*>(&f.ri);
        const uint4* src = reinterpret_cast<const uint4*>(P.row_info + (f.in ? r : 0));
#pragma unroll
        for (int u = 0; u < (int)(sizeof(RcpRowInfo) / 16); ++u) d[u] = f.in ? src[u] : make_uint4(0u, 0u, 0u, 0u);
    }
    const RcpRowInfo& ri = f.ri;
    const RcpSeg& sg = ri.seg0;
    f.ok = f.in && !ri.stat && ri.chrom >= 0 && ri.chrom < P.n_chrom && ri.j1 == ri.j0 + 1 && sg.query_ok &&
           (sg.streams & 1);
    // the chunk's slice of the row (decode_row)
    int32_t head = 0;
    rcp_part_slice(part, ri.row_len, &head, &f.L);
    f.n = part.n_bins;
    m.kend = min(k0 + part.chunk_bins, f.n);
    f.pile = false;
    if (f.in && k0 < f.n && !(!part.per_base && f.L < f.n)) {
        if (part.per_base && f.L != f.n) {
            m.flag = 1;  // (a width mismatch: raised by fold_finish when the row is valid)
        } else {
            f.pile = true;
            if (part.per_base) {
                m.bs = 1;
            } else {
                m.bs = f.L / f.n;
                const int32_t dif = f.L - m.bs * f.n;
                if (dif) {
                    m.lay = P.lay_index[part.lay_base + dif];
                    if (m.lay < 0) m.lay = -1;
                }
            }
            const int32_t e0 = bin_edge(m.bs, m.lay, P.lay_cnt, k0);
            const int32_t e1 = bin_edge(m.bs, m.lay, P.lay_cnt, m.kend);
            m.P0 = head + e0;
            m.npos = e1 - e0;
        }
    }
    // the chunk's genomic piece of the range
    const int32_t len = sg.hi - sg.lo + 1;
    const int32_t a = max(m.P0, sg.off), b = min(m.P0 + m.npos, sg.off + len);
    f.piece = f.pile && a < b;
    f.gps = f.gpe = 0;
    if (f.piece) {
        if (!sg.rev) {
            f.gps = sg.lo + (a - sg.off);
            f.gpe = sg.lo + (b - 1 - sg.off);
        } else {
            f.gpe = sg.hi - (a - sg.off);
            f.gps = sg.hi - (b - 1 - sg.off);
        }
    }
}

// first: the lane that writes the row's validity and raises its status bits; coop_min: chunks of
// more candidate reads (fused-bins rows) are marked heavy = -2 -- the general kernel's workgroup
// piles them together (coop_row) -- or 0: never
template <bool MEDIAN>
__device__ __forceinline__ RowMeta fold_finish(const RcpPlanDev& P, const RcpPart& part, int cidx, int r, FoldRow& f,
                                               uint32_t rlo, uint32_t rhi, uint32_t plo, uint32_t phi, bool first,
                                               uint32_t coop_min) {
    RowMeta& m = f.m;
    const RcpRowInfo& ri = f.ri;
    const RcpSeg& sg = ri.seg0;
    rhi = max(rlo, rhi);
    bool valid = f.ok && rlo < rhi;
    // Rle[i2k] past the Rle -> NULL: seqlength, or the hits' last end when NA (locate_rows)
    if (valid) valid = ri.seqlen >= 0 ? (int64_t)sg.hi <= ri.seqlen : sg.hi <= P.pmax[rhi - 1];
    if (f.in && first && cidx == 0) {
        P.valid[r] = valid ? 1 : 0;
        if (P.valid_out) P.valid_out[r] = valid ? 1 : 0;
    }
    if (!f.in) return m;
    if (!valid) {
        m.flag = 1;  // NULL row -> zeros (profile.R:191-197)
        return m;
    }
    if (!f.pile) {
        if (m.flag == 1 && first) atomicOr(P.status, RCP_STATUS_WIDTH);  // per-base width mismatch
        return m;
    }
    if (m.lay < 0 && !part.per_base && f.L - m.bs * f.n != 0) {
        if (first) atomicOr(P.status, RCP_STATUS_INTERP);
    }
    m.flag = 0;
    if (MEDIAN && m.bs + (m.lay >= 0 ? 1 : 0) > P.chunk_cap) {
        m.flag = 2;
        return m;
    }
    if (m.npos <= P.chunk_cap) {
        m.fast = 1;
        m.off = sg.off; m.slo = sg.lo; m.shi = sg.hi; m.rev = sg.rev;
        if (f.piece) {
            m.gps = f.gps;
            m.gpe = f.gpe;
            const uint32_t clo = max(rlo, plo);
            m.lo[0] = clo;
            m.hi[0] = max(clo, min(rhi, phi));
            const int need = (m.npos + 1 + 63) >> 6;
            const int per = need <= 4 ? 4 : 1 << (32 - __clz(need - 1));
            const bool fused = !MEDIAN && m.lay < 0 && (m.bs & (m.bs - 1)) == 0 && m.bs <= per && per <= 16;
            if (coop_min && fused && m.hi[0] - m.lo[0] > coop_min) m.heavy = -2;
        }
    }
    return m;
}

// A bound search (dir_bound_multi: lower_bound(pmax >= v) or, up, upper_bound(start > v),
// inside v's bucket of the directory at entry d0, nb buckets) by a group of G consecutive lanes
// of one wave (G divides 64, group-aligned): after the bucket's directory line, each step probes G
// points at once and keeps the (G + 1)-th of the interval holding the answer -- log_{G+1} of the
// bucket's reads in dependent loads instead of log_2.  Returns the same index as the bisection, in
// every lane of the group.
template <int G>
__device__ __forceinline__ uint32_t dir_bound_group(const RcpPlanDev& P, int64_t d0, int32_t nb, int32_t v, bool up,
                                                    bool active) {
    const int lane = threadIdx.x & 63;
    const int j = lane % G;
    const int gbase = lane - j;
    const int64_t thr = (int64_t)v + (up ? 1 : 0);
    uint32_t lo = 0, hi = 0;
    if (active) {
        const int32_t b = min(max(v, 0) >> P.dir_shift, nb - 1);
        if (P.dir_k) {
            constexpr int kQ = 4, kKeys = 4 * kQ - 2;
            const int4* src = reinterpret_cast<const int4*>(P.dir_k + 32 * (d0 + b) + (up ? 16 : 0));
            int4 w[kQ];
#pragma unroll
            for (int q = 0; q < kQ; ++q) w[q] = src[q];
            const int32_t* x = reinterpret_cast<const int32_t*>(w);
            const int32_t n = x[1] - x[0];
            uint32_t c = 0;
#pragma unroll
            for (int i = 0; i < kKeys; ++i) c += (i < n && (int64_t)x[2 + i] < thr) ? 1u : 0u;
            if (n <= kKeys) {
                lo = (uint32_t)x[0] + c;
                hi = c < (uint32_t)kKeys ? lo : (uint32_t)x[1];
            } else {
                lo = (uint32_t)x[0] + (c ? (uint32_t)rcp_dirk_offset(n, (int)c - 1) + 1u : 0u);
                hi = c < (uint32_t)kKeys ? (uint32_t)x[0] + (uint32_t)rcp_dirk_offset(n, (int)c) : (uint32_t)x[1];
            }
        } else {
            const int32_t* dir = up ? P.dir_u : P.dir_l;
            lo = (uint32_t)dir[2 * (d0 + b)];
            hi = (uint32_t)dir[2 * (d0 + b + 1)];
        }
    }
    const int32_t* se = reinterpret_cast<const int32_t*>(P.se);
    const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << gbase;
    while (true) {
        const bool go = active && lo < hi;  // (uniform in the group)
        if (!__ballot(go)) break;
        const uint64_t width = hi - lo;
        const uint32_t m = lo + (uint32_t)(((uint64_t)(j + 1) * width) / (G + 1));
        bool pred = false;
        if (go) pred = (int64_t)(up ? se[(size_t)m << 1] : P.pmax[m]) < thr;
        // the probes below the threshold are a prefix (sorted keys): the answer is past the c-th
        const uint32_t c = (uint32_t)__popcll(__ballot(pred) & gmask);
        if (go) {
            const uint32_t nlo = c ? lo + (uint32_t)(((uint64_t)c * width) / (G + 1)) + 1u : lo;
            const uint32_t nhi = c < (uint32_t)G ? lo + (uint32_t)(((uint64_t)(c + 1) * width) / (G + 1)) : hi;
            lo = nlo;
            hi = nhi;
        }
    }
    return lo;
}

// The general kernel's fold: the 4 G lanes of the row (G = 512 / (4 x the workgroup's rows): the
// whole workgroup), search s by lanes G s .. G s + G - 1 (dir_bound_group); skewed fused-bins
// chunks marked for the workgroup (P.coop_min)
template <bool MEDIAN, int G>
__device__ __forceinline__ RowMeta fold_row(const RcpPlanDev& P, const RcpPart& part, int32_t k0, int cidx, int r) {
    const int lane = threadIdx.x & 63;
    const int rbase = lane & ~(4 * G - 1);  // the row's first lane
    const int q = (lane - rbase) / G;       // its search
    FoldRow f;
    fold_geom(P, part, k0, r, f);
    const RcpSeg& sg = f.ri.seg0;
    const int32_t v = q == 0 ? sg.lo : (q == 1 ? sg.hi : (q == 2 ? f.gps : f.gpe));
    const uint32_t res = dir_bound_group<G>(P, f.ri.d0, f.ri.nb, v, (q & 1) != 0, f.ok && (q < 2 || f.piece));
    return fold_finish<MEDIAN>(P, part, cidx, r, f, (uint32_t)__shfl((int)res, rbase),
                               (uint32_t)__shfl((int)res, rbase + G), (uint32_t)__shfl((int)res, rbase + 2 * G),
                               (uint32_t)__shfl((int)res, rbase + 3 * G), lane == rbase, (uint32_t)P.coop_min);
}

// The lean kernel's fold (store wave 0 decoding the next item's 32 rows): two lanes per row, each
// bisecting two bounds in lockstep (dir_bound_multi) -- lane 2 i the row's, lane 2 i + 1 the
// chunk piece's; no cooperative rows (the lean kernel deals rows to single waves)
__device__ __forceinline__ RowMeta fold_row_pair(const RcpPlanDev& P, const RcpPart& part, int32_t k0, int cidx, int r) {
    const int lane = threadIdx.x & 63;
    const int h = lane & 1, rb = lane & ~1;
    FoldRow f;
    fold_geom(P, part, k0, r, f);
    const RcpSeg& sg = f.ri.seg0;
    const int64_t d0[2] = {f.ri.d0, f.ri.d0};
    const int32_t nb[2] = {f.ri.nb, f.ri.nb};
    const int32_t v[2] = {h ? f.gps : sg.lo, h ? f.gpe : sg.hi};
    const int dst[2] = {-2, -1};
    uint32_t res[2] = {0u, 0u};
    dir_bound_multi<2>(P, d0, nb, v, dst, (f.ok && (h == 0 || f.piece)) ? 2 : 0, res);
    return fold_finish<false>(P, part, cidx, r, f, (uint32_t)__shfl((int)res[0], rb), (uint32_t)__shfl((int)res[1], rb),
                              (uint32_t)__shfl((int)res[0], rb + 1), (uint32_t)__shfl((int)res[1], rb + 1), h == 0, 0u);
}

template <bool MEDIAN, bool CSR, bool UNI>
__global__ void __launch_bounds__(kPBlock) __attribute__((amdgpu_waves_per_eu(4))) rcp_pileup_kernel(RcpPlanDev P, double* __restrict__ out,
                                                            int64_t* __restrict__ binsum) {
    // UNI (plan st != null): reads of one width, streamed as their starts alone (the lean kernel's
    // start-only stream): 4-B loads, end = start + st_w formed when a read is added
    using RdT = typename std::conditional<UNI, int32_t, int2>::type;
    auto rd_load = [&](uint32_t idx) -> RdT {
        if constexpr (UNI) return P.st[idx];
        else return P.se[idx];
    };
    auto rd_pair = [&](RdT v) -> int2 {
        if constexpr (UNI) return make_int2(v, v + P.st_w);
        else return v;
    };
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int T = kTile;
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    // ---- decode (row block, part, chunk)
    // blocks of one row block (all its column chunks) are b, b + 8, b + 16, ...: one XCD
    // under round-robin dispatch, so a chunk's re-read of the rows' reads hits that L2
    // (placement only changes speed, never results)
    const int grp = blockIdx.x / (8 * P.n_chunks_total);
    const int wg = blockIdx.x - grp * 8 * P.n_chunks_total;
    int c = wg >> 3;
    const int cidx = c;  // column chunk over all parts
    const int blk = grp * 8 + (wg & 7);
    const int rounds = P.rounds;        // rounds of T rows (<= kRounds)
    const int rows_wg = T * rounds;     // rows of this workgroup
    if (blk * rows_wg >= P.n_rows) return;
    int p = 0;
    while (p < P.n_parts - 1 && c >= P.part[p].n_chunks) {
        c -= P.part[p].n_chunks;
        ++p;
    }
    const RcpPart part = P.part[p];
    const int32_t k0 = c * part.chunk_bins;
    const int row0 = blk * rows_wg;

    // per wave: 8 zero words (so cum[lp(-1)] == 0) then the padded difference / depth /
    // cumulative array; the stage is [row][RS] (stage_stride)
    const int RS = stage_stride(P.stage_cap);
    int32_t* diff = reinterpret_cast<int32_t*>(smem) + wave * (P.wave_words + 8) + 8;
    uint32_t* stage = reinterpret_cast<uint32_t*>(smem) + kPWaves * (P.wave_words + 8);
    RowMeta* meta = reinterpret_cast<RowMeta*>(stage + (CSR ? 0 : T * RS));

    // ---- per-row metadata, one thread per row, from the locate kernel's 64-byte records -- or,
    // in a fold plan, a quad of lanes per row searching its read ranges (fold_row)
    if (!CSR && P.fold) {
        // the whole workgroup: 512 / rows_wg lanes per row, a quarter of them per search
        auto fold = [&](auto gc) {
            constexpr int G = decltype(gc)::value;
            const int i = tid / (4 * G);
            const RowMeta m = fold_row<MEDIAN, G>(P, part, k0, cidx, row0 + i);
            if (tid % (4 * G) == 0) meta[i] = m;
        };
        static_assert(kPBlock == 512, "fold lanes per row: 512 / rows");
        if (rows_wg == 64) fold(std::integral_constant<int, 2>());
        else if (rows_wg == 32) fold(std::integral_constant<int, 4>());
        else fold(std::integral_constant<int, 8>());
        // no heavy launch: the status set the next execution uses is zeroed here (nothing in this
        // execution reads it)
        if (blockIdx.x == 0 && tid < RCP_STATUS_WORDS) P.status_prev[tid] = 0u;
    } else if (tid < rows_wg) {
        meta[tid] = decode_row<MEDIAN, CSR>(P, part, k0, cidx, row0 + tid);
    }
    uint32_t* ctr = reinterpret_cast<uint32_t*>(meta + kRows);  // row counter (RCP_GEN_DYN), in the tail words
    if (tid == 0) *ctr = 0u;
    lds_barrier();
    // fold plans: the rows the whole workgroup piles (heavy = -2), one bit per workgroup row
    uint64_t coop_bits = 0;
    if (!CSR && !MEDIAN && P.fold) coop_bits = __ballot(lane < rows_wg && meta[lane].heavy == -2);

    // ---- rows of this wave (static dealing): round rd, sub s -> row rd*T + s*kPWaves + wave
    [[maybe_unused]] auto row_of = [&](int step) { return (step / kRowsPerWave) * T + (step % kRowsPerWave) * kPWaves + wave; };
    // software pipeline: the first 256 candidate reads of the next kAhead rows are in flight
    // while a row is piled up (registers are free: LDS, not VGPRs, limits occupancy)
    [[maybe_unused]] const int n_steps = kRowsPerWave * rounds;
    auto prefetch = [&](int i, RdT* dst) {
        const RowMeta m = uniform_meta(meta[i]);
        const uint32_t n = (m.flag == 0 && m.fast && m.heavy != -2) ? fast_candidates(m) : 0;
        if (n) {  // wave-uniform
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                // unconditional (clamped) loads: no divergent branch, no early vmcnt wait
                const uint32_t q = lane + 64 * u;
                dst[u] = rd_load(fast_index(m, q < n ? q : n - 1));
            }
        }
    };
    static_assert(kAhead == 1 && kRowsPerWave % 2 == 0, "ping-pong prefetch buffers: one row ahead, even rows per round");
    // Two read buffers used alternately (no register copies across steps): a copy at the loop
    // back-edge would need the prefetched reads to have landed right after the epilogue's
    // stores, and gfx9's single in-order vmcnt would make that wait for the stores too.
    RdT bufA[4], bufB[4];
    // ---- round epilogue: stage row -> out[col * n_rows + row].  Thread t serves row t % 16
    // and column quads t / 16, t / 16 + 32, ...: one 16-B stage read feeds four stores, and
    // the 16 lanes of a quad column write 16 consecutive rows (128 B) of one column.
    auto flush = [&](int rd) {
        const int rbase = rd * T;
        const int ii = tid & (T - 1);
        const int r = row0 + rbase + ii;
        const RowMeta& mr = meta[rbase + ii];
        const int32_t flag = mr.flag, kend = mr.kend, bs = mr.bs, lay = mr.lay;
        if (r >= P.n_rows || flag == 2) return;
        const size_t R = (size_t)P.out_ld;  // column stride of the output (>= n_rows)
        constexpr int kQuads = kPBlock / T;  // column quads per pass
        constexpr int kStep = 4 * kQuads;    // columns per pass
        const int32_t kq = k0 + 4 * (tid / T);
        const size_t o0 = (size_t)(part.col_off + kq) * R + (size_t)r;
        const size_t ostep = (size_t)kStep * R;
        const uint32_t* st0 = stage + ii * RS + 4 * (tid / T);
        // value of bin k from its stage count: zero row / one divisor / splitVector layout
        const double sc = P.scale;
        const int32_t den = MEDIAN ? 2 : bs;
        const double dd = (double)den;
        const bool pow2 = (MEDIAN || lay < 0) && (den & (den - 1)) == 0;
        const double rdd = 1.0 / dd;
        auto put4 = [&](int32_t k, double* o, const double (&x)[4]) {
            if (k + 3 < kend) {
#pragma unroll
                for (int u = 0; u < 4; ++u) out_store(x[u], o + u * R);
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (k + u < kend) out_store(x[u], o + u * R);
            }
        };
        double* o = out + o0;
        if (flag == 1) {
            const double z[4] = {0.0, 0.0, 0.0, 0.0};
            for (int32_t k = kq; k < kend; k += kStep, o += ostep) put4(k, o, z);
        } else if (pow2) {
            // a power of two divides exactly by its reciprocal
            const uint32_t* st = st0;
            for (int32_t k = kq; k < kend; k += kStep, o += ostep, st += kStep) {
                const uint4 q = *reinterpret_cast<const uint4*>(st);
                const double x[4] = {((double)q.x * sc) * rdd, ((double)q.y * sc) * rdd,
                                     ((double)q.z * sc) * rdd, ((double)q.w * sc) * rdd};
                put4(k, o, x);
            }
        } else if (MEDIAN || lay < 0) {
            // RN(x / den) through the row's correctly rounded reciprocal (rcp_div_rn: bit-equal
            // to the division, a third of its instructions)
            const uint32_t* st = st0;
            for (int32_t k = kq; k < kend; k += kStep, o += ostep, st += kStep) {
                const uint4 q = *reinterpret_cast<const uint4*>(st);
                const double x[4] = {rcp_div_rn((double)q.x * sc, dd, rdd), rcp_div_rn((double)q.y * sc, dd, rdd),
                                     rcp_div_rn((double)q.z * sc, dd, rdd), rcp_div_rn((double)q.w * sc, dd, rdd)};
                put4(k, o, x);
            }
        } else {
            // splitVector layout: bins of bs or bs + 1 positions, one reciprocal each
            const int32_t* cnt = P.lay_cnt + lay;
            const double dd1 = (double)(bs + 1), rdd1 = 1.0 / dd1;
            const uint32_t* st = st0;
            for (int32_t k = kq; k < kend; k += kStep, o += ostep, st += kStep) {
                const uint4 q = *reinterpret_cast<const uint4*>(st);
                const uint32_t num[4] = {q.x, q.y, q.z, q.w};
                double x[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool enl = k + u < kend && cnt[k + u + 1] != cnt[k + u];
                    x[u] = k + u < kend ? rcp_div_rn((double)num[u] * sc, enl ? dd1 : dd, enl ? rdd1 : rdd) : 0.0;
                }
                put4(k, o, x);
            }
        }
        if (binsum) {  // optional int64 bin sums, same layout
            int64_t* bo = binsum + o0;
            const uint32_t* st = st0;
            for (int32_t k = kq; k < kend; k += kStep, bo += ostep, st += kStep) {
                const uint4 q = flag == 1 ? make_uint4(0u, 0u, 0u, 0u) : *reinterpret_cast<const uint4*>(st);
                const uint32_t num[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (k + u < kend) bo[u * R] = (int64_t)num[u];
            }
        }
    };
    bool clean = false;  // this wave's difference array is all zero (layout clean_sh)
    int clean_sh = -1;
    // one row of this wave: `cur` holds its first reads; the next row's go to `nxt`
    // pile row i of the workgroup (round i / T), its first reads in `cur`
    auto pile_row = [&](int i, RdT (&cur)[4]) __attribute__((always_inline)) {
        const RowMeta m = uniform_meta(meta[i]);
        uint32_t* sbuf = stage;  // this round's stage
        if (m.flag == 0 && m.heavy != -2) {  // wave-uniform: scalar branch (-2: piled by coop_row)
            const int r = row0 + i;
            const int32_t npos = m.npos;
            const int32_t bs = m.bs, lay = m.lay, kend = m.kend;
            const int ii = i & (T - 1);
            const int32_t e0 = bin_edge(bs, lay, P.lay_cnt, k0);
            // positions [P0, P0 + npos) in sub-chunks of at most chunk_cap positions; a bin
            // that straddles sub-chunks accumulates its partial sums in the stage
            for (int32_t s0 = 0; s0 < npos; s0 += P.chunk_cap) {
                const int32_t sn = min(P.chunk_cap, npos - s0);
                const bool whole = sn == npos;
                if (MEDIAN && !whole) {  // the host keeps median bins inside one chunk
                    if (lane == 0) atomicOr(P.status, RCP_STATUS_INTERP);
                    break;
                }
                // per-lane positions: a power of two >= 4 (lane chunks padded by 4 words)
                const int need = (sn + 1 + 63) >> 6;
                const int sh = need <= 4 ? 2 : 32 - __clz(need - 1);
                const int per = 1 << sh;
                // the fused pass leaves the array zeroed for the next row of the same geometry
                const bool fast_bins = !MEDIAN && !CSR && whole && lay < 0 && (bs & (bs - 1)) == 0 && bs <= per &&
                                       per <= 16;
                if (!(clean && clean_sh == sh)) {
                    int4* d4 = reinterpret_cast<int4*>(diff);
                    for (int q = lane - 2; q < (per + 4) * 16; q += 64) d4[q] = make_int4(0, 0, 0, 0);
                }
                clean = fast_bins;
                clean_sh = sh;
                lds_order();
                if (m.heavy >= 0) {
                    // skewed row: its difference array was piled up by rcp_heavy_pileup_kernel
                    const int32_t* g = P.heavy_gdiff + (size_t)m.heavy * P.heavy_stride;
                    const int32_t base = m.P0 + s0;
                    int32_t carry = 0;
                    for (int q = lane; q < base; q += 64) carry += g[q];
                    carry = wave_sum(carry);
                    for (int q = lane; q <= sn; q += 64) diff[lp(q, sh)] = g[base + q] + (q == 0 ? carry : 0);
                } else if (m.fast && whole) {
                    const uint32_t n = fast_candidates(m);
                    // batch q0 + 256 is loaded while batch q0 is added
                    for (uint32_t q0 = 0; q0 < n; q0 += 256) {
                        RdT nx[4];
                        if (q0 + 256 < n) {
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const uint32_t q = q0 + 256 + lane + 64 * u;
                                nx[u] = rd_load(fast_index(m, q < n ? q : n - 1));
                            }
                        }
                        if (m.rev) {  // wave-uniform orientation
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                if (q0 + lane + 64u * u < n) add_read_fast_t<true>(m, rd_pair(cur[u]), diff, sh);
                        } else {
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                if (q0 + lane + 64u * u < n) add_read_fast_t<false>(m, rd_pair(cur[u]), diff, sh);
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) cur[u] = nx[u];
                    }
                } else {
                    pileup_row_wave(P, r, m.P0 + s0, sn, diff, sh);
                }
                lds_order();
                if (!MEDIAN && !CSR && fast_bins) {
                    uint32_t* srow = sbuf + ii * RS;
                    const int lbs = 31 - __clz(bs);
                    if (sh == 2) scan_bins_fast<4>(diff, lbs, srow, kend - k0);
                    else if (sh == 3) scan_bins_fast<8>(diff, lbs, srow, kend - k0);
                    else scan_bins_fast<16>(diff, lbs, srow, kend - k0);
                    lds_order();
                    continue;
                }
                scan_wave<!(MEDIAN || CSR)>(diff, per);
                lds_order();
                if (CSR && P.csr_rs) {
                    // run starts of this chunk (its first position always: the seams are
                    // merged by rcp_cov_runs_plan_kernel), compacted in position order
                    int2* rs_out = P.csr_rs + P.csr_off[r] + k0 + s0;
                    const uint64_t below = (1ull << lane) - 1;
                    uint32_t e = 0;
                    int32_t carry = 0, lastv = 0;
                    for (int32_t q0 = 0; q0 < sn; q0 += 64) {
                        const int32_t q = q0 + lane;
                        const bool in = q < sn;
                        const int32_t v = in ? diff[lp(q, sh)] : 0;
                        const int32_t pv = __builtin_amdgcn_update_dpp(carry, v, 0x138, 0xf, 0xf, false);
                        const bool f = in && (q == 0 || v != pv);
                        const uint64_t mk = __ballot(f);
                        if (f) rs_out[e + (uint32_t)__popcll(mk & below)] = make_int2(v, k0 + s0 + q);
                        e += (uint32_t)__popcll(mk);
                        carry = __builtin_amdgcn_readlane(v, 63);
                        if (q0 + 64 >= sn) lastv = __builtin_amdgcn_readlane(v, sn - 1 - q0);
                    }
                    if (lane == 0) P.csr_sub[P.csr_sub_off[r] + cidx + s0 / P.chunk_cap] = make_int2((int32_t)e, lastv);
                } else if (CSR) {
                    int32_t* orow = P.csr_out + P.csr_off[r];
                    for (int32_t q = lane; q < sn; q += 64) orow[k0 + s0 + q] = diff[lp(q, sh)];
                } else if (MEDIAN) {
                    for (int32_t k = k0 + lane; k < kend; k += 64) {
                        const int32_t a = bin_edge(bs, lay, P.lay_cnt, k) - e0;
                        const int32_t b = bin_edge(bs, lay, P.lay_cnt, k + 1) - e0;
                        const int32_t mm = b - a;
                        int32_t vmin = INT32_MAX, vmax = INT32_MIN;
                        for (int32_t q = a; q < b; ++q) {
                            const int32_t v = diff[lp(q, sh)];
                            vmin = min(vmin, v);
                            vmax = max(vmax, v);
                        }
                        const int32_t h = (mm + 1) >> 1;
                        const uint32_t x1 = (vmin == vmax) ? (uint32_t)vmin : kth_smallest(diff, a, b, h, vmin, vmax, sh);
                        uint32_t x2 = x1;
                        if (!(mm & 1))
                            x2 = (vmin == vmax) ? (uint32_t)vmin : kth_smallest(diff, a, b, h + 1, vmin, vmax, sh);
                        sbuf[ii * RS + (k - k0)] = x1 + x2;  // 2 x median
                    }
                } else if (whole && lay < 0) {
                    // uniform bins: bin k spans cum positions [a, a + bs), cum[lp(-1)] == 0
                    const uint32_t* cum = reinterpret_cast<const uint32_t*>(diff);
                    int32_t a = lane * bs;
                    uint32_t* st = sbuf + ii * RS + lane;
                    for (int32_t k = k0 + lane; k < kend; k += 64, a += 64 * bs, st += 64)
                        *st = cum[lp(a + bs - 1, sh)] - cum[lp(a - 1, sh)];
                } else if (whole) {
                    // splitVector layout: enlarged bins from set.seed(42); sample(1:n, dif)
                    const uint32_t* cum = reinterpret_cast<const uint32_t*>(diff);
                    for (int32_t k = k0 + lane; k < kend; k += 64) {
                        const int32_t a = bin_edge(bs, lay, P.lay_cnt, k) - e0;
                        const int32_t b = bin_edge(bs, lay, P.lay_cnt, k + 1) - e0;
                        sbuf[ii * RS + (k - k0)] = cum[lp(b - 1, sh)] - cum[lp(a - 1, sh)];
                    }
                } else {
                    // sub-chunk [s0, s0 + sn): add each overlapping bin's partial sum
                    const uint32_t* cum = reinterpret_cast<const uint32_t*>(diff);
                    for (int32_t k = k0 + lane; k < kend; k += 64) {
                        const int32_t a = max(bin_edge(bs, lay, P.lay_cnt, k) - e0, s0) - s0;
                        const int32_t b = min(bin_edge(bs, lay, P.lay_cnt, k + 1) - e0, s0 + sn) - s0;
                        uint32_t* st = sbuf + ii * RS + (k - k0);
                        const uint32_t part_sum = a < b ? cum[lp(b - 1, sh)] - cum[lp(a - 1, sh)] : 0u;
                        *st = (s0 == 0 ? 0u : *st) + part_sum;
                    }
                }
                lds_order();
            }
        }
    };
    // rows of round rd piled by the whole workgroup (coop_row, below)
    auto round_coop = [&](int rd) { return (uint32_t)(coop_bits >> (rd * T)) & ((1u << T) - 1u); };
    auto pile_step = [&](int step, RdT (&cur)[4], RdT (&nxt)[4]) __attribute__((always_inline)) {
        // (a round that starts with cooperative rows prefetches its first row after them: no read
        // buffer is held across that phase)
        const int ns = step + 1;
        if (ns < n_steps && !(ns % kRowsPerWave == 0 && round_coop(ns / kRowsPerWave))) prefetch(row_of(ns), nxt);
        pile_row(row_of(step), cur);
    };
    // a skewed row of a fold plan (no heavy slices): every wave piles batches w, w + 8, ... of its
    // reads into the difference array of wave `owner`, which then stages its bin sums (fused
    // pass) -- 8 waves on the row instead of one
    auto coop_row = [&](int i, int owner) __attribute__((always_inline)) {
        const RowMeta m = uniform_meta(meta[i]);
        const int need = (m.npos + 1 + 63) >> 6;
        const int sh = need <= 4 ? 2 : 32 - __clz(need - 1);
        int32_t* od = reinterpret_cast<int32_t*>(smem) + owner * (P.wave_words + 8) + 8;
        if (wave == owner) {
            if (!(clean && clean_sh == sh)) {
                int4* d4 = reinterpret_cast<int4*>(od);
                for (int q = lane - 2; q < ((1 << sh) + 4) * 16; q += 64) d4[q] = make_int4(0, 0, 0, 0);
            }
            clean = false;
        }
        lds_barrier();
        // every lane keeps KC reads in flight (a wave's 64 KC consecutive reads per round trip, the
        // workgroup's 8 waves on interleaved batches: the heavy-slice kernel's memory parallelism);
        // a skewed row's reads pile onto few positions, so equal positions of neighbouring lanes
        // are one LDS add per run (run_add)
        constexpr int KC = UNI ? 16 : 8;
        const uint32_t n = fast_candidates(m);
        const int32_t kf = m.off - m.slo - m.P0, kr = m.off + m.shi - m.P0;
        for (uint32_t wb = 64u * KC * (uint32_t)wave; wb < n; wb += 64u * KC * kPWaves) {
            RdT rdv[KC];
#pragma unroll
            for (int u = 0; u < KC; ++u) {
                const uint32_t q = wb + 64u * u + lane;
                rdv[u] = rd_load(fast_index(m, q < n ? q : n - 1));
            }
#pragma unroll
            for (int u = 0; u < KC; ++u) {
                const int2 x = rd_pair(rdv[u]);
                const bool act = wb + 64u * u + lane < n && !(x.y < m.gps || x.x > m.gpe);
                const int32_t x0 = max(x.x, m.gps), x1 = min(x.y, m.gpe);
                const int32_t a0 = m.rev ? kr - x1 : x0 + kf;
                const int32_t b0 = m.rev ? kr - x0 + 1 : x1 + kf + 1;
                run_add(od, lp(a0, sh), act, 1);
                run_add(od, lp(b0, sh), act, -1);
            }
        }
        lds_barrier();
        if (wave == owner) {
            uint32_t* srow = stage + (i & (T - 1)) * RS;
            const int lbs = 31 - __clz(m.bs);
            if (sh == 2) scan_bins_fast<4>(od, lbs, srow, m.kend - k0);
            else if (sh == 3) scan_bins_fast<8>(od, lbs, srow, m.kend - k0);
            else scan_bins_fast<16>(od, lbs, srow, m.kend - k0);
            lds_order();
            clean = true;  // (the fused pass leaves the array zeroed)
            clean_sh = sh;
        }
    };
    if (!round_coop(0)) prefetch(row_of(0), bufA);
    for (int rd = 0; rd < rounds; ++rd) {
        if (!CSR && !MEDIAN) {
            uint32_t cm = round_coop(rd);  // (wave-uniform)
            if (cm) {
                for (int c = 0; cm; ++c, cm &= cm - 1) coop_row(rd * T + __builtin_ctz(cm), c & (kPWaves - 1));
                prefetch(row_of(rd * kRowsPerWave), bufA);
            }
        }
        for (int s2 = 0; s2 < kRowsPerWave; s2 += 2) {
            pile_step(rd * kRowsPerWave + s2, bufA, bufB);
            pile_step(rd * kRowsPerWave + s2 + 1, bufB, bufA);
        }
        if (CSR) continue;
        lds_barrier();
        flush(rd);
        lds_barrier();
    }
}



#include "rcp_splitvector.h"  // splitVector interpolation (also rcp_interp_kernel below)

// ---------------------------------------------------------------------------------
// Row-wave pileup kernel (mean bins; P.lean == 3): every wave owns whole rows.  For plans
// whose rows are lists of ranges (coverageRnaRef's c(flank, exons, flank), genebody rows with
// flanks) the (row tile, column chunk) work items of the general kernel cost a dependent chain
// of round trips per chunk (pair table -> piece bounds -> first reads) and a workgroup barrier
// per round that waits for the round's longest row.  Here a wave claims a row (per-XCD
// counters, then the other XCDs' leftovers), loads its (segment, stream) pair table once, and
// walks the row's parts in windows of <= kRWCap positions -- usually one window per part --
// streaming each pair's reads once (pieces cut by a window edge are narrowed by the bucket
// directory, no bisection), then scans the window and writes its bins straight to the R
// column-major output.  No barrier anywhere: waves are independent, so the row-length skew
// of exon lists only costs the wave that drew the long row.
// ---------------------------------------------------------------------------------
constexpr int kRWaves = 4;                       // waves per workgroup (independent)
constexpr int kRWSh = 5;                         // 32 positions per lane at most
template <int SH>
struct RowWin {
    static constexpr int cap = 64 * (1 << SH) - 1;          // positions per window (+1 sentinel)
    static constexpr int words = 8 + 64 * ((1 << SH) + 4);  // per wave: 8 zero words + padded array
};
constexpr int kRWCap = RowWin<kRWSh>::cap;
// The tiles' bin numerators are staged row-major in HBM (uint32, P.rm32) and flushed
// column-major by the last wave to finish one of a tile's rows.  (Staging them in LDS instead --
// one 8-wave workgroup per CU, two 16-row slots -- measured slower: C3 0.73 vs 0.57 ms, and the
// fp64 means instead of numerators 1.21x vs 1.09x of the algorithmic traffic;
// profiles/r04/r4j/c3.log, r4n/)
constexpr int kRWGSlots = 4;   // tiles in flight per workgroup (<= 6)
constexpr int kRWGWaves = 16;  // waves per workgroup of the staged kernel (one 16-wave workgroup
                               // per CU keeps fewer tiles in flight: C3 pileup 0.573 -> 0.495 ms,
                               // profiles/r04/r4m/c3.log)
constexpr size_t kRowsQueueBytes = 64;  // tile queue word + slot table

extern "C" int rcp_rows_window_cap(void) { return kRWCap; }

static size_t rows_lds_bytes(int waves, int words) { return 4 * (size_t)waves * words + kRowsQueueBytes; }

// Stores of a row's bins without a stage (binsum, which keeps the column-major layout): 8 bytes
// per 128-B column line; the 16 rows of a line are claimed together by waves of one XCD, so
// plain stores meet in that L2.
__device__ __forceinline__ void rows_store(double x, double* p) { *p = x; }

// a bin's mean from its numerator: the same operations in the same order wherever it is made
// (pile or LDS flush), so the same bits
__device__ __forceinline__ double rows_mean(uint32_t num, double sc, bool pow2, int32_t w, int32_t bs, double dd,
                                            double rdd, double dd1, double rdd1) {
    if (pow2) return ((double)num * sc) * rdd;
    if (w == bs) return rcp_div_rn((double)num * sc, dd, rdd);
    return rcp_div_rn((double)num * sc, dd1, rdd1);  // w == bs + 1
}

// MODE 1: bin numerators staged in the row-major HBM stage P.rm32 (row stride n_cols, part
// info P.rinfo), tiles flushed by the last wave to finish one of their rows; 0 (binsum): means
// stored straight into the column-major output.
template <int MODE, int WAVES, int SH>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(4)))
rcp_pileup_rows_kernel(RcpPlanDev P, double* __restrict__ out, int64_t* __restrict__ binsum) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int kWinCap = RowWin<SH>::cap, kWords = RowWin<SH>::words;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    int32_t* diff = reinterpret_cast<int32_t*>(smem) + wave * kWords + 8;
    if (lane < 8) diff[lane - 8] = 0;  // cum[lp(-1)] == 0
    const int xcd = blockIdx.x & 7;
    const int n_tiles = (P.n_rows + kTile - 1) / kTile;
    const size_t R = (size_t)P.out_ld;
    const int ns = P.merged ? 1 : 3;
    const double sc = P.scale;
    // Work: tiles of 16 rows (one 128-B line of every output column).  Workgroups on XCD x take
    // tiles x, x + 8, ... from that XCD's counter (then the other XCDs' leftovers): one global
    // atomic per tile.  Inside the workgroup the four waves take the tile's rows one at a time
    // from a 64-bit LDS word (tile << 32 | next row); the wave that draws row index 16 fetches
    // the next tile and publishes it, waves drawing past 16 wait for the new tile.
    unsigned long long* queue = reinterpret_cast<unsigned long long*>(smem + 4 * WAVES * kWords);
    constexpr uint32_t kEmpty = 0xFFFFFFFEu, kDone = 0xFFFFFFFFu;
    // tile slots of the flush: tile id, rows finished (kFree: flushed),
    // and the workgroup's tile sequence number (slot = seq % kSlots)
    constexpr int kSlots = kRWGSlots;
    static_assert(8 + 8 * kSlots + 4 <= (int)kRowsQueueBytes, "slot table");
    constexpr uint32_t kFree = 0xFFFFFFFFu;
    uint32_t* slot_tile = reinterpret_cast<uint32_t*>(queue + 1);
    uint32_t* slot_cnt = slot_tile + kSlots;
    uint32_t* seq = slot_cnt + kSlots;
    // row r's staged numerators [n_cols] and part info [part] {bs, lay} (bs 0: zeros, -1: left
    // to the interpolation kernel)
    const int ldw = MODE == 1 ? (int)P.n_cols : 0;
    auto stage_row = [&](int r, int) -> uint32_t* { return MODE == 1 ? P.rm32 + (size_t)r * ldw : nullptr; };
    auto stage_info = [&](int r, int) -> int2* { return P.rinfo + (size_t)r * RCP_MAX_PARTS; };
    if (threadIdx.x == 0) *queue = ((unsigned long long)kEmpty << 32) | kTile;
    if (threadIdx.x < kSlots) {
        slot_tile[threadIdx.x] = kDone;
        slot_cnt[threadIdx.x] = kFree;
    }
    if (threadIdx.x == 0) *seq = 0;
    // a folded plan launches no locate / heavy kernel: zero the status set the next execution
    // uses here (nothing in this execution reads it)
    if (P.fold && blockIdx.x == 0 && threadIdx.x < RCP_STATUS_WORDS) P.status_prev[threadIdx.x] = 0u;
    __syncthreads();
    constexpr bool staged = MODE != 0;
    auto fetch_tile = [&]() -> uint32_t {
        for (int k = 0; k < 8; ++k) {
            const int xs = (xcd + k) & 7;
            const uint32_t nt = (uint32_t)max((n_tiles - xs + 7) / 8, 0);
            if (nt == 0) continue;
            uint32_t j = 0;
            if (lane == 0) j = atomicAdd(&P.status[8 + xs], 1u);
            j = __builtin_amdgcn_readfirstlane(j);
            if (j < nt) return P.tile_perm && P.interp_stage ? (uint32_t)P.tile_perm[j * 8 + xs] : j * 8 + xs;
        }
        return kDone;
    };
    auto claim = [&]() -> int {
        while (true) {
            unsigned long long w = 0;
            if (lane == 0) w = atomicAdd(queue, 1ull);
            const uint32_t tile = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(w >> 32));
            const uint32_t idx = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)w);
            if (tile == kDone) return -1;
            if (idx < (uint32_t)kTile && tile != kEmpty) {
                const int r = (int)tile * kTile + (int)idx;
                if (r < P.n_rows) return r;
                continue;  // the short last tile
            }
            if (idx == (uint32_t)kTile) {
                const uint32_t t = fetch_tile();
                if (staged && t != kDone) {
                    // the tile's slot: free once the tile kSlots before it has been flushed (its
                    // last rows are in progress on other waves, which never wait on this one)
                    const uint32_t sl = *(volatile uint32_t*)seq % kSlots;
                    while ((uint32_t)__builtin_amdgcn_readfirstlane((int)*(volatile uint32_t*)&slot_cnt[sl]) != kFree)
                        __builtin_amdgcn_s_sleep(2);
                    if (lane == 0) {
                        slot_tile[sl] = t;
                        slot_cnt[sl] = 0;
                        *seq = *seq + 1;
                    }
                    lds_order();
                }
                if (lane == 0) atomicExch(queue, ((unsigned long long)t << 32));
                continue;
            }
            // another wave is fetching the next tile
            while ((uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(*(volatile unsigned long long*)queue >> 32)) == tile)
                __builtin_amdgcn_s_sleep(2);
        }
    };
    // the matrix cell (row r, column c) of the unstaged mode (binsum)
    auto cell = [&](int r, int64_t c) -> double* { return out + (size_t)c * R + r; };
    auto zero_cols = [&](int r, const RcpPart& part, int32_t n) {
        if (staged) return;  // the row's part info says zeros
        for (int32_t k = lane; k < n; k += 64) {
            rows_store(0.0, cell(r, part.col_off + k));
            if (binsum) binsum[(size_t)(part.col_off + k) * R + r] = 0;
        }
    };
    // the last wave to finish a row of tile T writes the tile's 16 rows of every column from the
    // stage as whole 128-B column lines (release / acquire: the other waves' staging stores are
    // visible to it); lane = (row i, column quarter): 4 columns x 16 rows per store
    auto flush = [&](uint32_t T, int sl) {
        const int32_t t16 = (int32_t)T * kTile;
        const int32_t nrow = min(kTile, P.n_rows - t16);
        const int i = lane & 15, cq = lane >> 4;
        {
            // numerators -> means (the pile's operations), 4 columns x 16 rows per store
            const uint32_t* srow = stage_row(t16 + i, sl);
            const int2* inf = stage_info(t16 + i, sl);
            const double sc = P.scale;
            for (int p = 0; p < P.n_parts; ++p) {
                const int32_t n = P.part[p].n_bins, c0p = P.part[p].col_off;
                const int2 f = i < nrow ? inf[p] : make_int2(-1, -1);
                const int32_t bs = max(f.x, 1), lay = f.y;
                const bool pow2 = lay < 0 && (bs & (bs - 1)) == 0;
                const double dd = (double)bs, rdd = 1.0 / dd;
                const double dd1 = (double)(bs + 1), rdd1 = 1.0 / dd1;
                // the stage words (and the enlarged-bin mask word) of the next 32 columns are
                // loaded before this step's stores: one vmcnt counts loads and stores in order on
                // gfx9, so a load issued after the stores would wait for their acknowledgements
                auto load_step = [&](int32_t k0, uint32_t (&q)[8], uint32_t& bits) {
                    // enlarged bins of the 32 columns (R-RNG layout) as one mask word
                    bits = (f.x > 0 && lay >= 0) ? P.lay_bit[lay + (k0 >> 5)] : 0u;
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int32_t k = k0 + 4 * u + cq;
                        q[u] = (f.x > 0 && k < n) ? srow[c0p + k] : 0u;
                    }
                };
                uint32_t q[8], bits = 0;
                load_step(0, q, bits);
                for (int32_t k0 = 0; k0 < n; k0 += 32) {
                    uint32_t qn[8], bitsn = 0;
                    if (k0 + 32 < n) load_step(k0 + 32, qn, bitsn);
                    double v[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int32_t k = k0 + 4 * u + cq;
                        v[u] = 0.0;
                        if (f.x > 0 && k < n) {
                            const int32_t w = bs + (int32_t)((bits >> (4 * u + cq)) & 1u);
                            v[u] = rows_mean(q[u], sc, pow2, w, bs, dd, rdd, dd1, rdd1);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int32_t k = k0 + 4 * u + cq;
                        if (f.x >= 0 && k < n)
                            __builtin_nontemporal_store(v[u], out + (size_t)(c0p + k) * R + (size_t)(t16 + i));
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) q[u] = qn[u];
                    bits = bitsn;
                }
            }
        }
    };
    auto slot_of = [&](int r) {
        const uint32_t T = (uint32_t)(r / kTile);
        int sl = 0;
        for (int k = 1; k < kSlots; ++k)
            if (slot_tile[k] == T) sl = k;
        return sl;
    };
    auto row_done = [&](int r, int sl) {
        const uint32_t T = (uint32_t)(r / kTile);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        uint32_t old = 0;
        if (lane == 0) old = atomicAdd(&slot_cnt[sl], 1u);
        old = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
        if ((int32_t)old + 1 == min(kTile, P.n_rows - (int32_t)T * kTile)) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            flush(T, sl);
            lds_order();
            if (lane == 0) atomicExch(&slot_cnt[sl], kFree);
        }
    };
    auto row_body = [&](int r, int sl) {
        const RcpRowInfo& ri = P.row_info[r];
        const int j0 = ri.j0, j1 = ri.j1;
        const int64_t d0 = ri.d0;
        const int32_t dnb = ri.nb;
        const int n_all = (j1 - j0) * ns;
        int32_t flags = 0, nr = 0, heavy = -1;
        uint32_t itp_parts = 0;  // parts this wave interpolates after the row (interp_rows)
        if (P.fold) {
            nr = ri.row_len;
        } else {
            const uint4 rc = *reinterpret_cast<const uint4*>(P.rec + r);  // flags, row_len, heavy, off
            flags = (int32_t)__builtin_amdgcn_readfirstlane((int)rc.x);
            nr = (int32_t)__builtin_amdgcn_readfirstlane((int)rc.y);
            heavy = (int32_t)__builtin_amdgcn_readfirstlane((int)rc.z);
        }
        // P.fold: rcp_locate_kernel's searches for this row, here (bucket directory + bisection,
        // dir_bound_multi).  Pairs t0 .. t0 + 63: in round k lane l searches bound l >> 5 (lower,
        // upper) of pair t0 + 32 k + (l & 31) -- one search's directory line per lane, not two --
        // and lane t then gathers pair t0 + t's two bounds; a second round only for > 32 pairs.
        // Call with the whole wave.
        const int32_t chrom = ri.chrom;
        const bool rok = P.fold && !ri.stat && chrom >= 0 && chrom < P.n_chrom && j1 > j0;
        auto fold_bounds = [&](int t0, uint32_t& lo, uint32_t& hi) {
            uint32_t res[2] = {0u, 0u};
            const int half = lane >> 5;
            for (int k = 0; k < 2 && t0 + 32 * k < n_all; ++k) {  // (wave-uniform)
                const int q = t0 + 32 * k + (lane & 31);
                int64_t dd[1] = {d0};
                int32_t nb1[1] = {dnb};
                int32_t v[1] = {0};
                const int dst[1] = {half ? -1 : -2};
                int cnt = 0;
                if (rok && q < n_all) {
                    const int st = q % ns;
                    const RcpSeg sg = P.segs[j0 + q / ns];
                    if (sg.query_ok && ((sg.streams >> st) & 1)) {
                        cnt = 1;
                        v[0] = half ? sg.hi : sg.lo;
                        if (!P.merged) {
                            dd[0] = P.dir_off[chrom * 3 + st];
                            nb1[0] = (int32_t)(P.dir_off[chrom * 3 + st + 1] - dd[0]) - 1;
                        }
                    }
                }
                uint32_t w[1];
                dir_bound_multi<1>(P, dd, nb1, v, dst, cnt, w);
                res[k] = w[0];
            }
            const int src = lane & 31;
            const uint32_t l0 = (uint32_t)__shfl((int)res[0], src), h0 = (uint32_t)__shfl((int)res[0], src + 32);
            const uint32_t l1 = (uint32_t)__shfl((int)res[1], src), h1 = (uint32_t)__shfl((int)res[1], src + 32);
            lo = lane < 32 ? l0 : l1;
            hi = max(lo, lane < 32 ? h0 : h1);
        };
        // lane t: pair t0 + t of the row (pairs 64.. are reloaded per window); the whole wave
        auto load_pair = [&](int t0, RcpSeg& sg, uint32_t& lo, uint32_t& hi, int& st) {
            const int t = t0 + lane;
            sg = RcpSeg{};
            lo = hi = 0;
            st = 0;
            uint32_t flo = 0, fhi = 0;
            if (P.fold) fold_bounds(t0, flo, fhi);
            if (t < n_all) {
                const int j = j0 + t / ns;
                st = t % ns;
                sg = P.segs[j];
                const bool use = sg.query_ok && ((sg.streams >> st) & 1);
                if (P.fold) {
                    lo = flo;
                    hi = fhi;
                } else {
                    lo = P.seg_lo[j * 3 + st];
                    hi = P.seg_hi[j * 3 + st];
                }
                if (!use) hi = lo;
            }
        };
        RcpSeg sg0;
        uint32_t plo0, phi0;
        int pst0;
        load_pair(0, sg0, plo0, phi0, pst0);
        if (P.fold) {
            // the NULL rules (R/coverage.R:189-225, as rcp_locate_kernel): every group of the row
            // needs a hit, and its last position inside seqlength -- or, when that is NA, inside
            // the group's hits' last end
            const int64_t seqlen = ri.seqlen;
            bool valid = rok;
            const bool wide = P.n_interp > 0 && !P.interp_stage;  // rcp_interp_kernel piles from seg_lo / seg_hi
            uint32_t present = 0, hit = 0, past = 0;
            int32_t maxpos[4] = {INT32_MIN, INT32_MIN, INT32_MIN, INT32_MIN};
            int32_t maxend[4] = {INT32_MIN, INT32_MIN, INT32_MIN, INT32_MIN};
            for (int t0 = 0; rok && t0 < n_all; t0 += 64) {
                RcpSeg sg = sg0;
                uint32_t lo = plo0, hi = phi0;
                int st = pst0;
                if (t0 > 0) load_pair(t0, sg, lo, hi, st);
                if (t0 + lane < n_all) {
                    const int g = sg.group & 3;
                    present |= 1u << g;
                    if (lo < hi) hit |= 1u << g;
                    if (seqlen >= 0) {
                        if ((int64_t)sg.hi > seqlen) past |= 1u << g;
                    } else {
                        const int32_t me = lo < hi ? P.pmax[hi - 1] : INT32_MIN;
#pragma unroll
                        for (int gg = 0; gg < 4; ++gg) {  // (registers: no dynamically indexed array)
                            if (gg == g) {
                                maxpos[gg] = max(maxpos[gg], sg.hi);
                                maxend[gg] = max(maxend[gg], me);
                            }
                        }
                    }
                    if (wide) {
                        const int j = j0 + (t0 + lane) / ns;
                        P.seg_lo[j * 3 + st] = lo;
                        P.seg_hi[j * 3 + st] = hi;
                    }
                }
            }
            if (rok) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    if (!__ballot((present >> g) & 1)) continue;
                    bool ok_g = __ballot((hit >> g) & 1) != 0;
                    if (seqlen >= 0) {
                        ok_g = ok_g && !__ballot((past >> g) & 1);
                    } else {
                        int32_t mp = maxpos[g], me = maxend[g];
                        for (int o = 32; o > 0; o >>= 1) {
                            mp = max(mp, __shfl_xor(mp, o));
                            me = max(me, __shfl_xor(me, o));
                        }
                        ok_g = ok_g && mp <= me;
                    }
                    valid = valid && ok_g;
                }
            }
            flags = valid ? RCP_REC_VALID : 0;
        }
        uint32_t* const srow = stage_row(r, sl);
        int2* const sinfo = stage_info(r, sl);
        // the row's validity and its parts' stage info (lane p: part p; zeros unless piled
        // below) are stored when the row is done: one vmcnt counts loads and stores in order on
        // gfx9, so a store here would put its round trip on the row's first read loads
        int2 info = make_int2(0, -1);
        auto commit = [&]() {
            if (P.fold && lane == 0) {
                P.valid[r] = (flags & RCP_REC_VALID) ? 1 : 0;
                if (P.valid_out) P.valid_out[r] = (flags & RCP_REC_VALID) ? 1 : 0;
            }
            if (staged && lane < P.n_parts) sinfo[lane] = info;
        };
        if (!(flags & RCP_REC_VALID)) {  // NULL row -> zeros (profile.R:191-197)
            for (int p = 0; p < P.n_parts; ++p) zero_cols(r, P.part[p], P.part[p].n_bins);
            commit();
            return itp_parts;
        }

        for (int p = 0; p < P.n_parts; ++p) {
            const RcpPart part = P.part[p];
            int32_t head, L;
            rcp_part_slice(part, nr, &head, &L);
            const int32_t n_bins = part.n_bins;
            // interpolation row (fewer positions than bins): rcp_interp_kernel writes its columns.
            // With the HBM stage (P.interp_stage) this wave piles its L positions as L one-position
            // bins into the first L stage words of the part, and the interpolation kernel, run
            // after this one, takes the depth from there instead of piling the row again.
            const bool itp = !part.per_base && L < n_bins;
            if (itp) {
                if (lane == p) info = make_int2(-1, -1);
                if (!staged || !P.interp_stage) continue;
            }
            const int32_t n = itp ? L : n_bins;  // the bins of this pass
            // ... and with P.interp_of this wave interpolates the row itself (below): the depth goes
            // to the entry's scratch doubles, the spline's serial chains run here, beside the other
            // waves' pileup, instead of in a kernel after it
            const int e_itp = itp && P.interp_of ? P.interp_of[(size_t)r * P.n_parts + p] : -1;
            double* const xs = e_itp >= 0 ? P.interp_scratch + (size_t)e_itp * P.interp_stride : nullptr;
            if (part.per_base && L != n) {
                if (lane == 0) atomicOr(P.status, RCP_STATUS_WIDTH);
                zero_cols(r, part, n);
                continue;
            }
            int32_t bs = 1, lay = -1;
            if (!part.per_base && !itp) {
                bs = L / n;
                const int32_t dif = L - bs * n;
                if (dif) {
                    lay = P.lay_index[part.lay_base + dif];
                    if (lay < 0) {
                        if (lane == 0) atomicOr(P.status, RCP_STATUS_INTERP);
                        lay = -1;
                    }
                }
            }
            if (lane == p && !itp) info = make_int2(bs, lay);
            const int32_t kw = max(1, kWinCap / (bs + (lay >= 0 ? 1 : 0)));  // bins per window
            const bool pow2 = lay < 0 && (bs & (bs - 1)) == 0;
            const double dd = (double)bs, rdd = 1.0 / dd;
            const double dd1 = (double)(bs + 1), rdd1 = 1.0 / dd1;  // an enlarged bin's width
            for (int32_t k0 = 0; k0 < n; k0 += kw) {
                const int32_t k1 = min(n, k0 + kw);
                const int32_t e0 = bin_edge(bs, lay, P.lay_cnt, k0);
                const int32_t npos = bin_edge(bs, lay, P.lay_cnt, k1) - e0;
                const int32_t W0 = head + e0, W1 = W0 + npos;
                const int need = (npos + 1 + 63) >> 6;
                const int sh = need <= 4 ? 2 : 32 - __clz(need - 1);
                const int per = 1 << sh;
                {
                    int4* d4 = reinterpret_cast<int4*>(diff);
                    for (int q = lane; q < (per + 4) * 16; q += 64) d4[q] = make_int4(0, 0, 0, 0);
                }
                lds_order();
                if (heavy >= 0) {
                    // skewed row: its difference array was piled up by rcp_heavy_pileup_kernel
                    const int32_t* g = P.heavy_gdiff + (size_t)heavy * P.heavy_stride;
                    int32_t carry = 0;
                    for (int q = lane; q < W0; q += 64) carry += g[q];
                    carry = wave_sum(carry);
                    for (int q = lane; q <= npos; q += 64) diff[lp(q, sh)] = g[W0 + q] + (q == 0 ? carry : 0);
                } else {
                    for (int t0 = 0; t0 < n_all; t0 += 64) {
                        RcpSeg sg = sg0;
                        uint32_t lo = plo0, hi = phi0;
                        int st = pst0;
                        if (t0 > 0) load_pair(t0, sg, lo, hi, st);
                        // this pair's piece of the window
                        const int32_t len = sg.hi - sg.lo + 1;
                        const int32_t a = max(W0, sg.off), b = min(W1, sg.off + len);
                        int32_t gps = 0, gpe = -1;
                        if (a < b && lo < hi) {
                            if (!sg.rev) {
                                gps = sg.lo + (a - sg.off);
                                gpe = sg.lo + (b - 1 - sg.off);
                            } else {
                                gpe = sg.hi - (a - sg.off);
                                gps = sg.hi - (b - 1 - sg.off);
                            }
                            const bool full = (a == sg.off) && (b == sg.off + len);
                            if (!full && (P.merged || st == 0)) {
                                // reads of the piece lie inside the directory buckets of its ends
                                const int32_t bl = min(max(gps, 0) >> P.dir_shift, dnb - 1);
                                const int32_t bu = min(max(gpe, 0) >> P.dir_shift, dnb - 1);
                                lo = max(lo, (uint32_t)P.dir_l[2 * (d0 + bl)]);
                                hi = min(hi, (uint32_t)P.dir_u[2 * (d0 + bu + 1)]);
                            } else if (!full && hi - lo > 1024) {
                                lo = lower_bound_pmax(P.pmax, lo, hi, gps);
                                hi = upper_bound_start(P.se, lo, hi, gpe);
                            }
                            if (hi < lo) hi = lo;
                        } else {
                            hi = lo;
                        }
                        pile_pairs(P, sg, gps, gpe, lo, hi, W0, diff, sh);
                    }
                }
                lds_order();
                scan_wave<true>(diff, per);
                lds_order();
                // bins [k0, k1): numerator = cum[b - 1] - cum[a - 1] (exact integers; the same
                // divisions as the general kernel's epilogue, so the same bits)
                const uint32_t* cum = reinterpret_cast<const uint32_t*>(diff);
                // four bins a lane per step, their layout edges loaded together before any store:
                // gfx9 waits for a load and every earlier store with one counter, so a store
                // between two bins' edge loads put a store round trip on each bin
                for (int32_t kb = k0 + lane; kb < k1; kb += 256) {
                    int32_t ea[4], eb[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int32_t k = min(kb + 64 * u, k1 - 1);
                        ea[u] = bin_edge(bs, lay, P.lay_cnt, k) - e0;
                        eb[u] = bin_edge(bs, lay, P.lay_cnt, k + 1) - e0;
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int32_t k = kb + 64 * u;
                        if (k >= k1) break;
                        const int32_t a = ea[u], b = eb[u];
                        const uint32_t num = cum[lp(b - 1, sh)] - cum[lp(a - 1, sh)];
                        if (xs) {
                            xs[k] = (double)num * sc;  // (rcp_interp_kernel's x[i])
                            continue;
                        }
                        if (staged) {
                            srow[part.col_off + k] = num;
                            continue;
                        }
                        rows_store(rows_mean(num, sc, pow2, b - a, bs, dd, rdd, dd1, rdd1), cell(r, part.col_off + k));
                        if (binsum) binsum[(size_t)(part.col_off + k) * R + r] = (int64_t)num;
                    }
                }
                lds_order();
            }
            if (xs) itp_parts |= 1u << p;
        }
        commit();
        return itp_parts;
    };
    // splitVector of row r's piled slices (itp_parts: the parts with an interpolation entry) into
    // their columns, as rcp_interp_kernel would: run after the row, where little else is live
    auto interp_rows = [&](int r, uint32_t itp_parts) {
        for (int p = 0; p < P.n_parts; ++p) {
            if (!((itp_parts >> p) & 1)) continue;
            const int e = P.interp_of[(size_t)r * P.n_parts + p];
            const RcpPart part = P.part[p];
            int32_t head, L;
            rcp_part_slice(part, P.row_info[r].row_len, &head, &L);
            const int mode = P.interp_mode[e];
            interp_finish_wave(mode, L, part.n_bins, P.interp_scratch + (size_t)e * P.interp_stride,
                               mode == 3 ? P.nb_pos + P.interp_pos[e] : nullptr, P.spl_tb,
                               out + (size_t)part.col_off * R + r, R);
        }
    };
    for (int r = claim(); r >= 0; r = claim()) {
        const int sl = staged ? slot_of(r) : 0;
        const uint32_t itp_parts = row_body(r, sl);
        if (staged) row_done(r, sl);
        if (itp_parts) interp_rows(r, itp_parts);
    }
    // the last workgroup out resets the tile counters for the next launch
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const uint32_t done = atomicAdd(&P.status[16], 1u);
        if (done == gridDim.x - 1) {
            for (int x = 0; x < 8; ++x) atomicExch(&P.status[8 + x], 0u);
            atomicExch(&P.status[16], 0u);
        }
    }
}

// ---------------------------------------------------------------------------------
// Lean pileup kernel: persistent workgroups of pile waves + store waves.
// For plans whose every row is one plain range with uniform power-of-two bins of one
// wave chunk (C4 peaks, C5 per-base, TSS/TES windows: rcp_plan decides, `P.lean`), the
// row work is the fused pass only, so the kernel drops the general paths and splits the
// workgroup by role:
//   waves 0..7  (pile)  pile rows into their LDS difference arrays and stage bin sums;
//                       they never store to global memory
//   waves 8..11 (store) copy a finished round of the stage into registers and write it
//                       as R column-major fp64; they never wait for a global load, except
//                       store wave 0 fetching the next work item (below)
// gfx9 has one in-order vmcnt for loads and stores, so a wave that stores and then waits
// for a read also waits for its stores to be acknowledged.  With the roles split, the
// epilogue's writes of round rd drain while the pile waves already stream round rd + 1.
// Two LDS-only barriers per round: (A) stage full, (B) stage copied out.
//
// Work items are (row tile of kRows rows, column chunk).  Workgroups are persistent (two
// per CU) and take items from a per-XCD counter: workgroup b serves XCD b % 8 and only
// tiles t = xcd (mod 8), so the column chunks of one tile (which stream the same reads)
// share that XCD's L2.  While the pile waves work on item k, store wave 0 claims item
// k + 1 and decodes its 64 row records into the second metadata buffer, and the pile waves
// prefetch its first reads during item k's last row: no workgroup start-up latency.
// ---------------------------------------------------------------------------------
// Not adopted (same-box A/B, DESIGN_HISTORY.md, round 4): 2 or 6 store waves, 10 pile waves, a third batch
// of reads in flight per row (neutral), 8-read batches for start-only streams.
constexpr int kLPWaves = 8;       // pile waves per lean workgroup (<= 16 rows of a round)
constexpr int kLStoreWaves = 4;
constexpr int kLWpe = 6;          // waves per SIMD asked of the lean kernel
constexpr int kLBatchUni = 4;     // reads per lane per batch of a start-only (uniform-width) lean plan
constexpr int kLBlock = 64 * (kLPWaves + kLStoreWaves);
constexpr int kLQuads = 64 * kLStoreWaves / kTile;  // column quads per store pass
constexpr int kLMaxPass = 8;                        // stage_cap <= 4 * kLQuads * kLMaxPass
static_assert(kRows == 64 && kRounds >= 2, "store wave 0 decodes one row per lane");

// Row metadata of the lean kernel (64 B): w0 = flag | fast << 2 | rev << 3 | log2(bin) << 4
// | (heavy slot + 1) << 9; the read -> chunk position offset `k` folds orientation and origin.
struct LeanMeta {
    int32_t w0, P0, npos, kend;
    int32_t k, gps, gpe, bs;   // bs: bin width (general-bins mode)
    uint32_t lo[3], hi[3];
    int32_t lay, pad2;         // lay: R-RNG layout (-1: none)
};
static_assert(sizeof(LeanMeta) == 64, "LeanMeta is four b128 words");

__device__ __forceinline__ LeanMeta lean_pack(const RowMeta& m) {
    LeanMeta q;
    const int lbs = m.bs > 0 ? 31 - __clz(m.bs) : 0;
    q.w0 = m.flag | (m.fast << 2) | (m.rev << 3) | (lbs << 4) | ((m.heavy + 1) << 9);
    q.P0 = m.P0;
    q.npos = m.npos;
    q.kend = m.kend;
    q.k = m.rev ? m.off + m.shi - m.P0 : m.off - m.slo - m.P0;
    q.gps = m.gps;
    q.gpe = m.gpe;
    q.bs = m.bs;
    for (int s = 0; s < 3; ++s) {
        q.lo[s] = m.lo[s];
        q.hi[s] = m.hi[s];
    }
    q.lay = m.lay;
    q.pad2 = 0;
    return q;
}

struct LeanRow {  // wave-uniform view (SGPRs)
    int32_t flag, fast, rev, lbs, heavy, P0, npos, kend, k, gps, gpe, bs, lay;
    uint32_t lo[3], hi[3];
};

__device__ __forceinline__ LeanRow lean_row(const LeanMeta& src) {
    const int32_t* s = reinterpret_cast<const int32_t*>(&src);
    int32_t v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = q == 15 ? 0 : __builtin_amdgcn_readfirstlane(s[q]);
    LeanRow m;
    m.flag = v[0] & 3;
    m.fast = (v[0] >> 2) & 1;
    m.rev = (v[0] >> 3) & 1;
    m.lbs = (v[0] >> 4) & 31;
    m.heavy = (v[0] >> 9) - 1;
    m.P0 = v[1]; m.npos = v[2]; m.kend = v[3]; m.k = v[4]; m.gps = v[5]; m.gpe = v[6];
    m.bs = v[7]; m.lay = v[14];
    for (int q = 0; q < 3; ++q) {
        m.lo[q] = (uint32_t)v[8 + q];
        m.hi[q] = (uint32_t)v[11 + q];
    }
    return m;
}

__device__ __forceinline__ uint32_t lean_candidates(const LeanRow& m) {
    return (m.hi[0] - m.lo[0]) + (m.hi[1] - m.lo[1]) + (m.hi[2] - m.lo[2]);
}

__device__ __forceinline__ uint32_t lean_index(const LeanRow& m, uint32_t q) {
    if (m.hi[1] == m.lo[1] && m.hi[2] == m.lo[2]) return m.lo[0] + q;
    const uint32_t c0 = m.hi[0] - m.lo[0];
    const uint32_t c1 = m.hi[1] - m.lo[1];
    return q < c0 ? m.lo[0] + q : (q < c0 + c1 ? m.lo[1] + (q - c0) : m.lo[2] + (q - c0 - c1));
}

template <bool REV>
__device__ __forceinline__ void lean_add(const LeanRow& m, int2 rd, int32_t* diff, int sh) {
    if (rd.y < m.gps || rd.x > m.gpe) return;
    const int32_t x0 = max(rd.x, m.gps);
    const int32_t x1 = min(rd.y, m.gpe);
    const int32_t a = REV ? m.k - x1 : x0 + m.k;
    const int32_t b = REV ? m.k - x0 + 1 : x1 + m.k + 1;
    atomicAdd(&diff[lp(a, sh)], 1);
    atomicAdd(&diff[lp(b, sh)], -1);
}

// Dense rows (at least one candidate read per position, e.g. C5's per-base DNase rows): the
// 64 reads of a wave are consecutive in start order and pile onto a few dozen positions, so
// plain LDS atomics serialise on equal addresses (C5: 1.7e8 bank-conflict cycles, 10x C4's).
// Equal positions of neighbouring lanes are merged into one add per run (run_add); all lanes
// of the wave take part (`act` false for lanes past the row's candidates).
template <bool REV>
__device__ __forceinline__ void lean_add_runs(const LeanRow& m, int2 rd, bool act, int32_t* diff, int sh) {
    act = act && !(rd.y < m.gps || rd.x > m.gpe);
    const int32_t x0 = max(rd.x, m.gps);
    const int32_t x1 = min(rd.y, m.gpe);
    const int32_t a = REV ? m.k - x1 : x0 + m.k;
    const int32_t b = REV ? m.k - x0 + 1 : x1 + m.k + 1;
    run_add(diff, lp(a, sh), act, 1);
    run_add(diff, lp(b, sh), act, -1);
}

// lean_add_runs for reads of one width w (the start-only stream): a read covers window
// positions [u, u + w] with u = s + k (forward) or k - s - w (reversed), so its two keys are
// functions of u alone -- one run detection over u serves both atomics (clipped to the
// chunk's window [lo_w, hi_w]); equal u gives equal keys, as the pair path's runs would.
template <bool REV>
__device__ __forceinline__ void lean_add_runs_uni(const LeanRow& m, int32_t s, int32_t w, int32_t lo_w, int32_t hi_w,
                                                  bool act, int32_t* diff, int sh) {
    const int lane = threadIdx.x & 63;
    const int32_t u = REV ? m.k - s - w : s + m.k;
    act = act && u <= hi_w && u + w >= lo_w;
    const int32_t key = act ? u : INT32_MIN;  // never a window position
    const int32_t prev = __builtin_amdgcn_update_dpp(INT32_MIN + 1, key, 0x138, 0xf, 0xf, false);  // wave_shr:1
    const bool head = lane == 0 || key != prev;
    const uint64_t heads = __ballot(head);
    const uint64_t above = lane == 63 ? 0ull : heads & (~0ull << (lane + 1));
    const int len = (above ? __builtin_ctzll(above) : 64) - lane;
    if (head && act) {
        atomicAdd(&diff[lp(max(u, lo_w), sh)], len);
        atomicSub(&diff[lp(min(u + w, hi_w) + 1, sh)], len);
    }
}

// (tile, chunk) of an item code, its part and first bin
struct LeanItem {
    int tile, cidx, p;
    int32_t k0;
};

__device__ __forceinline__ LeanItem lean_item(const RcpPlanDev& P, int code) {
    LeanItem it;
    it.tile = code / P.n_chunks_total;
    it.cidx = code - it.tile * P.n_chunks_total;
    int c = it.cidx, p = 0;
    while (p < P.n_parts - 1 && c >= P.part[p].n_chunks) {
        c -= P.part[p].n_chunks;
        ++p;
    }
    it.p = p;
    it.k0 = c * P.part[p].chunk_bins;
    return it;
}

// MAXPER: positions per lane of the widest chunk (16: <= 1023 positions, 8: <= 511).
// GEN (plan lean == 2): general bins -- any uniform width or R-RNG layouts (splitVector's
// enlarged bins), multi-range rows (exon lists).  Pile waves then stage bin numerators from a
// cumulative scan (bin-edge differences, as the general kernel) plus a per-row bitmask of the
// enlarged bins, and store waves divide by the bin width.
constexpr int kLMaxPassGen = 4;  // general-bins mode: <= 4 * kLQuads * 4 = 256 bins per chunk
template <int MAXPER, bool GEN, int LR, bool UNI>
__global__ void __launch_bounds__(kLBlock) __attribute__((amdgpu_waves_per_eu(kLWpe)))
rcp_pileup_lean_kernel(RcpPlanDev P, double* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int T = kTile;
    // LR rounds of T rows per item (kIRows rows); the metadata buffers keep kRows slots
    constexpr int kIRows = LR * kTile;
    static_assert(LR >= 2 && LR <= kRounds, "the next item's metadata is published a round before it is read");
    // UNI (plan st != null): reads of one width -- the candidate streams are their starts alone
    // (4 B per read instead of the (start, end) pair: half the pile's read traffic); the end
    // is formed when the read is added, so the prefetched loads stay in flight until then
    static_assert(!(UNI && GEN), "uniform-width reads: single-range mode only");
    using RdT = typename std::conditional<UNI, int32_t, int2>::type;
    // reads per lane per batch
    constexpr int BL = UNI ? kLBatchUni : 4;
    constexpr uint32_t BQ = 64u * BL;  // reads per batch
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    const int RS = stage_stride(P.stage_cap);
    uint32_t* stage = reinterpret_cast<uint32_t*>(smem) + kLPWaves * P.wave_words;
    uint32_t* emask = stage + T * RS;  // GEN: [row][16] enlarged-bin bits of the round
    LeanMeta* lmeta = reinterpret_cast<LeanMeta*>(emask + (GEN ? T * 16 : 0));  // [2][kRows]
    int32_t* item = reinterpret_cast<int32_t*>(lmeta + 2 * kRows);  // [2]: item code or -1
    const int xcd = blockIdx.x & 7;
    const int n_tiles = (P.n_rows + kIRows - 1) / kIRows;
    auto n_items_of = [&](int x) { return (uint32_t)((n_tiles - x + 7) / 8) * (uint32_t)P.n_chunks_total; };

    // store wave 0: claim the next item of this XCD, decode its rows into buffer buf; once
    // this XCD's items are gone, take the other XCDs' remaining ones (tail balance)
    auto claim = [&](int buf) {
        uint32_t j = 0;
        int xs = xcd;
        int code = -1;
        if (P.lpt) {
            // heaviest first: one counter over the class lists, highest class first
            if (lane == 0) j = atomicAdd(&P.status[8], 1u);
            j = __builtin_amdgcn_readfirstlane(j);
            for (int c = RCP_LPT_CLASSES - 1; c >= 0; --c) {
                const uint32_t n = min(__builtin_amdgcn_readfirstlane(P.status[RCP_LPT_STATUS + c]),
                                       (uint32_t)P.lpt_cap);
                if (j < n) {
                    code = __builtin_amdgcn_readfirstlane(P.item_order[c * P.lpt_cap + j]);
                    break;
                }
                j -= n;
            }
        } else {
            if (lane == 0) j = atomicAdd(&P.status[8 + xcd], 1u);
            j = __builtin_amdgcn_readfirstlane(j);
            for (int k = 1; k < 8 && j >= n_items_of(xs); ++k) {
                xs = (xcd + k) & 7;
                if (lane == 0) j = atomicAdd(&P.status[8 + xs], 1u);
                j = __builtin_amdgcn_readfirstlane(j);
            }
            if (j < n_items_of(xs)) {
                const int tl = (int)(j / P.n_chunks_total);
                code = (tl * 8 + xs) * P.n_chunks_total + (int)(j - (uint32_t)tl * P.n_chunks_total);
            }
        }
        if (code >= 0) {
            const LeanItem it = lean_item(P, code);
            if (LR == 2 && P.fold) {
                // fold plans (per-base shards): the item's 32 rows searched here, two lanes a row --
                // while the pile waves work on the current item, as a decode would be
                const int i = lane >> 1;
                const RowMeta m = fold_row_pair(P, P.part[it.p], it.k0, it.cidx, it.tile * kIRows + i);
                if ((lane & 1) == 0) lmeta[buf * kRows + i] = lean_pack(m);
            } else if (lane < kIRows) {
                lmeta[buf * kRows + lane] =
                    lean_pack(decode_row<false, false>(P, P.part[it.p], it.k0, it.cidx, it.tile * kIRows + lane));
            }
        }
        if (lane == 0) item[buf] = code;
        // nothing of the claim stays in flight: later register writes of this wave never
        // wait on its loads (only its stores remain outstanding, and nothing waits on them)
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
    };
    if (wave == kLPWaves) claim(0);
    // a fold plan launches no heavy kernel: zero the status set the next execution uses here
    if (P.fold && blockIdx.x == 0 && tid < RCP_STATUS_WORDS) P.status_prev[tid] = 0u;
    if (tid == 0) {
        item[1] = -1;  // (always written by a claim before it is read; defined anyway)
        item[2] = 0;   // the pile waves' row counter (RCP_LEAN_DYN)
    }
    lds_barrier();

    if (wave < kLPWaves) {
        // ================= pile waves
        int32_t* diff = reinterpret_cast<int32_t*>(smem) + wave * P.wave_words;
        [[maybe_unused]] auto row_of = [&](int step) { return (step / kRowsPerWave) * T + (step % kRowsPerWave) * kLPWaves + wave; };
        auto rd_load = [&](uint32_t idx) -> RdT {
            if constexpr (UNI) return P.st[idx];
            else return P.se[idx];
        };
        auto rd_pair = [&](RdT v) -> int2 {
            if constexpr (UNI) return make_int2(v, v + P.st_w);
            else return v;
        };
        auto prefetch = [&](const LeanMeta& mm, RdT* dst) {
            const LeanRow m = lean_row(mm);
            const uint32_t n = (m.flag == 0 && m.fast) ? lean_candidates(m) : 0;
            if (n) {
#pragma unroll
                for (int u = 0; u < BL; ++u) {
                    const uint32_t q = lane + 64 * u;
                    dst[u] = rd_load(lean_index(m, q < n ? q : n - 1));
                }
            }
        };
        int clean_sh = -1;  // the difference array is all zero for this lane geometry
        int buf = 0;
        int code = item[0];
        // one row: `cur` holds its first reads; the next row's (possibly the next item's
        // first row) go to `nxt`
        // pile row i of the item (tile row), its first reads in `cur`; bin sums -> stage
        auto pile_row = [&](const LeanItem& it, int i, RdT (&cur)[BL]) __attribute__((always_inline)) {
            const LeanRow m = lean_row(lmeta[buf * kRows + i]);
            if (m.flag != 0) return;
            if (!GEN && !m.fast && m.heavy < 0) {  // the plan promised single-range rows
                if (lane == 0) atomicOr(P.status, RCP_STATUS_INTERP);
                return;
            }
            const int32_t npos = m.npos;
            const int need = (npos + 1 + 63) >> 6;
            const int sh = need <= 4 ? 2 : 32 - __clz(need - 1);
            if (clean_sh != sh) {
                int4* d4 = reinterpret_cast<int4*>(diff);
                for (int q = lane; q < ((1 << sh) + 4) * 16; q += 64) d4[q] = make_int4(0, 0, 0, 0);
            }
            lds_order();
            if (m.heavy >= 0) {
                // skewed row: difference array piled up by rcp_heavy_pileup_kernel
                const int32_t* g = P.heavy_gdiff + (size_t)m.heavy * P.heavy_stride;
                int32_t carry = 0;
                for (int q = lane; q < m.P0; q += 64) carry += g[q];
                carry = wave_sum(carry);
                for (int q = lane; q <= npos; q += 64) diff[lp(q, sh)] = g[m.P0 + q] + (q == 0 ? carry : 0);
            } else if (GEN && !m.fast) {
                // several ranges (exon list): the wave streams the row's (segment, stream) pairs
                pileup_row_wave(P, it.tile * kIRows + i, m.P0, npos, diff, sh);
            } else {
                const uint32_t n = lean_candidates(m);
                // batches of 64 BL reads, two in flight: `cur` (prefetched with the previous row)
                // and the next
                auto load_batch = [&](uint32_t q0, RdT (&dst)[BL]) {
                    if (q0 < n) {
#pragma unroll
                        for (int u = 0; u < BL; ++u) {
                            const uint32_t q = q0 + lane + 64 * u;
                            dst[u] = rd_load(lean_index(m, q < n ? q : n - 1));
                        }
                    }
                };
                // dense rows (more reads than positions): run-merged adds
                const bool dense = n >= (uint32_t)npos;  // wave-uniform
                auto add_batch = [&](uint32_t q0, const RdT (&src)[BL]) {
                    if constexpr (UNI) {
                        if (dense) {  // start-only: one run detection for both atomics
                            const int32_t w = P.st_w;
                            const int32_t lo_w = m.rev ? m.k - m.gpe : m.gps + m.k;
                            const int32_t hi_w = m.rev ? m.k - m.gps : m.gpe + m.k;
                            if (m.rev) {
#pragma unroll
                                for (int u = 0; u < BL; ++u)
                                    lean_add_runs_uni<true>(m, src[u], w, lo_w, hi_w, q0 + lane + 64u * u < n, diff, sh);
                            } else {
#pragma unroll
                                for (int u = 0; u < BL; ++u)
                                    lean_add_runs_uni<false>(m, src[u], w, lo_w, hi_w, q0 + lane + 64u * u < n, diff, sh);
                            }
                            return;
                        }
                    }
                    if (dense) {
                        if (m.rev) {
#pragma unroll
                            for (int u = 0; u < BL; ++u) lean_add_runs<true>(m, rd_pair(src[u]), q0 + lane + 64u * u < n, diff, sh);
                        } else {
#pragma unroll
                            for (int u = 0; u < BL; ++u) lean_add_runs<false>(m, rd_pair(src[u]), q0 + lane + 64u * u < n, diff, sh);
                        }
                    } else if (m.rev) {
#pragma unroll
                        for (int u = 0; u < BL; ++u)
                            if (q0 + lane + 64u * u < n) lean_add<true>(m, rd_pair(src[u]), diff, sh);
                    } else {
#pragma unroll
                        for (int u = 0; u < BL; ++u)
                            if (q0 + lane + 64u * u < n) lean_add<false>(m, rd_pair(src[u]), diff, sh);
                    }
                };
                for (uint32_t q0 = 0; q0 < n; q0 += BQ) {
                    RdT nx[BL];
                    load_batch(q0 + BQ, nx);
                    add_batch(q0, cur);
#pragma unroll
                    for (int u = 0; u < BL; ++u) cur[u] = nx[u];
                }
            }
            lds_order();
            uint32_t* srow = stage + (i & (T - 1)) * RS;
            const int per = 1 << sh;
            if (!GEN || (m.lay < 0 && m.bs > 0 && (m.bs & (m.bs - 1)) == 0 && m.bs <= per)) {
                if (sh == 2) scan_bins_fast<4>(diff, m.lbs, srow, m.kend - it.k0);
                else if (MAXPER == 8 || sh == 3) scan_bins_fast<8>(diff, m.lbs, srow, m.kend - it.k0);
                else scan_bins_fast<MAXPER>(diff, m.lbs, srow, m.kend - it.k0);
                clean_sh = sh;
                if (GEN && lane < 16) emask[(i & (T - 1)) * 16 + lane] = 0u;
            } else {
                // cumulative depth, then bin k = cum[end - 1] - cum[start - 1] (uint32: a bin sum
                // that fits 32 bits comes out exact); enlarged bins (width bs + 1) flagged in emask
                scan_wave<true>(diff, per);
                lds_order();
                const uint32_t* cum = reinterpret_cast<const uint32_t*>(diff);
                const int32_t e0 = bin_edge(m.bs, m.lay, P.lay_cnt, it.k0);
                for (int32_t k0l = 0; k0l < 4 * kLQuads * kLMaxPassGen; k0l += 64) {
                    const int32_t k = it.k0 + k0l + lane;
                    bool enl = false;
                    if (k < m.kend) {
                        const int32_t a = bin_edge(m.bs, m.lay, P.lay_cnt, k) - e0;
                        const int32_t b = bin_edge(m.bs, m.lay, P.lay_cnt, k + 1) - e0;
                        srow[k - it.k0] = cum[lp(b - 1, sh)] - (a > 0 ? cum[lp(a - 1, sh)] : 0u);
                        enl = b - a > m.bs;
                    }
                    const uint64_t bits = __ballot(enl);
                    if (lane < 2) emask[(i & (T - 1)) * 16 + (k0l >> 5) + lane] = (uint32_t)(bits >> (32 * lane));
                }
                clean_sh = -1;  // the array now holds cumulative depth
            }
            lds_order();
        };
        RdT bufA[BL], bufB[BL];
        // Rows are dealt dynamically: a wave takes the workgroup's next row number g from an
        // LDS counter (rows 64 q .. 64 q + 63 = the q-th item of this workgroup, 16 per round)
        // when it starts its current row, and prefetches g's first reads.  A round ends when
        // its 16 rows are taken and piled, so a wave that drew a long row takes fewer of them
        // (a static 2 rows per wave waited at barrier A for the round's slowest pair).  A wave
        // holds at most one row ahead: the next round's, or the next item's round 0, whose
        // metadata store wave 0 published rounds ago.
        static_assert(kLPWaves <= kTile, "pending rows of one round fit the next round");
        uint32_t* ctr = reinterpret_cast<uint32_t*>(item + 2);
        auto take = [&]() -> uint32_t {
            uint32_t v = 0;
            if (lane == 0) v = atomicAdd(ctr, 1u);
            return __builtin_amdgcn_readfirstlane(v);
        };
        auto fetch = [&](uint32_t rel, RdT (&dst)[BL]) {  // rel: row number relative to this item
            if (rel < (uint32_t)kIRows) {
                prefetch(lmeta[buf * kRows + rel], dst);
            } else {
                const int nc = item[buf ^ 1];
                if (nc >= 0) prefetch(lmeta[(buf ^ 1) * kRows + (rel - kIRows)], dst);
            }
        };
        uint32_t base = 0;       // first row number of the current item
        uint32_t g = take();     // this wave's pending row
        bool in_a = true;        // its first reads sit in bufA (else bufB)
        if (code >= 0) fetch(g, bufA);
        while (code >= 0) {
            const LeanItem it = lean_item(P, code);
            for (int rd = 0; rd < LR; ++rd) {
                const uint32_t lim = base + (uint32_t)(T * (rd + 1));
                while (g < lim) {
                    const uint32_t gn = take();
                    if (in_a) {
                        fetch(gn - base, bufB);
                        pile_row(it, (int)(g - base), bufA);
                    } else {
                        fetch(gn - base, bufA);
                        pile_row(it, (int)(g - base), bufB);
                    }
                    in_a = !in_a;
                    g = gn;
                }
                lds_barrier();  // A: the round's stage rows are complete
                lds_barrier();  // B: the store waves hold them in registers
            }
            base += kIRows;
            buf ^= 1;
            code = item[buf];
        }
    } else {
        // ================= store waves: thread (row ii, column quad qd)
        const int st = tid - 64 * kLPWaves;
        const int ii = st & (T - 1);
        const int qd = st / T;
        const size_t R = (size_t)P.out_ld;  // column stride of the output (>= n_rows)
        const double sc = P.scale;
        const int npass = (P.stage_cap + 4 * kLQuads - 1) / (4 * kLQuads);
        constexpr int kPass = GEN ? kLMaxPassGen : kLMaxPass;
        int buf = 0;
        int code = item[0];
        while (code >= 0) {
            const LeanItem it = lean_item(P, code);
            const int32_t col0 = P.part[it.p].col_off + it.k0 + 4 * qd;
            for (int rd = 0; rd < LR; ++rd) {
                // two rounds per item: the next item is claimed before the first round's barrier A
                // (pile waves prefetch its first rows during the second round; every wave read
                // the buffer it overwrites before the previous item's last barrier B)
                if (LR == 2 && rd == 0 && wave == kLPWaves) claim(buf ^ 1);
                lds_barrier();  // A
                const int rb = rd * T + ii;
                const int r = it.tile * kIRows + rb;
                const LeanMeta& mr = lmeta[buf * kRows + rb];
                const int32_t w0 = mr.w0, kend = mr.kend;
                const int32_t bsr = GEN ? mr.bs : 1;  // (all metadata reads before barrier B)
                const int32_t flag = w0 & 3;
                const bool live = r < P.n_rows && flag != 2;
                // the round's stage -> registers (uniform pass count; the reads past a row's
                // kend stay inside LDS and are never stored)
                uint4 v[kPass];
                const uint32_t* st0 = stage + ii * RS + 4 * qd;
#pragma unroll
                for (int j = 0; j < kPass; ++j)
                    v[j] = j < npass ? *reinterpret_cast<const uint4*>(st0 + 4 * kLQuads * j) : make_uint4(0u, 0u, 0u, 0u);
                // GEN: 4 enlarged-bin bits per pass (bins 4 qd + 64 j .. + 3), packed
                uint32_t enl = 0;
                if (GEN) {
#pragma unroll
                    for (int j = 0; j < kPass; ++j)
                        if (j < npass) enl |= ((emask[ii * 16 + 2 * j + (qd >> 3)] >> ((4 * qd) & 31)) & 15u) << (4 * j);
                }
                lds_barrier();  // B: the stage is free for the next round
                // opaque after the barrier: keeps the conversions (2 VGPRs per value) below it
#pragma unroll
                for (int j = 0; j < kPass; ++j)
                    if (j < npass) asm volatile("" : "+v"(v[j].x), "+v"(v[j].y), "+v"(v[j].z), "+v"(v[j].w));
                if (live) {
                    // power-of-two bin width: multiplying by its reciprocal is exact; a NULL row
                    // (flag 1) scales its (unwritten) stage words by 0.0 -> zeros
                    const double rdd = 1.0 / (double)(1 << ((w0 >> 4) & 31));
                    const double scf = flag == 0 ? sc : 0.0;
                    const int32_t nk = kend - (it.k0 + 4 * qd);  // columns left from this thread's first quad
                    double* o = out + (size_t)col0 * R + (size_t)r;
#pragma unroll
                    for (int j = 0; j < kPass; ++j) {
                        constexpr int kStep = 4 * kLQuads;
                        if (j >= npass || kStep * j >= nk) break;
                        double* oj = o + (size_t)(kStep * j) * R;
                        double x[4];
                        if (GEN) {
                            // mean of a bin = numerator * scale / width (profile.R via splitVector;
                            // the general kernel's flush, rcp_div_rn); a NULL row writes zeros
                            const uint32_t q4[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
                            const double d0 = (double)bsr, d1 = (double)(bsr + 1);
                            const double r0 = 1.0 / d0, r1 = 1.0 / d1;
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const bool e = (enl >> (4 * j + u)) & 1;
                                x[u] = flag == 0 ? rcp_div_rn((double)q4[u] * sc, e ? d1 : d0, e ? r1 : r0) : 0.0;
                            }
                        } else {
                            x[0] = ((double)v[j].x * scf) * rdd;
                            x[1] = ((double)v[j].y * scf) * rdd;
                            x[2] = ((double)v[j].z * scf) * rdd;
                            x[3] = ((double)v[j].w * scf) * rdd;
                        }
                        if (kStep * j + 3 < nk) {
#pragma unroll
                            for (int u = 0; u < 4; ++u) out_store(x[u], oj + u * R);
                        } else {
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                if (kStep * j + u < nk) out_store(x[u], oj + u * R);
                        }
                    }
                }
                // the next item: claimed and decoded after round 0's stores were issued (its
                // loads wait for them, with a whole round of pile work to hide that); read
                // by the pile waves from round 2 on, after this wave has passed barrier A(1)
                if (LR > 2 && rd == 0 && wave == kLPWaves) claim(buf ^ 1);
            }
            buf ^= 1;
            code = item[buf];
        }
    }
    // the last workgroup out resets the item counters for the next launch
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const uint32_t done = atomicAdd(&P.status[16], 1u);
        if (done == gridDim.x - 1) {
            for (int x = 0; x < 8; ++x) atomicExch(&P.status[8 + x], 0u);
            atomicExch(&P.status[16], 0u);
        }
    }
}

// =================================================================================
// bin-difference pileup (P.lean == 4): mean profiles whose rows are single ranges cut into
// uniform bins (every row's slice L = n bs positions: no splitVector layout, no interpolation)
// of at least kBDMinWidth positions, at most kBDMaxBins bins.  A read adds to BINS, not to
// positions: its covered row positions [u, v] (clipped) give bins ku = u / bs and kv = v / bs
// the partial overlaps bs (ku + 1) - u and v - bs kv + 1 (or v - u + 1 when ku == kv), and the
// bins strictly between take bs each through a difference array F (+1 at ku + 1, -1 at kv):
// numerator[k] = D[k] + bs * prefix(F)[k], the exact integer sum the position pileup gives
// (R/util.R:74-84 with dif = 0, R/profile.R:159-208).  Per row the work is O(n bins) instead
// of O(L positions) -- C2's 200 bins of 20 bp instead of 4000 positions in four column chunks
// -- and a whole row is one wave's pass (no column chunks, no per-chunk read ranges).
// Workgroups of kBDWaves waves own 16-row tiles (one 128-B line of every output column);
// each wave piles its rows into its own D / F arrays and stages their numerators; the
// workgroup then writes the tile column-major.
// =================================================================================
constexpr int kBDWaves = 8;  // waves per 16-row tile, two rows each, located in one chain of searches:
                             // four 8-wave workgroups fit a CU (one 16-wave one did: 106 SGPRs), so
                             // C2's 625 tiles are one generation -- pass 0.033 -> 0.027 ms (16 / 8 / 4
                             // waves: 0.033 / 0.027 / 0.032, profiles/r06/c2/ab_waves.log)
static_assert(kTile % kBDWaves == 0, "a tile's rows are split evenly over the waves");
constexpr int kBDMaxBins = 512;
constexpr int kBDMinWidth = 4;
extern "C" int rcp_bins_max_bins(void) { return kBDMaxBins; }
extern "C" int rcp_bins_min_width(void) { return kBDMinWidth; }

__host__ __device__ __forceinline__ int bd_stage_stride(int n) { return ((n + 3) >> 2 << 2) + 4; }
__host__ __device__ __forceinline__ int bd_wave_words(int n) { return 2 * (((n + 2) + 63) & ~63); }

static size_t bins_lds_bytes(int n, int waves) {
    return 4 * ((size_t)kTile * bd_stage_stride(n) + (size_t)waves * bd_wave_words(n) + 2 * kTile);
}
extern "C" size_t rcp_pileup_bins_lds_bytes(const RcpPlanDev* P) { return bins_lds_bytes(P->part[0].n_bins, 16); }

template <bool UNI, int WAVES>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(4)))
rcp_pileup_bins_kernel(RcpPlanDev P, double* __restrict__ out, int64_t* __restrict__ binsum) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    using RdT = typename std::conditional<UNI, int32_t, int2>::type;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const RcpPart part = P.part[0];
    const int32_t n = part.n_bins;
    const int RS = bd_stage_stride(n);
    const int WW = bd_wave_words(n);
    uint32_t* stage = reinterpret_cast<uint32_t*>(smem);                 // [16][RS] numerators
    int32_t* D = reinterpret_cast<int32_t*>(stage + kTile * RS) + wave * WW;  // partial overlaps
    int32_t* F = D + WW / 2;                                              // full-bin differences
    int32_t* rbs = reinterpret_cast<int32_t*>(stage + kTile * RS) + WAVES * WW;  // [16] bs, 0 NULL, -1 none
    // tiles of one XCD's workgroups are consecutive (round-robin dispatch over 8 XCDs):
    // neighbouring regions share reads in that L2
    const int nt = (P.n_rows + kTile - 1) / kTile;
    const int per_x = (nt + 7) / 8;
    const int tile = (blockIdx.x & 7) * per_x + (blockIdx.x >> 3);
    if (tile >= nt) return;
    const int row0 = tile * kTile;
    // a folded plan launches no heavy kernel: zero the status set the next execution uses here
    // (nothing in this execution reads it)
    if (P.fold && blockIdx.x == 0 && tid < RCP_STATUS_WORDS) P.status_prev[tid] = 0u;
    for (int q = lane; q < WW; q += 64) D[q] = 0;  // D and F
    auto rd_load = [&](uint32_t idx) -> RdT {
        if constexpr (UNI) return P.st[idx];
        else return P.se[idx];
    };
    auto rd_pair = [&](RdT v) -> int2 {
        if constexpr (UNI) return make_int2(v, v + P.st_w);
        else return v;
    };
    // a row's wave-uniform description, from the locate kernel's record
    struct Row {
        int32_t flag, heavy, bs, k, gps, gpe, rev, head, L;
        uint32_t lo[3], hi[3];
    };
    // P.fold: the locate kernel's work for row r done here -- the single range's candidate reads
    // per strand stream (lanes 2s / 2s + 1: lower / upper bound of stream s, bucket directory +
    // bisection as rcp_locate_kernel) and the NULL rules (no hit; the range past seqlength, or
    // past the hits' last end when seqlength is NA: R/coverage.R:189-225); writes the row's
    // validity and returns the record rcp_locate_kernel would have left
    auto locate_row = [&](int r) -> RcpRowRec {
        RcpRowInfo ri;
        {
            const uint4* src = reinterpret_cast<const uint4*>(P.row_info + r);
            uint4 w[sizeof(RcpRowInfo) / 16];
#pragma unroll
            for (int q = 0; q < (int)(sizeof(RcpRowInfo) / 16); ++q) w[q] = src[q];
            int32_t v[sizeof(RcpRowInfo) / 4];
            __builtin_memcpy(v, w, sizeof v);
#pragma unroll
            for (int q = 0; q < (int)(sizeof(RcpRowInfo) / 4); ++q) v[q] = __builtin_amdgcn_readfirstlane(v[q]);
            __builtin_memcpy(&ri, v, sizeof ri);
        }
        RcpRowRec R{};
        R.row_len = ri.row_len;
        R.heavy = -1;
        const RcpSeg sg = ri.seg0;
        const bool ok = !ri.stat && ri.chrom >= 0 && ri.chrom < P.n_chrom && ri.j1 == ri.j0 + 1 && sg.query_ok;
        bool valid = false;
        if (ok) {  // wave-uniform
            const int ns = P.merged ? 1 : 3;
            uint32_t res = 0;
            if (lane < 2 * ns && ((sg.streams >> (lane >> 1)) & 1)) {
                const int st = lane >> 1;
                int64_t d0[1] = {ri.d0};
                int32_t nb[1] = {ri.nb};
                if (!P.merged) {
                    d0[0] = P.dir_off[ri.chrom * 3 + st];
                    nb[0] = (int32_t)(P.dir_off[ri.chrom * 3 + st + 1] - d0[0]) - 1;
                }
                const int32_t v[1] = {(lane & 1) ? sg.hi : sg.lo};
                const int dst[1] = {(lane & 1) ? -1 : -2};
                uint32_t out1[1];
                dir_bound_multi<1>(P, d0, nb, v, dst, 1, out1);
                res = out1[0];
            }
            bool hit = false;
            int32_t maxend = INT32_MIN;
#pragma unroll
            for (int st = 0; st < 3; ++st) {
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)res, 2 * st);
                const uint32_t hi = max(lo, (uint32_t)__builtin_amdgcn_readlane((int)res, 2 * st + 1));
                R.lo[st] = R.hi[st] = 0;
                if (st < ns && ((sg.streams >> st) & 1) && lo < hi) {
                    R.lo[st] = lo;
                    R.hi[st] = hi;
                    hit = true;
                    if (ri.seqlen < 0) maxend = max(maxend, P.pmax[hi - 1]);  // only NA seqlengths need it
                }
            }
            valid = hit && (ri.seqlen >= 0 ? (int64_t)sg.hi <= ri.seqlen : sg.hi <= maxend);
        }
        if (lane == 0) {
            P.valid[r] = valid ? 1 : 0;
            if (P.valid_out) P.valid_out[r] = valid ? 1 : 0;
        }
        R.flags = valid ? (RCP_REC_VALID | RCP_REC_FAST) : 0;
        R.off = sg.off;
        R.slo = sg.lo;
        R.shi = sg.hi;
        R.rev = sg.rev;
        return R;
    };
    // a row's description from its record (the locate kernel's, or the folded searches')
    auto describe = [&](const RcpRowRec& R) -> Row {
        Row m{};
        if (!(R.flags & RCP_REC_VALID)) {
            m.flag = 0;  // NULL row -> zeros (profile.R:191-197)
            return m;
        }
        rcp_part_slice(part, R.row_len, &m.head, &m.L);
        m.bs = m.L / n;
        if (m.L < n || m.L != m.bs * n || !(R.flags & RCP_REC_FAST)) {
            // the plan promised uniform bins of single-range rows
            if (lane == 0) atomicOr(P.status, RCP_STATUS_INTERP);
            m.flag = 0;
            return m;
        }
        m.flag = 1;
        m.heavy = R.heavy;
        m.rev = R.rev;
        const int32_t len = R.shi - R.slo + 1;
        const int32_t a = max(m.head, R.off), b = min(m.head + m.L, R.off + len);
        m.gps = 0;
        m.gpe = -1;
        if (a < b) {
            if (!R.rev) {
                m.gps = R.slo + (a - R.off);
                m.gpe = R.slo + (b - 1 - R.off);
            } else {
                m.gpe = R.shi - (a - R.off);
                m.gps = R.shi - (b - 1 - R.off);
            }
        }
        // row position (slice-relative) of genomic g: g + k forward, k - g reversed
        m.k = R.rev ? R.off + R.shi - m.head : R.off - R.slo - m.head;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            m.lo[s] = R.lo[s];
            m.hi[s] = a < b ? R.hi[s] : R.lo[s];
        }
        return m;
    };
    auto row_of = [&](int r) -> Row {
        Row m{};
        m.flag = -1;
        if (r >= P.n_rows) return m;
        RcpRowRec R;
        if (P.fold) {
            R = locate_row(r);
        } else {
            RcpRowRec rec;
            const uint4* src = reinterpret_cast<const uint4*>(P.rec + r);
            uint4* dst = reinterpret_cast<uint4*>(&rec);
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[q] = src[q];
            int32_t v[16];
            __builtin_memcpy(v, &rec, sizeof v);
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = __builtin_amdgcn_readfirstlane(v[q]);
            __builtin_memcpy(&R, v, sizeof R);
        }
        return describe(R);
    };
    // P.fold with several rows a wave (kMine > 1): the locate work of all of them in ONE chain of
    // round trips -- their row records loaded together, lane l bisecting bound l % 2ns of row
    // l / 2ns (2ns lanes a row: lower / upper bound per strand stream), their NULL rules after --
    // instead of one chain per row
    constexpr int kMine = kTile / WAVES;
    auto locate_rows = [&](const int (&rr)[kMine], Row (&rows)[kMine]) {
        RcpRowInfo ri[kMine];
        {
            uint4 w[kMine][sizeof(RcpRowInfo) / 16];
#pragma unroll
            for (int j = 0; j < kMine; ++j) {
                const uint4* src = reinterpret_cast<const uint4*>(P.row_info + min(rr[j], P.n_rows - 1));
#pragma unroll
                for (int q = 0; q < (int)(sizeof(RcpRowInfo) / 16); ++q) w[j][q] = src[q];
            }
#pragma unroll
            for (int j = 0; j < kMine; ++j) {
                int32_t v[sizeof(RcpRowInfo) / 4];
                __builtin_memcpy(v, w[j], sizeof v);
#pragma unroll
                for (int q = 0; q < (int)(sizeof(RcpRowInfo) / 4); ++q) v[q] = __builtin_amdgcn_readfirstlane(v[q]);
                __builtin_memcpy(&ri[j], v, sizeof(RcpRowInfo));
            }
        }
        const int ns = P.merged ? 1 : 3, per = 2 * ns;
        const int jl = lane / per, e = lane - jl * per, st = e >> 1;
        bool ok[kMine];
        int64_t d0[1] = {0};
        int32_t nb[1] = {0};
        int32_t v[1] = {0};
        const int dst[1] = {(e & 1) ? -1 : -2};
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < kMine; ++j) {
            const RcpSeg& sg = ri[j].seg0;
            ok[j] = rr[j] < P.n_rows && !ri[j].stat && ri[j].chrom >= 0 && ri[j].chrom < P.n_chrom &&
                    ri[j].j1 == ri[j].j0 + 1 && sg.query_ok;
            if (jl == j && ok[j] && ((sg.streams >> st) & 1)) {
                cnt = 1;
                v[0] = (e & 1) ? sg.hi : sg.lo;
                d0[0] = ri[j].d0;
                nb[0] = ri[j].nb;
                if (!P.merged) {
                    d0[0] = P.dir_off[ri[j].chrom * 3 + st];
                    nb[0] = (int32_t)(P.dir_off[ri[j].chrom * 3 + st + 1] - d0[0]) - 1;
                }
            }
        }
        uint32_t res[1];
        dir_bound_multi<1>(P, d0, nb, v, dst, cnt, res);
        RcpRowRec R[kMine];
        int32_t maxend[kMine];
        bool hit[kMine];
#pragma unroll
        for (int j = 0; j < kMine; ++j) {
            const RcpSeg& sg = ri[j].seg0;
            R[j] = RcpRowRec{};
            R[j].row_len = ri[j].row_len;
            R[j].heavy = -1;
            hit[j] = false;
            maxend[j] = INT32_MIN;
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)res[0], j * per + 2 * s);
                const uint32_t hi = max(lo, (uint32_t)__builtin_amdgcn_readlane((int)res[0], j * per + 2 * s + 1));
                R[j].lo[s] = R[j].hi[s] = 0;
                if (ok[j] && s < ns && ((sg.streams >> s) & 1) && lo < hi) {
                    R[j].lo[s] = lo;
                    R[j].hi[s] = hi;
                    hit[j] = true;
                    if (ri[j].seqlen < 0) maxend[j] = max(maxend[j], P.pmax[hi - 1]);  // only NA seqlengths need it
                }
            }
        }
#pragma unroll
        for (int j = 0; j < kMine; ++j) {
            const RcpSeg& sg = ri[j].seg0;
            const bool valid = ok[j] && hit[j] && (ri[j].seqlen >= 0 ? (int64_t)sg.hi <= ri[j].seqlen : sg.hi <= maxend[j]);
            if (lane == 0 && rr[j] < P.n_rows) {
                P.valid[rr[j]] = valid ? 1 : 0;
                if (P.valid_out) P.valid_out[rr[j]] = valid ? 1 : 0;
            }
            R[j].flags = valid ? (RCP_REC_VALID | RCP_REC_FAST) : 0;
            R[j].off = sg.off;
            R[j].slo = sg.lo;
            R[j].shi = sg.hi;
            R[j].rev = sg.rev;
            if (rr[j] < P.n_rows) {
                rows[j] = describe(R[j]);
            } else {
                rows[j] = Row{};
                rows[j].flag = -1;
            }
        }
    };
    auto n_cand = [&](const Row& m) -> uint32_t {
        return (m.hi[0] - m.lo[0]) + (m.hi[1] - m.lo[1]) + (m.hi[2] - m.lo[2]);
    };
    auto cand_index = [&](const Row& m, uint32_t q) -> uint32_t {
        if (m.hi[1] == m.lo[1] && m.hi[2] == m.lo[2]) return m.lo[0] + q;
        const uint32_t c0 = m.hi[0] - m.lo[0], c1 = m.hi[1] - m.lo[1];
        return q < c0 ? m.lo[0] + q : (q < c0 + c1 ? m.lo[1] + (q - c0) : m.lo[2] + (q - c0 - c1));
    };
    // candidate slot u of a lane in a batch: 4 lane + u (ps_slot), so the 64 adds of one
    // instruction are 4 reads apart: start-sorted reads of one lane group spread over 4x the bins,
    // fewer same-address LDS atomics (a 180-bp read spans 9 bins of 20 bp)
    auto load_batch = [&](const Row& m, uint32_t nc, uint32_t q0, RdT (&dst)[4]) {
        if (m.flag == 1 && m.heavy < 0 && q0 < nc) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t q = q0 + ps_slot(lane, u);
                dst[u] = rd_load(cand_index(m, q < nc ? q : nc - 1));
            }
        }
    };
    // bin of slice position x (0 <= x < L): x / bs through a float reciprocal, corrected
    auto bin_of = [&](int32_t x, int32_t bs, float rb) -> int32_t {
        int32_t kb = (int32_t)((float)x * rb);
        kb -= kb * bs > x ? 1 : 0;
        kb += (kb + 1) * bs <= x ? 1 : 0;
        return kb;
    };
    auto add_read = [&](const Row& m, int2 rd, float rb) {
        if (rd.y < m.gps || rd.x > m.gpe) return;
        const int32_t x0 = max(rd.x, m.gps), x1 = min(rd.y, m.gpe);
        const int32_t u = m.rev ? m.k - x1 : x0 + m.k;
        const int32_t v = m.rev ? m.k - x0 : x1 + m.k;
        const int32_t ku = bin_of(u, m.bs, rb), kv = bin_of(v, m.bs, rb);
        if (ku == kv) {
            atomicAdd(&D[ku], v - u + 1);
        } else {
            atomicAdd(&D[ku], m.bs * (ku + 1) - u);
            atomicAdd(&D[kv], v - m.bs * kv + 1);
            if (kv > ku + 1) {
                atomicAdd(&F[ku + 1], 1);
                atomicAdd(&F[kv], -1);
            }
        }
    };
    // my rows of the tile: wave, wave + WAVES, ...
    RdT buf[kMine][4];
    auto pile = [&](const Row& m, int i, RdT (&c)[4]) {
        if (lane == 0) rbs[i] = m.flag == 1 ? m.bs : (m.flag == 0 ? 0 : -1);
        if (m.flag != 1) return;
        const float rb = 1.0f / (float)m.bs;
        if (m.heavy >= 0) {
            // skewed row: its position difference array was piled up by
            // rcp_heavy_pileup_kernel; depth by a wave scan, summed into D per position
            const int32_t* g = P.heavy_gdiff + (size_t)m.heavy * P.heavy_stride;
            int32_t carry = 0;
            for (int q = lane; q < m.head; q += 64) carry += g[q];
            carry = wave_sum(carry);
            for (int32_t b0 = 0; b0 < m.L; b0 += 64) {
                const int32_t x = b0 + lane;
                const int32_t gv = x < m.L ? g[m.head + x] : 0;
                const int32_t incl = (int32_t)wave_inclusive_scan((uint32_t)gv);
                const int32_t depth = carry + incl;
                carry += __builtin_amdgcn_readlane(incl, 63);
                if (x < m.L && depth) atomicAdd(&D[bin_of(x, m.bs, rb)], depth);
            }
        } else {
            const uint32_t nc = n_cand(m);
            for (uint32_t q0 = 0; q0 < nc; q0 += 256) {
                RdT nb[4];
                load_batch(m, nc, q0 + 256, nb);
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (q0 + ps_slot(lane, u) < nc) add_read(m, rd_pair(c[u]), rb);
#pragma unroll
                for (int u = 0; u < 4; ++u) c[u] = nb[u];
            }
        }
        lds_order();
        // numerators: D[k] + bs * prefix(F)[k], 64 bins per step (lane t: bin 64 j + t; one
        // wave scan per step): consecutive lanes, consecutive words -- no bank conflicts
        uint32_t* srow = stage + i * RS;
        int32_t carry = 0;
        for (int32_t k0 = 0; k0 < n; k0 += 64) {
            const int k = k0 + lane;
            const int32_t f = k < n ? F[k] : 0;
            const int32_t run = carry + (int32_t)wave_inclusive_scan((uint32_t)f);
            carry = __builtin_amdgcn_readlane(run, 63);
            if (k < n) {
                srow[k] = (uint32_t)(D[k] + m.bs * run);
                D[k] = 0;
                F[k] = 0;
            }
        }
        lds_order();
    };
    if (P.fold && kMine > 1) {
        // all my rows' searches in one chain, then all their first batches in flight together
        int rr[kMine];
#pragma unroll
        for (int j = 0; j < kMine; ++j) rr[j] = row0 + wave + WAVES * j;
        Row rows[kMine];
        locate_rows(rr, rows);
#pragma unroll
        for (int j = 0; j < kMine; ++j) load_batch(rows[j], n_cand(rows[j]), 0, buf[j]);
#pragma unroll
        for (int j = 0; j < kMine; ++j) pile(rows[j], wave + WAVES * j, buf[j]);
    } else {
        Row cur = row_of(row0 + wave);
        load_batch(cur, n_cand(cur), 0, buf[0]);
#pragma unroll
        for (int j = 0; j < kMine; ++j) {
            const int i = wave + WAVES * j;  // tile row
            RdT (&c)[4] = buf[j & 1 ? (kMine > 1 ? 1 : 0) : 0];
            RdT (&nx)[4] = buf[j & 1 ? 0 : (kMine > 1 ? 1 : 0)];
            Row nxt{};
            nxt.flag = -1;
            if (j + 1 < kMine) {
                nxt = row_of(row0 + i + WAVES);
                load_batch(nxt, n_cand(nxt), 0, nx);
            }
            pile(cur, i, c);
            cur = nxt;
        }
    }
    lds_barrier();
    // ---- the tile's 16 rows, column-major: thread (row ii, column group cg) stores columns cg,
    // cg + kCG, ...; the 16 lanes of a column write its 128-B line of the tile
    constexpr int kCG = 64 * WAVES / kTile;
    const int ii = tid & (kTile - 1), cg = tid >> 4;
    const int r = row0 + ii;
    if (r >= P.n_rows) return;
    const int32_t bs = rbs[ii];
    if (bs < 0) return;
    const size_t R = (size_t)P.out_ld;
    const double sc = P.scale;
    const double dd = (double)max(bs, 1), rdd = 1.0 / dd;
    const bool pow2 = bs > 0 && (bs & (bs - 1)) == 0;
    const uint32_t* srow = stage + ii * RS;
    for (int32_t k = cg; k < n; k += kCG) {
        const size_t o = (size_t)(part.col_off + k) * R + (size_t)r;
        const uint32_t num = bs > 0 ? srow[k] : 0u;
        const double x = bs == 0 ? 0.0 : (pow2 ? ((double)num * sc) * rdd : rcp_div_rn((double)num * sc, dd, rdd));
        out_store(x, out + o);
        if (binsum) binsum[o] = (int64_t)num;
    }
}

template <int WAVES>
static hipError_t launch_pileup_bins_w(const RcpPlanDev* P, double* out, int64_t* binsum, hipStream_t stream) {
    const int nt = (P->n_rows + kTile - 1) / kTile;
    const unsigned grid = (unsigned)(((nt + 7) / 8) * 8);
    const size_t lds = bins_lds_bytes(P->part[0].n_bins, WAVES);
    if (P->st) {
        hipLaunchKernelGGL((rcp_pileup_bins_kernel<true, WAVES>), dim3(grid), dim3(64 * WAVES), lds, stream, *P, out, binsum);
    } else {
        hipLaunchKernelGGL((rcp_pileup_bins_kernel<false, WAVES>), dim3(grid), dim3(64 * WAVES), lds, stream, *P, out, binsum);
    }
    return hipGetLastError();
}

static hipError_t launch_pileup_bins(const RcpPlanDev* P, double* out, int64_t* binsum, hipStream_t stream) {
    // (RCP_BD_WAVES=16: diagnostics A/B against round 5's one-row-a-wave tiles)
    static const bool w16 = std::getenv("RCP_BD_WAVES") && std::atoi(std::getenv("RCP_BD_WAVES")) == 16;
    if (w16) return launch_pileup_bins_w<16>(P, out, binsum, stream);
    return launch_pileup_bins_w<kBDWaves>(P, out, binsum, stream);
}

// =================================================================================
// interpolation rows (length(x) < n): spline "fmm", neighborhood, "inear" no-op
// (rcp_splitvector.h, included above the row-wave kernel, which runs them too)
// =================================================================================

// Block-level window: depth of row r over row positions [w0, w0 + wn) into diff[0 .. wn)
// (reads piled by all 256 threads, or copied from a heavy row's global difference array).
__device__ void block_window_depth(const RcpPlanDev& P, int r, int32_t w0, int32_t wn, int32_t* diff,
                                   uint32_t* scratch) {
    const int per = (wn + 1 + kBlock - 1) / kBlock;
    for (int q = threadIdx.x; q < per * kBlock; q += kBlock) diff[q] = 0;
    __syncthreads();
    const int32_t slot = P.heavy_threshold > 0 ? P.rec[r].heavy : -1;  // (folded plans: no record)
    if (slot >= 0) {
        const int32_t* g = P.heavy_gdiff + (size_t)slot * P.heavy_stride;
        if (threadIdx.x == 0) {
            int32_t carry = 0;
            for (int q = 0; q < w0; ++q) carry += g[q];
            diff[0] = carry;
        }
        __syncthreads();
        for (int q = threadIdx.x; q <= wn; q += kBlock) diff[q] += g[w0 + q];
    } else {
        // the row's (segment, stream) pairs as one stream of candidate batches, dealt to the
        // block's waves (pileup_row walked the pairs one after the other: one round trip each,
        // a dozen per interpolated C3 gene)
        pileup_row_wave(P, r, w0, wn, diff, 30, (int)(threadIdx.x >> 6), kWaves);
    }
    __syncthreads();
    scan_block_depth(diff, per, scratch);
    __syncthreads();
}

// Rows the pileup kernel leaves out: interpolation (length(x) < n bins, modes 1-3) and
// median bins wider than a wave chunk (mode 4, bins taken in groups that fit the window).
__global__ void __launch_bounds__(kBlock) rcp_interp_kernel(RcpPlanDev P, double* __restrict__ out) {
    // these blocks run beside the persistent pileup workgroups (a side stream forked after
    // locate) and are latency-bound (the spline's serial chains): their waves issue first on a
    // shared SIMD, so the pass does not wait for them after the memory-bound pileup has ended
    __builtin_amdgcn_s_setprio(2);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int32_t* diff = reinterpret_cast<int32_t*>(smem);
    const int diff_words = (P.interp_cap + 8 + 1023) & ~1023;
    uint32_t* scratch = reinterpret_cast<uint32_t*>(smem) + diff_words;
    // (no static __shared__: the dynamic region may take all 160 KB)
    int32_t& group_end = reinterpret_cast<int32_t*>(scratch)[2 * kWaves];
    const int e = blockIdx.x;
    const int r = P.interp_row[e];
    const RcpPart part = P.part[P.interp_part[e]];
    const int n = part.n_bins;
    const size_t R = (size_t)P.out_ld;  // column stride of the output (>= n_rows)
    if (!P.valid[r]) {
        for (int k = threadIdx.x; k < n; k += kBlock) out[(size_t)(part.col_off + k) * R + r] = 0.0;
        return;
    }
    int32_t head, L;
    rcp_part_slice(part, P.row_len[r], &head, &L);
    const int mode = P.interp_mode[e];
    if (mode == 4) {  // median over bins wider than a wave chunk
        const int32_t bs = L / n;
        const int32_t lay = P.interp_pos[e];  // layout of dif = L - bs * n, or -1
        for (int32_t k = 0; k < n;) {
            if (threadIdx.x == 0) {
                int32_t ke = k + 1;
                const int32_t ek = bin_edge(bs, lay, P.lay_cnt, k);
                while (ke < n && bin_edge(bs, lay, P.lay_cnt, ke + 1) - ek <= P.interp_cap) ++ke;
                group_end = ke;
            }
            __syncthreads();
            const int32_t ke = group_end;
            const int32_t e0 = bin_edge(bs, lay, P.lay_cnt, k);
            const int32_t wn = bin_edge(bs, lay, P.lay_cnt, ke) - e0;
            if (wn > P.interp_cap) {
                if (threadIdx.x == 0) atomicOr(P.status, RCP_STATUS_INTERP);
                return;
            }
            block_window_depth(P, r, head + e0, wn, diff, scratch);
            for (int32_t kk = k + threadIdx.x; kk < ke; kk += kBlock) {
                const int32_t a = bin_edge(bs, lay, P.lay_cnt, kk) - e0;
                const int32_t b = bin_edge(bs, lay, P.lay_cnt, kk + 1) - e0;
                int32_t vmin = INT32_MAX, vmax = INT32_MIN;
                for (int32_t q = a; q < b; ++q) {
                    vmin = min(vmin, diff[q]);
                    vmax = max(vmax, diff[q]);
                }
                const int32_t mm = b - a, h = (mm + 1) >> 1;
                const uint32_t x1 = (vmin == vmax) ? (uint32_t)vmin : kth_smallest(diff, a, b, h, vmin, vmax, 30);
                uint32_t x2 = x1;
                if (!(mm & 1)) x2 = (vmin == vmax) ? (uint32_t)vmin : kth_smallest(diff, a, b, h + 1, vmin, vmax, 30);
                out[(size_t)(part.col_off + kk) * R + r] = ((double)(x1 + x2) * P.scale) / 2.0;
            }
            __syncthreads();
            k = ke;
        }
        return;
    }
    if (L > P.interp_cap) {
        if (threadIdx.x == 0) atomicOr(P.status, RCP_STATUS_INTERP);
        return;
    }
    // the spline / fill works on LDS copies (global scratch only for huge rows)
    double* x = P.interp_lds >= 0 ? reinterpret_cast<double*>(smem + P.interp_lds)
                                  : P.interp_scratch + (size_t)e * P.interp_stride;
    if (P.interp_stage) {
        // piled by the row-wave kernel into the row's stage words (rcp_pileup_rows_kernel)
        const uint32_t* src = P.rm32 + (size_t)r * (size_t)P.n_cols + part.col_off;
        for (int i = threadIdx.x; i < L; i += kBlock) x[i] = (double)src[i] * P.scale;
    } else {
        block_window_depth(P, r, head, L, diff, scratch);
        for (int i = threadIdx.x; i < L; i += kBlock) x[i] = (double)diff[i] * P.scale;
    }
    __syncthreads();
    interp_finish(mode, L, n, x, mode == 3 ? P.nb_pos + P.interp_pos[e] : nullptr, P.spl_tb,
                  out + (size_t)part.col_off * R + r, R);
}

// =================================================================================
// host-callable launchers
// =================================================================================
namespace {
// hipFuncSetAttribute acts on the function object of the CURRENT device, so the 160 KB
// dynamic-LDS opt-in is made once per (kernel, device); host threads driving different GPUs
// (rcp_profile_multi) may launch concurrently.
hipError_t allow_big_lds_fn(const void* fn) {
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(mu);
    if (done.count({fn, dev})) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess) done.insert({fn, dev});
    return e;
}
template <class K>
hipError_t allow_big_lds(K kernel) {
    return allow_big_lds_fn(reinterpret_cast<const void*>(kernel));
}
}  // namespace

extern "C" hipError_t rcp_launch_locate(const RcpPlanDev* P, hipStream_t stream) {
    if (P->n_rows == 0) return hipSuccess;
    const int64_t grid = (4 * (int64_t)P->n_rows + kBlock - 1) / kBlock;  // four lanes per row
    // a single-range row's searches: its two bounds + the interior chunk edges, dealt to the quad;
    // more than 16 (over 8 column chunks) take lockstep rounds of 8 (one chain, not two)
    // single-range plans of <= 3 column chunks (<= 8 searches a row): 2 per lane
    const int searches = 2 + (P->crange ? 2 * (P->n_chunks_total - 1) : 0);  // a single-range row's
    if (P->crange && 2 * P->n_chunks_total > 4 * 4)
        hipLaunchKernelGGL((rcp_locate_kernel<8, 4>), dim3((unsigned)grid), dim3(kBlock), 0, stream, *P);
    // (occupancy pays on big tables -- C4: 100 -> 91 us -- and plans without chunk searches,
    // C2: 33 -> 30 us; the 25k-row C4 shard runs in one generation anyway and measured 4 us
    // slower: profiles/r04/r4j/ab.log new vs ks2off)
    else if (searches <= 2 * 4 && !P->multi_rows && (!P->crange || P->n_rows >= 50000))
        hipLaunchKernelGGL((rcp_locate_kernel<2, 2>), dim3((unsigned)grid), dim3(kBlock), 0, stream, *P);
    else
        hipLaunchKernelGGL((rcp_locate_kernel<4, 4>), dim3((unsigned)grid), dim3(kBlock), 0, stream, *P);
    return hipGetLastError();
}

// Always launched after locate (one block without a heavy path): it also zeroes status_prev.
extern "C" hipError_t rcp_launch_heavy(const RcpPlanDev* P, int grid, hipStream_t stream) {
    if (P->n_rows == 0 || P->heavy_threshold <= 0) {
        hipLaunchKernelGGL(rcp_heavy_pileup_kernel, dim3(1), dim3(kBlock), 64, stream, *P);
        return hipGetLastError();
    }
    {
        const hipError_t e = allow_big_lds(rcp_heavy_pileup_kernel);
        if (e != hipSuccess) return e;
    }
    // difference array of one row + the slots' slice offsets
    const size_t lds = 4 * (16 + (size_t)P->heavy_max_len + 1 + 64) + 4 * ((size_t)P->heavy_cap + 1);
    hipLaunchKernelGGL(rcp_heavy_pileup_kernel, dim3(grid), dim3(kBlock), lds, stream, *P);
    return hipGetLastError();
}

extern "C" size_t rcp_pileup_lds_bytes(const RcpPlanDev* P, int csr) {
    const size_t stage_words = csr ? 0 : (size_t)kTile * stage_stride(P->stage_cap);
    return 4 * ((size_t)kPWaves * (P->wave_words + 8) + stage_words + (size_t)kRows * kMetaWords + 8);
}

extern "C" int rcp_tile_rows(void) { return kRows; }  // lean items of kRounds rounds (lean_rounds 0)

// rows per round of the general pileup kernel and its maximum rounds per workgroup
extern "C" void rcp_tile_geometry(int* tile, int* rounds_max) {
    *tile = kTile;
    *rounds_max = kRounds;
}

// bins per column chunk the lean kernel's store waves can hold
extern "C" int rcp_lean_max_bins(void) { return 4 * kLQuads * kLMaxPass; }
extern "C" int rcp_lean_gen_max_bins(void) { return 4 * kLQuads * kLMaxPassGen; }

extern "C" size_t rcp_pileup_lean_lds_bytes(const RcpPlanDev* P);

template <int MAXPER, bool GEN, int LR, bool UNI>
static hipError_t launch_pileup_lean_t(const RcpPlanDev* P, double* out, hipStream_t s) {
    {
        const hipError_t e = allow_big_lds(rcp_pileup_lean_kernel<MAXPER, GEN, LR, UNI>);
        if (e != hipSuccess) return e;
    }
    // [pile waves' difference arrays | one stage | row metadata x 2 | item codes x 2]
    const size_t lds = rcp_pileup_lean_lds_bytes(P);
    // persistent: as many workgroups as fit at once (LDS: two per CU), a multiple of 8
    // (workgroup b serves XCD b % 8), never more than there are work items
    const int cus = std::max(1, P->n_cus);  // of the plan's device (rcp_plan_create)
    const int per_cu = std::max(1, std::min(2, (int)((160 * 1024) / lds)));
    const int tiles = (P->n_rows + LR * kTile - 1) / (LR * kTile);
    const int64_t items = (int64_t)((tiles + 7) / 8) * 8 * P->n_chunks_total;
    // (P->grid_fill < 8: room for another sample's locate / heavy launches, rcp_plan_opts.concurrent)
    const int fill = P->grid_fill > 0 && P->grid_fill <= 8 ? P->grid_fill : 8;
    const int64_t grid = std::min<int64_t>(std::max<int64_t>(((int64_t)per_cu * cus * fill / 8 + 7) / 8 * 8, 8), items);
    hipLaunchKernelGGL((rcp_pileup_lean_kernel<MAXPER, GEN, LR, UNI>), dim3((unsigned)grid), dim3(kLBlock), lds, s, *P,
                       out);
    return hipGetLastError();
}

template <int MAXPER, bool GEN>
static hipError_t launch_pileup_lean_r(const RcpPlanDev* P, double* out, hipStream_t s) {
    if constexpr (!GEN) {
        if (P->st)
            return P->lean_rounds == 2 ? launch_pileup_lean_t<MAXPER, false, 2, true>(P, out, s)
                                       : launch_pileup_lean_t<MAXPER, false, kRounds, true>(P, out, s);
    }
    return P->lean_rounds == 2 ? launch_pileup_lean_t<MAXPER, GEN, 2, false>(P, out, s)
                               : launch_pileup_lean_t<MAXPER, GEN, kRounds, false>(P, out, s);
}

extern "C" size_t rcp_pileup_lean_lds_bytes(const RcpPlanDev* P) {
    // [pile waves' difference arrays | stage | (general bins) enlarged-bin bits | row metadata
    //  x 2 | item codes x 2]
    return 4 * ((size_t)kLPWaves * P->wave_words + (size_t)kTile * stage_stride(P->stage_cap) +
                (P->lean == 2 ? (size_t)kTile * 16 : 0)) +
           2 * (size_t)kRows * sizeof(LeanMeta) + 16;
}

static hipError_t launch_pileup_lean(const RcpPlanDev* P, double* out, hipStream_t s) {
    if (P->lean == 2)
        return P->chunk_cap <= 511 ? launch_pileup_lean_r<8, true>(P, out, s) : launch_pileup_lean_r<16, true>(P, out, s);
    return P->chunk_cap <= 511 ? launch_pileup_lean_r<8, false>(P, out, s) : launch_pileup_lean_r<16, false>(P, out, s);
}

template <bool MEDIAN, bool CSR, bool UNI>
static hipError_t launch_pileup_u(const RcpPlanDev* P, double* out, int64_t* binsum, size_t lds, hipStream_t s) {
    {
        const hipError_t e = allow_big_lds(rcp_pileup_kernel<MEDIAN, CSR, UNI>);
        if (e != hipSuccess) return e;
    }
    const int rows_wg = kTile * P->rounds;
    const int tiles = (P->n_rows + rows_wg - 1) / rows_wg;
    const int64_t grid = (int64_t)((tiles + 7) / 8) * 8 * P->n_chunks_total;
    hipLaunchKernelGGL((rcp_pileup_kernel<MEDIAN, CSR, UNI>), dim3((unsigned)grid), dim3(kPBlock), lds, s, *P, out,
                       binsum);
    return hipGetLastError();
}

template <bool MEDIAN, bool CSR>
static hipError_t launch_pileup_t(const RcpPlanDev* P, double* out, int64_t* binsum, size_t lds, hipStream_t s) {
    return P->st ? launch_pileup_u<MEDIAN, CSR, true>(P, out, binsum, lds, s)
                 : launch_pileup_u<MEDIAN, CSR, false>(P, out, binsum, lds, s);
}

// dynamic LDS of the row-wave launch: the staged kernel's windows (kRWGWaves waves; the
// binsum launch takes the 4-wave unstaged kernel)
extern "C" size_t rcp_pileup_rows_lds_bytes(const RcpPlanDev*) { return rows_lds_bytes(kRWGWaves, RowWin<kRWSh>::words); }

static hipError_t launch_pileup_rows(const RcpPlanDev* P, double* out, int64_t* binsum, hipStream_t s) {
    // persistent: a multiple of 8 workgroups (workgroup b serves XCD b % 8), never more
    // workgroups than tiles
    const int cus = std::max(1, P->n_cus);
    const int64_t tiles = ((int64_t)P->n_rows + kTile - 1) / kTile;  // at least a tile per workgroup
    const RcpPlanDev& Q = *P;
    if (binsum || !P->rm32) {
        // four 4-wave workgroups per CU, means stored straight into the output
        const int64_t grid = std::min<int64_t>(((int64_t)4 * cus + 7) / 8 * 8, (tiles + 7) / 8 * 8);
        hipLaunchKernelGGL((rcp_pileup_rows_kernel<0, kRWaves, kRWSh>), dim3((unsigned)grid), dim3(64 * kRWaves),
                           rows_lds_bytes(kRWaves, RowWin<kRWSh>::words), s, Q, out, binsum);
        return hipGetLastError();
    }
    // HBM stage: 16 waves per CU, as kRWGWaves-wave workgroups
    constexpr int kG = kRWGWaves;
    auto k = rcp_pileup_rows_kernel<1, kG, kRWSh>;
    const size_t lds = rows_lds_bytes(kG, RowWin<kRWSh>::words);
    if (lds > 64 * 1024) {
        const hipError_t e = allow_big_lds(k);
        if (e != hipSuccess) return e;
    }
    const int fill = P->grid_fill > 0 && P->grid_fill <= 8 ? P->grid_fill : 8;  // rcp_plan_opts.concurrent
    const int64_t grid = std::min<int64_t>(std::max<int64_t>(((int64_t)(16 / kG) * cus * fill / 8 + 7) / 8 * 8, 8),
                                           (tiles + 7) / 8 * 8);
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * kG), lds, s, Q, out, binsum);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_pileup(const RcpPlanDev* P, double* out, int64_t* binsum, int csr,
                                        hipStream_t stream) {
    if (P->n_rows == 0) return hipSuccess;
    if (!csr && P->lean == 3 && P->stat == 0) return launch_pileup_rows(P, out, binsum, stream);
    if (!csr && P->lean == 4 && P->stat == 0) return launch_pileup_bins(P, out, binsum, stream);
    const size_t lds = rcp_pileup_lds_bytes(P, csr);
    if (!csr && (P->lean == 1 || P->lean == 2) && P->stat == 0 && !binsum) return launch_pileup_lean(P, out, stream);
    if (csr) return launch_pileup_t<false, true>(P, out, binsum, lds, stream);
    if (P->stat == 1) return launch_pileup_t<true, false>(P, out, binsum, lds, stream);
    return launch_pileup_t<false, false>(P, out, binsum, lds, stream);
}

// [depth window | block-scan scratch | (when it fits) the row's spline / fill doubles]
static size_t interp_int_bytes(const RcpPlanDev* P) {
    return 4 * ((size_t)((P->interp_cap + 8 + 1023) & ~1023) + 2 * kWaves + 8);
}

static bool interp_in_lds(const RcpPlanDev* P) {
    // (the spline's arrays in global scratch instead, which lets every row's block be resident
    // at once, measured slower alone on C3: 0.128 vs 0.123 ms, profiles/r02h/c3_transpose_interp_ab.log;
    // beside the row-wave pileup the smaller block is what fits, interp_lds_budget)
    const size_t budget = (P->interp_lds_budget > 0 && !P->interp_stage) ? (size_t)P->interp_lds_budget : 160 * 1024;
    return interp_int_bytes(P) + 8 * (size_t)P->interp_stride + 16 <= budget;
}

extern "C" size_t rcp_interp_lds_bytes(const RcpPlanDev* P) {
    return interp_int_bytes(P) + (interp_in_lds(P) ? 8 * (size_t)P->interp_stride + 16 : 0);
}

extern "C" hipError_t rcp_launch_interp(const RcpPlanDev* P, double* out, hipStream_t stream) {
    if (P->n_interp == 0) return hipSuccess;
    {
        const hipError_t e = allow_big_lds(rcp_interp_kernel);
        if (e != hipSuccess) return e;
    }
    RcpPlanDev Q = *P;
    Q.interp_lds = interp_in_lds(P) ? (int32_t)((interp_int_bytes(P) + 15) / 16 * 16) : -1;
    hipLaunchKernelGGL(rcp_interp_kernel, dim3(P->n_interp), dim3(kBlock), rcp_interp_lds_bytes(P), stream, Q, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// Numerator download (rcp_profile_reads and the other host-matrix paths): a one-part plan's means
// are (q * scale) / bs of a uint32 bin numerator q and the row's bin width bs -- with bs a power
// of two, (q * scale) * (1 / bs) -- so the host can make every double of the matrix from q and bs
// with the same IEEE operations, and PCIe carries 4 bytes a cell instead of 8.  This kernel
// recovers q from each mean and checks that the forward operation gives back the mean's bits;
// rows whose means are not such quotients (interpolated rows, R-RNG layouts: bins of two widths)
// are marked in bad[r] and the caller fetches their doubles apart (rcp_gather_rows_kernel), or
// all doubles when there are many.  div[r] = bs, 0 for a NULL row (its means are +0.0).
constexpr int kPackCols = 8;  // columns per thread
__global__ void __launch_bounds__(kBlock) rcp_pack_kernel(RcpPlanDev P, const double* __restrict__ out,
                                                          uint32_t* __restrict__ q_out, uint32_t* __restrict__ div,
                                                          uint32_t* __restrict__ bad_row) {
    const int r = blockIdx.x * kBlock + threadIdx.x;
    if (r >= P.out_ld) return;
    if (r >= P.n_rows) {  // column padding: zeros (the download packs whole column runs)
        for (int64_t k = (int64_t)blockIdx.y * kPackCols; k < min<int64_t>((int64_t)(blockIdx.y + 1) * kPackCols, P.n_cols); ++k)
            q_out[k * P.out_ld + r] = 0u;
        return;
    }
    const RcpPart& part = P.part[0];
    const int32_t n = part.n_bins;
    uint32_t bs = 0;
    bool bad = false;
    if (P.valid[r]) {
        int32_t head, L;
        rcp_part_slice(part, P.row_len[r], &head, &L);
        if (part.per_base) {
            bs = 1;
            bad = L != n;
        } else {
            bad = L < n || L % n != 0;
            bs = bad ? 0u : (uint32_t)(L / n);
        }
    }
    if (blockIdx.y == 0) div[r] = bs;
    const double sc = P.scale;
    const double dd = (double)max(bs, 1u), rdd = 1.0 / dd;
    const bool pow2 = (bs & (bs - 1)) == 0;
    const size_t ld = (size_t)P.out_ld;
    const int64_t k0 = (int64_t)blockIdx.y * kPackCols;
    uint32_t why = bad ? 4u : 0u;  // (bits: 1 a mean that is no quotient, 2 a NULL row's nonzero, 4 row shape)
    for (int64_t k = k0; k < min<int64_t>(k0 + kPackCols, P.n_cols); ++k) {
        const double v = out[k * ld + r];
        uint32_t q = 0;
        if (bs) {
            const double x = rint(v * dd / sc);
            q = (x >= 0.0 && x <= 4294967295.0) ? (uint32_t)x : 0u;
            const double back = pow2 ? ((double)q * sc) * rdd : rcp_div_rn((double)q * sc, dd, rdd);
            if (__double_as_longlong(back) != __double_as_longlong(v)) why |= 1u;
        } else if (__double_as_longlong(v) != 0) {
            why |= 2u;  // a NULL row's +0.0
        }
        q_out[k * ld + r] = q;
    }
    if (why) atomicOr(bad_row + r, why);
}

// rows[i]'s doubles (column-major, stride ld) into dst[c * n + i]: the rows the numerator download
// could not carry
__global__ void __launch_bounds__(kBlock) rcp_gather_rows_kernel(const double* __restrict__ out, int64_t ld,
                                                                 const int32_t* __restrict__ rows, int32_t n,
                                                                 int64_t n_cols, double* __restrict__ dst) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (int64_t)n * n_cols) return;
    const int64_t c = t / n;
    const int32_t i = (int32_t)(t - c * n);
    dst[t] = out[c * ld + rows[i]];
}

extern "C" hipError_t rcp_launch_gather_rows(const double* out, int64_t ld, const int32_t* rows, int32_t n,
                                             int64_t n_cols, double* dst, hipStream_t stream) {
    const int64_t cells = (int64_t)n * n_cols;
    if (cells == 0) return hipSuccess;
    hipLaunchKernelGGL(rcp_gather_rows_kernel, dim3((unsigned)((cells + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                       out, ld, rows, n, n_cols, dst);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_pack(const RcpPlanDev* P, const double* out, uint32_t* q_out, uint32_t* div,
                                      uint32_t* bad_row, hipStream_t stream) {
    if (P->n_rows == 0 || P->n_cols == 0) return hipSuccess;
    const dim3 grid((unsigned)((P->out_ld + kBlock - 1) / kBlock), (unsigned)((P->n_cols + kPackCols - 1) / kPackCols));
    hipLaunchKernelGGL(rcp_pack_kernel, grid, dim3(kBlock), 0, stream, *P, out, q_out, div, bad_row);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_readset(int64_t n, const int32_t* chrom, const int32_t* start, const int32_t* end,
                                         const int8_t* strand, int32_t n_chrom, int32_t strand_filter, int merge,
                                         uint64_t* keys, int32_t* vals, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const int64_t grid = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(rcp_make_keys_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream, n, chrom, start, end,
                       strand, n_chrom, strand_filter, merge, keys, vals);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_unsorted(int64_t n, const uint64_t* keys, uint32_t* flag, hipStream_t stream) {
    if (n < 2) return hipSuccess;
    hipLaunchKernelGGL(rcp_unsorted_kernel, dim3((unsigned)((n - 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, n,
                       keys, flag);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_width_end(int64_t n, const int32_t* start, int32_t* width_end, uint32_t* overflow,
                                           hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rcp_width_end_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, n,
                       start, width_end, overflow);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_order(int64_t n, const int32_t* chrom, const int32_t* start, uint32_t* flag,
                                       hipStream_t stream) {
    if (n < 2) return hipSuccess;
    hipLaunchKernelGGL(rcp_order_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, n,
                       chrom, start, flag);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_expand_runs(int64_t n, int32_t n_runs, const int64_t* run_start,
                                             const int32_t* run_value, int32_t* out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rcp_expand_runs_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, n,
                       n_runs, run_start, run_value, out);
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

extern "C" hipError_t rcp_launch_stream_maxend(int64_t n_streams, const int64_t* off, const int32_t* pmax,
                                               int32_t* out, hipStream_t stream) {
    if (n_streams == 0) return hipSuccess;
    hipLaunchKernelGGL(rcp_stream_maxend_kernel, dim3((unsigned)((n_streams + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       stream, n_streams, off, pmax, out);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_dirk(int64_t n_entries, const int32_t* dir_lu, const int32_t* pmax, const int2* se,
                                      int32_t* dir_k, hipStream_t stream) {
    if (n_entries == 0) return hipSuccess;
    hipLaunchKernelGGL(rcp_dirk_kernel, dim3((unsigned)((2 * n_entries + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                       n_entries, dir_lu, pmax, se, dir_k);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_dir(int64_t n_entries, int64_t n_streams, const int64_t* dir_off, const int64_t* off,
                                     const int32_t* pmax, const int2* se, int shift, int32_t* dir_l, int32_t* dir_u,
                                     hipStream_t stream) {
    if (n_entries == 0) return hipSuccess;
    hipLaunchKernelGGL(rcp_dir_kernel, dim3((unsigned)((n_entries + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                       n_entries, n_streams, dir_off, off, pmax, se, shift, dir_l, dir_u);
    return hipGetLastError();
}

// =================================================================================
// run-length encoding of CSR coverage (the Rle objects of calcCoverage, S4Vectors)
// =================================================================================
// One wave per row, 256 positions per step (lane: positions base + lane + 64 u, coalesced): a
// run starts at the row's first position or where the value differs from the one before.
// Pass 1 counts each row's runs; an exclusive scan of the counts gives the rows' run offsets;
// pass 2 writes every run's value and length at its final place (run lengths from the next
// run start in the same 64 positions, else carried as the wave's pending run).
constexpr int kRleWaves = 4;

__global__ void __launch_bounds__(64 * kRleWaves) rcp_rle_count_kernel(int32_t n_rows, const int64_t* __restrict__ off,
                                                                     const int32_t* __restrict__ cov,
                                                                     int64_t* __restrict__ count) {
    const int r = blockIdx.x * kRleWaves + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t a = off[r], b = off[r + 1];
    int64_t c = 0;
    for (int64_t base = a; base < b; base += 256) {
        int32_t v[4], pv[4];
        bool in[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = base + lane + 64 * u;
            in[u] = i < b;
            v[u] = in[u] ? cov[i] : 0;
            pv[u] = (in[u] && i > a) ? cov[i - 1] : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = base + lane + 64 * u;
            c += __popcll(__ballot(in[u] && (i == a || v[u] != pv[u])));
        }
    }
    if (lane == 0) count[r] = c;
}

__global__ void __launch_bounds__(64 * kRleWaves) rcp_rle_emit_kernel(int32_t n_rows, const int64_t* __restrict__ off,
                                                                    const int32_t* __restrict__ cov,
                                                                    const int64_t* __restrict__ run_off,
                                                                    int32_t* __restrict__ values,
                                                                    int32_t* __restrict__ lengths,
                                                                    uint32_t* __restrict__ bad) {
    const int r = blockIdx.x * kRleWaves + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t end = run_off[r + 1];  // the row's runs, as the counts sized them
    if (end == run_off[r]) return;        // no runs: an empty or NULL row
    const int64_t a = off[r], b = off[r + 1];
    const uint64_t below = (1ull << lane) - 1;  // lanes < this one
    int64_t k = run_off[r];                      // next run index
    int64_t pend = -1, pstart = 0;               // the last run written, its length still open
    for (int64_t base = a; base < b; base += 256) {
        int32_t v[4], pv[4];
        bool in[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = base + lane + 64 * u;
            in[u] = i < b;
            v[u] = in[u] ? cov[i] : 0;
            pv[u] = (in[u] && i > a) ? cov[i - 1] : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = base + lane + 64 * u;
            const bool f = in[u] && (i == a || v[u] != pv[u]);
            const uint64_t m = __ballot(f);
            if (m == 0) continue;
            const int first = __builtin_ctzll(m);
            const int64_t s0 = base + 64 * u;  // position of lane 0 in this step
            if (pend >= 0 && pend < end && lane == first) lengths[pend] = (int32_t)(i - pstart);
            if (f) {
                const int64_t idx = k + __popcll(m & below);
                if (idx < end) {  // never past the row's runs, whatever the counts said
                    values[idx] = v[u];
                    const uint64_t after = m & ~(below | (1ull << lane));
                    if (after) lengths[idx] = __builtin_ctzll(after) - lane;
                }
            }
            const int last = 63 - __builtin_clzll(m);
            k += __popcll(m);
            pend = k - 1;
            pstart = s0 + last;
        }
    }
    if (pend >= 0 && pend < end && lane == 0) lengths[pend] = (int32_t)(b - pstart);
    if (lane == 0 && k != end) atomicOr(bad, 1u);  // the counting pass and this one disagree
}

// Rle runs from the pileup's run-start lists (P.csr_rs / csr_sub, no dense depth array).
// Plan (a thread per row): a chunk's first start is a run start only at the row's first
// position or where its depth differs from the previous chunk's last depth; per chunk j the
// kept starts cnt[j] (scanned into the run offsets), and info[j] = (skipped first entry, row
// position of the next kept start after the chunk -- the end of its last run --, the chunk's
// dense offset).  NULL rows keep no runs.
__global__ void __launch_bounds__(kBlock) rcp_cov_runs_plan_kernel(int32_t n_rows, const int64_t* __restrict__ off,
                                                                 const int64_t* __restrict__ sub_off,
                                                                 const int2* __restrict__ sub,
                                                                 const int2* __restrict__ rs,
                                                                 const uint8_t* __restrict__ valid, int32_t chunk,
                                                                 int64_t* __restrict__ cnt, int4* __restrict__ info,
                                                                 uint32_t* __restrict__ bad) {
    const int r = blockIdx.x * kBlock + threadIdx.x;
    if (r >= n_rows) return;
    const int64_t j0 = sub_off[r], j1 = sub_off[r + 1];
    const int64_t a = off[r];
    const int32_t L = (int32_t)(off[r + 1] - a);
    if (!valid[r] || L == 0) {
        for (int64_t j = j0; j < j1; ++j) cnt[j] = 0;
        return;
    }
    if ((int64_t)(L + chunk - 1) / chunk != j1 - j0) atomicOr(bad, 1u);
    int32_t prev = 0;
    for (int64_t j = j0; j < j1; ++j) {
        const int2 sb = sub[j];
        const int32_t d0 = (int32_t)(a + (j - j0) * chunk);
        const int32_t len = min(chunk, L - (int32_t)(j - j0) * chunk);
        if (sb.x < 1 || sb.x > len) {  // every chunk records its first position
            atomicOr(bad, 1u);
            cnt[j] = 0;
            info[j] = make_int4(0, 0, d0, 0);
            continue;
        }
        const int skip = (j > j0 && rs[d0].x == prev) ? 1 : 0;
        cnt[j] = sb.x - skip;
        info[j] = make_int4(skip, 0, d0, 0);
        prev = sb.y;
    }
    int32_t next = L;  // row position of the next kept run start
    for (int64_t j = j1 - 1; j >= j0; --j) {
        if (cnt[j] == 0) continue;
        const int4 in = info[j];
        info[j] = make_int4(in.x, next, in.z, 0);
        next = rs[in.z + in.x].y;
    }
}

// run offsets of the rows: the scanned chunk counts at each row's first chunk
__global__ void __launch_bounds__(kBlock) rcp_cov_runs_rowoff_kernel(int32_t n_rows, const int64_t* __restrict__ sub_off,
                                                                   const int64_t* __restrict__ base,
                                                                   int64_t* __restrict__ run_off) {
    const int r = blockIdx.x * kBlock + threadIdx.x;
    if (r <= n_rows) run_off[r] = base[sub_off[r]];
}

// Compaction: a wave per chunk copies its kept starts to their final places as (value, length);
// a run's length reaches the next kept start (the chunk's last run: info.y, possibly in a
// later chunk)
__global__ void __launch_bounds__(kBlock) rcp_cov_runs_emit_kernel(int64_t n_sub, const int64_t* __restrict__ base,
                                                                 const int4* __restrict__ info,
                                                                 const int2* __restrict__ rs,
                                                                 int32_t* __restrict__ values,
                                                                 int32_t* __restrict__ lengths,
                                                                 uint32_t* __restrict__ bad) {
    const int64_t j = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (j >= n_sub) return;
    const int lane = threadIdx.x & 63;
    const int64_t b = base[j];
    const int32_t c = (int32_t)(base[j + 1] - b);
    if (c <= 0) return;
    const int4 in = info[j];
    const int2* src = rs + in.z + in.x;
    bool ok = true;
    for (int32_t e = lane; e < c; e += 64) {
        const int2 x = src[e];
        const int32_t nx = e + 1 < c ? src[e + 1].y : in.y;
        values[b + e] = x.x;
        lengths[b + e] = nx - x.y;
        ok = ok && nx > x.y;
    }
    if (!ok) atomicOr(bad, 1u);
}

extern "C" hipError_t rcp_cov_runs_dev(int32_t n_rows, const int64_t* d_off, const int64_t* d_sub_off, int64_t n_sub,
                                       const int2* d_sub, const int2* d_rs, const uint8_t* d_valid, int32_t chunk,
                                       int64_t* d_cnt, int4* d_info, int64_t* d_base, int64_t* d_run_off, void* temp,
                                       size_t* temp_bytes, int32_t* d_values, int32_t* d_lengths, uint32_t* d_bad,
                                       int pass, hipStream_t stream) {
    // pass 0: temp size of the scan; 1: plan + scan + row offsets (d_cnt[n_sub] must be 0);
    // 2: emit (values / lengths of d_run_off[n_rows] runs)
    if (pass == 0) return hipcub::DeviceScan::ExclusiveSum(nullptr, *temp_bytes, d_cnt, d_base, (int)n_sub + 1, stream);
    if (pass == 1) {
        if (n_rows > 0)
            hipLaunchKernelGGL(rcp_cov_runs_plan_kernel, dim3((unsigned)((n_rows + kBlock - 1) / kBlock)), dim3(kBlock),
                               0, stream, n_rows, d_off, d_sub_off, d_sub, d_rs, d_valid, chunk, d_cnt, d_info, d_bad);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        e = hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, d_cnt, d_base, (int)n_sub + 1, stream);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(rcp_cov_runs_rowoff_kernel, dim3((unsigned)((n_rows + 1 + kBlock - 1) / kBlock)), dim3(kBlock),
                           0, stream, n_rows, d_sub_off, d_base, d_run_off);
        return hipGetLastError();
    }
    if (n_sub > 0)
        hipLaunchKernelGGL(rcp_cov_runs_emit_kernel, dim3((unsigned)((n_sub + kBlock / 64 - 1) / (kBlock / 64))),
                           dim3(kBlock), 0, stream, n_sub, d_base, d_info, d_rs, d_values, d_lengths, d_bad);
    return hipGetLastError();
}

extern "C" hipError_t rcp_rle_encode_dev(int32_t n_rows, const int64_t* d_off, const int32_t* d_cov, int64_t* d_count,
                                         int64_t* d_run_off, void* temp, size_t* temp_bytes, int32_t* d_values,
                                         int32_t* d_lengths, int pass, hipStream_t stream) {
    // pass 0: temp size of the scan; 1: count + scan (d_run_off[n_rows] = total); 2: emit
    // (temp: a zeroed uint32 flag, set when a row's runs differ from its count)
    if (pass == 0)
        return hipcub::DeviceScan::ExclusiveSum(nullptr, *temp_bytes, d_count, d_run_off, (int)n_rows + 1, stream);
    const unsigned grid = (unsigned)((n_rows + kRleWaves - 1) / kRleWaves);
    if (pass == 1) {
        hipError_t e = hipMemsetAsync(d_count + n_rows, 0, 8, stream);
        if (e != hipSuccess) return e;
        if (n_rows > 0)
            hipLaunchKernelGGL(rcp_rle_count_kernel, dim3(grid), dim3(64 * kRleWaves), 0, stream, n_rows, d_off, d_cov,
                               d_count);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, d_count, d_run_off, (int)n_rows + 1, stream);
    }
    if (n_rows > 0)
        hipLaunchKernelGGL(rcp_rle_emit_kernel, dim3(grid), dim3(64 * kRleWaves), 0, stream, n_rows, d_off, d_cov,
                           d_run_off, d_values, d_lengths, static_cast<uint32_t*>(temp));
    return hipGetLastError();
}

// Uniform-width readsets: the range of end - start over the layout's sorted (key, end) pairs
// (mm[0] min, mm[1] max; the caller seeds INT32_MAX / INT32_MIN).  When it is one value the
// ends ascend with the starts inside every stream, so the prefix max of the ends is the end
// itself (no segmented scan), and the starts are kept alone for the pileup kernels.
__global__ void __launch_bounds__(kBlock) rcp_width_range_kernel(int64_t n, const uint64_t* __restrict__ keys,
                                                                const int32_t* __restrict__ vals,
                                                                int32_t* __restrict__ mm) {
    __shared__ int32_t bmin, bmax;
    if (threadIdx.x == 0) {
        bmin = INT32_MAX;
        bmax = INT32_MIN;
    }
    __syncthreads();
    int32_t lo = INT32_MAX, hi = INT32_MIN;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const int32_t start = (int32_t)((uint32_t)keys[i] ^ 0x80000000u);
        const int32_t w = (int32_t)((int64_t)vals[i] - (int64_t)start);  // ends >= start - 1
        lo = min(lo, w);
        hi = max(hi, w);
    }
    atomicMin(&bmin, lo);
    atomicMax(&bmax, hi);
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicMin(&mm[0], bmin);
        atomicMax(&mm[1], bmax);
    }
}

// se -> starts alone (st) and the prefix max of the ends (= the ends, reads of one width)
__global__ void __launch_bounds__(kBlock) rcp_split_uniform_kernel(int64_t n, const int2* __restrict__ se,
                                                                  int32_t* __restrict__ st,
                                                                  int32_t* __restrict__ pmax) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const int2 r = se[i];
        st[i] = r.x;
        pmax[i] = r.y;
    }
}

extern "C" hipError_t rcp_launch_width_range(int64_t n, const uint64_t* keys, const int32_t* vals, int32_t* mm,
                                             hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const int64_t grid = std::min<int64_t>((n + kBlock - 1) / kBlock, 4096);
    hipLaunchKernelGGL(rcp_width_range_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream, n, keys, vals, mm);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_split_uniform(int64_t n, const int2* se, int32_t* st, int32_t* pmax,
                                               hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const int64_t grid = std::min<int64_t>((n + kBlock - 1) / kBlock, 16384);
    hipLaunchKernelGGL(rcp_split_uniform_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream, n, se, st, pmax);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_unpack_pmax(int64_t n, const uint64_t* scan_out, int32_t* pmax, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const int64_t grid = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(rcp_unpack_pmax_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream, n, scan_out, pmax);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// Packed uploads (rcp_stage.cpp stage_h2d_i32 / stage_h2d_strand): the host sends a chunk of
// int32 values as [base int32 x nb][slot int32 x nb][16-bit offsets x n][raw blocks], blocks of
// kPackBlock values -- value = base + offset, or, for a block whose span does not fit 16 bits,
// raw[slot] -- and strand codes four to a byte (3: a code outside 0..2, which drops the read).
// ---------------------------------------------------------------------------------
constexpr int kPackBlock = 1024;
__global__ void __launch_bounds__(kBlock) rcp_unpack_i32_kernel(const char* __restrict__ src, int64_t n, int64_t nb,
                                                                int32_t* __restrict__ dst) {
    const int64_t b = blockIdx.x;
    const int32_t base = reinterpret_cast<const int32_t*>(src)[b];
    const int32_t slot = reinterpret_cast<const int32_t*>(src)[nb + b];
    const uint16_t* off = reinterpret_cast<const uint16_t*>(src + 8 * nb) + b * kPackBlock;
    const int32_t* raw = reinterpret_cast<const int32_t*>(src + 8 * nb + 2 * ((n + 1) & ~int64_t(1)));
    const int64_t i0 = b * kPackBlock;
    for (int j = threadIdx.x; j < kPackBlock && i0 + j < n; j += kBlock)
        dst[i0 + j] = slot < 0 ? (int32_t)((uint32_t)base + off[j]) : raw[(int64_t)slot * kPackBlock + j];
}

__global__ void __launch_bounds__(kBlock) rcp_unpack_strand_kernel(const uint8_t* __restrict__ src, int64_t n,
                                                                   int8_t* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (4 * i >= n) return;
    const uint32_t w = src[i];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        if (4 * i + u >= n) break;
        const int c = (int)((w >> (2 * u)) & 3u);
        dst[4 * i + u] = (int8_t)(c == 3 ? -1 : c);
    }
}

// chromosome codes one byte each (rcp_stage.cpp stage_h2d_codes): 255 -> -1 (the read is dropped)
__global__ void __launch_bounds__(kBlock) rcp_unpack_code8_kernel(const uint8_t* __restrict__ src, int64_t n,
                                                                  int32_t* __restrict__ dst) {
    const int64_t i = 4 * ((int64_t)blockIdx.x * kBlock + threadIdx.x);
    if (i >= n) return;
    if (i + 4 <= n) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(src + i);
        int4 v;
        v.x = (int)(w & 255u);
        v.y = (int)((w >> 8) & 255u);
        v.z = (int)((w >> 16) & 255u);
        v.w = (int)(w >> 24);
        v.x = v.x == 255 ? -1 : v.x;
        v.y = v.y == 255 ? -1 : v.y;
        v.z = v.z == 255 ? -1 : v.z;
        v.w = v.w == 255 ? -1 : v.w;
        if ((reinterpret_cast<uintptr_t>(dst + i) & 15) == 0) {
            *reinterpret_cast<int4*>(dst + i) = v;
        } else {
            dst[i] = v.x; dst[i + 1] = v.y; dst[i + 2] = v.z; dst[i + 3] = v.w;
        }
        return;
    }
    for (int64_t j = i; j < n; ++j) dst[j] = src[j] == 255 ? -1 : (int32_t)src[j];
}

extern "C" hipError_t rcp_launch_unpack_code8(const void* src, int64_t n, int32_t* dst, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int64_t quads = (n + 3) / 4;
    hipLaunchKernelGGL(rcp_unpack_code8_kernel, dim3((unsigned)((quads + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       stream, static_cast<const uint8_t*>(src), n, dst);
    return hipGetLastError();
}

extern "C" int rcp_pack_block(void) { return kPackBlock; }

extern "C" hipError_t rcp_launch_unpack_i32(const void* src, int64_t n, int32_t* dst, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int64_t nb = (n + kPackBlock - 1) / kPackBlock;
    hipLaunchKernelGGL(rcp_unpack_i32_kernel, dim3((unsigned)nb), dim3(kBlock), 0, stream,
                       static_cast<const char*>(src), n, nb, dst);
    return hipGetLastError();
}

extern "C" hipError_t rcp_launch_unpack_strand(const void* src, int64_t n, int8_t* dst, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int64_t words = (n + 3) / 4;
    hipLaunchKernelGGL(rcp_unpack_strand_kernel, dim3((unsigned)((words + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       stream, static_cast<const uint8_t*>(src), n, dst);
    return hipGetLastError();
}

// The packed download of an int32 array (rcp_stage.cpp stage_d2h_i32): blocks of kPackBlock values
// as their minimum + 16-bit offsets ([base x nb][flag x nb][offsets x n]); flag 1: the block's
// values span 2^16 or more and the host copies it from the source itself
__global__ void __launch_bounds__(kBlock) rcp_pack_i32_kernel(const int32_t* __restrict__ src, int64_t n, int64_t nb,
                                                              char* __restrict__ dst) {
    static_assert(kPackBlock == 4 * kBlock, "four values per thread");
    __shared__ int32_t s_lo[kBlock / 64], s_hi[kBlock / 64];
    const int64_t b = blockIdx.x;
    const int64_t i0 = b * kPackBlock;
    const int len = (int)min<int64_t>(kPackBlock, n - i0);
    int32_t v[4];
    int32_t lo = INT32_MAX, hi = INT32_MIN;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int j = threadIdx.x + kBlock * u;
        v[u] = j < len ? src[i0 + j] : 0;
        if (j < len) {
            lo = min(lo, v[u]);
            hi = max(hi, v[u]);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o));
        hi = max(hi, __shfl_xor(hi, o));
    }
    if ((threadIdx.x & 63) == 0) {
        s_lo[threadIdx.x >> 6] = lo;
        s_hi[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        lo = min(lo, s_lo[w]);
        hi = max(hi, s_hi[w]);
    }
    const bool fits = (int64_t)hi - (int64_t)lo <= 65535;
    uint16_t* off = reinterpret_cast<uint16_t*>(dst + 8 * nb) + i0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int j = threadIdx.x + kBlock * u;
        if (j < len) off[j] = (uint16_t)((uint32_t)v[u] - (uint32_t)lo);
    }
    if (threadIdx.x == 0) {
        reinterpret_cast<int32_t*>(dst)[b] = lo;
        reinterpret_cast<int32_t*>(dst)[nb + b] = fits ? 0 : 1;
    }
}

extern "C" hipError_t rcp_launch_pack_i32(const int32_t* src, int64_t n, void* dst, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int64_t nb = (n + kPackBlock - 1) / kPackBlock;
    hipLaunchKernelGGL(rcp_pack_i32_kernel, dim3((unsigned)nb), dim3(kBlock), 0, stream, src, n, nb,
                       static_cast<char*>(dst));
    return hipGetLastError();
}
