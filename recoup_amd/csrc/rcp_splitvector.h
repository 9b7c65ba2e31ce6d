// rcp_splitvector.h -- device restatement of splitVector's interpolation (R/util.R:17-73) for
// one row whose slice is shorter than its bin count (length(x) < n), shared by the read-pileup
// interpolation kernel (rcp_kernels.hip) and the Rle-input profile kernel (rcp_rle.hip).
// Included by HIP sources only; everything lives in an anonymous namespace.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

#pragma clang fp contract(off)
// stats::spline method "fmm" (R splines.c fmm_spline) on knots x = 1..n: every knot spacing
// d[i] is 1.0, so the operations below are the original ones with the multiplications and
// divisions by d[i] = 1.0 (exact) dropped.  With unit spacing the elimination's pivots
// b_i and multipliers t_i = 1 / b_{i-1} do not depend on y: the host tabulates them once
// per plan (P.spl_tb, same operations in the same order), so the forward elimination is
// the dependent chain c_i = c_i - t_i c_{i-1} alone (one multiply, one subtract per step)
// and the back substitution divides by tabulated pivots; both chains run in
// the first wave's registers (below).  Data-parallel loops run over the block.
// Same operations in the same order per element as R: bit-equal.
// Call from all threads of the team; y, b, c, d in LDS (or global), 0-based.
//
// A team runs one row: the whole block (rcp_interp_kernel, rcp_rle.hip) or a single wave (the
// row-wave pileup kernel interpolates the rows it piles, its arrays in global scratch).
struct BlockTeam {
    __device__ int id() const { return (int)threadIdx.x; }
    __device__ int size() const { return (int)blockDim.x; }
    __device__ void sync() const { __syncthreads(); }
};
struct WaveTeam {
    __device__ int id() const { return (int)(threadIdx.x & 63); }
    __device__ int size() const { return 64; }
    __device__ void sync() const {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
};
// the first wave's stores visible to its own later loads (LDS or global arrays)
__device__ __forceinline__ void lead_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// lane j's double to every lane (j wave-uniform): two v_readlane, no LDS permute
__device__ __forceinline__ double lane_bcast(double v, int j) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), j);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

template <class Team>
__device__ void fmm_spline_team(const Team& tm, int n, const double* y, double* b, double* __restrict__ c, double* d,
                                const double* __restrict__ tb) {
    const int t = tm.id(), nt = tm.size();
    if (n < 3) {
        if (t == 0) {
            if (n == 2) {
                b[0] = b[1] = y[1] - y[0];
            } else if (n == 1) {
                b[0] = 0.0;
            }
            for (int i = 0; i < n; ++i) c[i] = d[i] = 0.0;
        }
        tm.sync();
        return;
    }
    // 1-based i = 2 .. n-1 (0-based i - 1): c[i] = (y[i+1] - y[i]) - (y[i] - y[i-1])
    for (int i = 1 + t; i < n - 1; i += nt) c[i] = (y[i + 1] - y[i]) - (y[i] - y[i - 1]);
    // the tabulated multipliers t_i and pivots b_i staged next to the data (b and d are free
    // until the coefficients below): thread 0's chains read them at LDS latency, not the
    // global table's (one round trip per 8 steps: 0.116 ms of C3's interpolation kernel)
    double* tt = b;
    double* tp = d;
    for (int i = t; i < n; i += nt) {
        tt[i] = tb[2 * i];
        tp[i] = tb[2 * i + 1];
    }
    tm.sync();
    // The two chains run in the first wave's REGISTERS: lane l holds elements 4 l .. 4 l + 3 of a
    // 256-element segment (c, the multipliers, the pivots and their reciprocals), and the lanes
    // take their turns in order, the running value passed on by v_readlane -- each step is its
    // dependent arithmetic alone, not an LDS round trip (thread 0 walking LDS spent ~80 cycles a
    // step: tools/spline_timing.hip).  Same operations in the same order: the same bits.
    if (t < 64) {
        constexpr int V = 4, SEG = 64 * V;  // elements per lane, per segment
        const int lane = t;
        double c1 = 0.0, cn = 0.0;  // (every lane: the same operations)
        if (n > 3) {
            c1 = c[2] / 2.0 - c[1] / 2.0;
            cn = c[n - 2] / 2.0 - c[n - 3] / 2.0;
            c1 = c1 / 3.0;  // * d[1] * d[1] (= 1) / 3
            cn = -cn / 3.0;
        }
        // forward elimination: t = d[i-1] / b[i-1]; b[i] -= t d[i-1]; c[i] -= t c[i-1], i = 1 .. n-1.
        // The padding past n - 1 enters as zeros, so the lanes' V steps run unconditionally (the
        // padding is never stored, and c[n - 1] is read back below); element 0 (lane 0 of the
        // first segment) is kept as c1 by the one conditional turn
        double cp = c1;
        for (int s0 = 0; s0 < n; s0 += SEG) {
            double cv[V], tv[V];
#pragma unroll
            for (int u = 0; u < V; ++u) {
                const int i = s0 + V * lane + u;
                cv[u] = i == 0 ? c1 : (i == n - 1 ? cn : (i < n ? c[i] : 0.0));
                tv[u] = (i >= 1 && i < n) ? tt[i] : 0.0;
            }
            const int last = min(63, (n - 1 - s0) / V);
            for (int j = 0; j <= last; ++j) {
                if (lane == j) {
                    if (s0 == 0 && j == 0) {
#pragma unroll
                        for (int u = 1; u < V; ++u) {
                            cp = cv[u] - tv[u] * cp;
                            cv[u] = cp;
                        }
                    } else {
#pragma unroll
                        for (int u = 0; u < V; ++u) {
                            cp = cv[u] - tv[u] * cp;
                            cv[u] = cp;
                        }
                    }
                }
                cp = lane_bcast(cp, j);
            }
#pragma unroll
            for (int u = 0; u < V; ++u) {
                const int i = s0 + V * lane + u;
                if (i < n) c[i] = cv[u];
            }
        }
        lead_wave_sync();
        cp = c[n - 1];  // (the padding steps ran past it)
        const double bn = -1.0 - tt[n - 1];  // b[n-1] = -1 - t_{n-1}
        // back substitution: c[i] = (c[i] - c[i+1]) / b[i].  The pivot's reciprocal is in the
        // table already -- t_{i+1} = RN(1 / b_i), the host's IEEE division -- so each quotient is
        // q = RN(x y), then corrected once: RN(q + RN(x - q b) y) with the remainder exact by
        // FMA is the correctly rounded x / b (Markstein), i.e. the division's bits, in three
        // dependent operations instead of the division's ten; zeros (signed) and extreme
        // exponents, where the theorem's assumptions fail, take the division itself
        // (the range test is off the dependent path: a segment any of whose steps left it is run
        // again with the division itself -- never on coverage data)
        // (+0 too: RN(+0 y) corrected is the division's signed zero for either sign of b; -0, which
        // coverage data never makes, and tiny or huge x take the division)
        auto in_range = [](double x) -> bool {
            const double ax = __builtin_fabs(x);
            return (ax >= 0x1p-960 && ax <= 0x1p+960) || __builtin_bit_cast(uint64_t, x) == 0;
        };
        double cnext = cp / bn;  // c[n-1]
        const int jn = ((n - 1) % SEG) / V;  // the lane holding element n - 1 in the last segment
        for (int s0 = ((n - 1) / SEG) * SEG; s0 >= 0; s0 -= SEG) {
            double cv[V], bv[V], yv[V];
#pragma unroll
            for (int u = 0; u < V; ++u) {
                const int i = s0 + V * lane + u;
                cv[u] = i < n ? c[i] : 0.0;
                bv[u] = i < n ? tp[i] : 1.0;
                yv[u] = i + 1 < n ? tt[i + 1] : 1.0;
            }
            const bool top = s0 + SEG >= n;  // the segment holding element n - 1
            const double centry = cnext;
            for (int exact = 0; exact < 2; ++exact) {
                bool off = false;
                double w[V];
#pragma unroll
                for (int u = 0; u < V; ++u) w[u] = cv[u];
                cnext = centry;
                for (int j = top ? jn : 63; j >= 0; --j) {
                    if (lane == j) {
                        if (top && j == jn) {  // element n - 1 and the padding above it
#pragma unroll
                            for (int u = V - 1; u >= 0; --u) {
                                const int i = s0 + V * j + u;
                                if (i == n - 1) {
                                    w[u] = cnext;
                                } else if (i < n - 1) {
                                    const double x = w[u] - cnext;
                                    if (exact) {
                                        cnext = x / bv[u];
                                    } else {
                                        off |= !in_range(x);
                                        const double q = x * yv[u];
                                        cnext = __builtin_fma(__builtin_fma(-q, bv[u], x), yv[u], q);
                                    }
                                    w[u] = cnext;
                                }
                            }
                        } else if (exact) {
#pragma unroll
                            for (int u = V - 1; u >= 0; --u) {
                                cnext = (w[u] - cnext) / bv[u];
                                w[u] = cnext;
                            }
                        } else {
#pragma unroll
                            for (int u = V - 1; u >= 0; --u) {
                                const double x = w[u] - cnext;
                                off |= !in_range(x);
                                const double q = x * yv[u];
                                cnext = __builtin_fma(__builtin_fma(-q, bv[u], x), yv[u], q);
                                w[u] = cnext;
                            }
                        }
                    }
                    cnext = lane_bcast(cnext, j);
                }
                if (!__builtin_amdgcn_ballot_w64(off)) {  // (exact: off stays false)
#pragma unroll
                    for (int u = 0; u < V; ++u) cv[u] = w[u];
                    break;
                }
            }
#pragma unroll
            for (int u = 0; u < V; ++u) {
                const int i = s0 + V * lane + u;
                if (i < n) c[i] = cv[u];
            }
        }
        lead_wave_sync();
        if (lane == 0) b[n - 1] = (y[n - 1] - y[n - 2]) + (c[n - 2] + 2.0 * c[n - 1]);
    }
    tm.sync();
    // coefficients: b[i] = (y[i+1] - y[i]) - (c[i+1] + 2 c[i]); d[i] = c[i+1] - c[i]; c[i] *= 3
    for (int i = t; i < n - 1; i += nt) {
        const double ci = c[i], cn1 = c[i + 1];
        b[i] = (y[i + 1] - y[i]) - (cn1 + 2.0 * ci);
        d[i] = cn1 - ci;
    }
    tm.sync();
    for (int i = t; i < n; i += nt) c[i] = 3.0 * c[i];
    if (t == 0) d[n - 1] = d[n - 2];
    tm.sync();
}

[[maybe_unused]] __device__ void fmm_spline_block(int n, const double* y, double* b, double* __restrict__ c, double* d,
                                 const double* __restrict__ tb) {
    fmm_spline_team(BlockTeam{}, n, y, b, c, d, tb);
}

__device__ double seq_point(int L, int n, int i) {
    // seq.int(1, L, length.out = n)[i] as do_seq computes it
    if (i == 0) return 1.0;
    if (i == n - 1) return (double)L;
    const double by = ((double)L - 1.0) / (double)(n - 1);
    return (i < n / 2) ? 1.0 + (double)i * by : (double)L - (double)(n - 1 - i) * by;
}

// spline_eval's interval walk (R splines.c): the previous interval i is kept while
// x[i] <= u <= x[i+1], else bisection (knots x = 1..n)
__device__ __forceinline__ int spline_bisect(int L, double u) {
    int i = 0, j = L;
    do {
        const int m = (i + j) / 2;
        if (u < (double)(m + 1)) j = m; else i = m;
    } while (j > i + 1);
    return i;
}

// The same interval for point k alone, for interpolated rows (L < n: output points closer
// than one knot apart).  The walk keeps interval i for u in [i+1, i+2] and bisects
// otherwise; the bisection lands on floor(u) - 1, so the two differ only at a point sitting
// exactly on a knot m = i + 2 just after a point of interval i (it keeps i, the evaluation
// runs at dx = 1).  Because consecutive points are less than 1 apart, the interval held at
// point k - 1 is bisect(u_{k-1}) whenever it matters, and each point is decided alone.
__device__ __forceinline__ int spline_interval_at(int L, int n, int k) {
    const double u = seq_point(L, n, k);
    const int prev = k == 0 ? 0 : spline_bisect(L, seq_point(L, n, k - 1));
    if (u < (double)(prev + 1) || (prev < L - 1 && (double)(prev + 2) < u)) return spline_bisect(L, u);
    return prev;
}

// spline_eval's cubic on interval i (no FMA contraction: R's rounding)
__device__ double spline_eval_at(const double* y, const double* b, const double* c, const double* d, int i,
                                 double u) {
    const double dx = u - (double)(i + 1);
    return y[i] + dx * (b[i] + dx * (c[i] + dx * d[i]));
}
#pragma clang fp contract(on)


// splitVector of a row slice x[0 .. L) (doubles, already x * scale) into n > L bins, written to
// out[k * ld] (k = 0 .. n - 1).  mode 1: spline(x, n)$y clipped at 0 (auto with (n - L) / n >= 0.2,
// or "spline"); 3: neighborhood fill with the R-RNG positions nb_pos (1-based, sorted,
// set.seed(42); sort(sample(3:(n - 2), L - 4))); otherwise "linear", whose switch arm is spelled
// "inear" (util.R:49): x stays short and rbind recycles it.  Scratch follows x: b, c, d (L + 1
// each) for the spline, or the n pre-fill values of the neighborhood fill; every output point is
// computed and stored by its own thread (no staging of the n outputs: the block's scratch stays
// small enough for every interpolated row's block to be resident at once).  Call with every
// thread of the team.
template <class Team>
__device__ void interp_finish_team(const Team& tm, int mode, int L, int n, double* x, const int32_t* nb_pos,
                                   const double* spl_tb, double* out, size_t ld) {
    const int t0 = tm.id(), nt = tm.size();
    double* b = x + L + 1;
    if (mode == 1) {  // spline(x, n = n)$y, then x[x < 0] <- 0
        double* c = b + L + 1;
        double* d = c + L + 1;
        fmm_spline_team(tm, L, x, b, c, d, spl_tb);
        auto put = [&](int k, int iv) {
            const double v = L == 1 ? x[0] : spline_eval_at(x, b, c, d, iv, seq_point(L, n, k));
            out[(size_t)k * ld] = v < 0 ? 0.0 : v;
        };
        if (L < n) {  // always, for rows of this kernel; the sequential walk stays as the rule
            for (int k = t0; k < n; k += nt) put(k, spline_interval_at(L, n, k));
        } else if (t0 == 0) {
            int i = 0;  // spline_eval's walk, point by point
            for (int k = 0; k < n; ++k) {
                const double u = seq_point(L, n, k);
                if (u < (double)(i + 1) || (i < L - 1 && (double)(i + 2) < u)) i = spline_bisect(L, u);
                put(k, i);
            }
        }
    } else if (mode == 3) {  // neighborhood fill (util.R:53-69), from the pre-fill vector
        const int32_t* pos = nb_pos;
        double* pre = b;
        for (int i = t0; i < n; i += nt) pre[i] = __builtin_nan("");
        tm.sync();
        if (t0 == 0) {
            pre[0] = x[0];
            pre[1] = x[1];
            pre[n - 2] = x[L - 2];
            pre[n - 1] = x[L - 1];
        }
        for (int i = t0; i < L - 4; i += nt) pre[pos[i] - 1] = x[2 + i];
        tm.sync();
        for (int z = t0; z < n; z += nt) {
            double v;
            if (!isnan(pre[z])) {
                v = pre[z];
            } else {
                double sm = 0.0;
                int m = 0;
                const int nb[4] = {z - 2, z - 1, z + 1, z + 2};
                for (int q = 0; q < 4; ++q)
                    if (nb[q] >= 0 && nb[q] < n && !isnan(pre[nb[q]])) {
                        sm += pre[nb[q]];
                        ++m;
                    }
                v = m ? sm / m : __builtin_nan("");
            }
            out[(size_t)z * ld] = v;
        }
    } else {  // "linear": the switch arm is spelled "inear" -> x unchanged; rbind recycles
        for (int i = t0; i < n; i += nt) out[(size_t)i * ld] = x[i % L];
    }
}

__device__ void interp_finish(int mode, int L, int n, double* x, const int32_t* nb_pos, const double* spl_tb,
                              double* out, size_t ld) {
    interp_finish_team(BlockTeam{}, mode, L, n, x, nb_pos, spl_tb, out, ld);
}

// one wave's interpolation of a row (the row-wave pileup kernel): a call, so that the spline's
// registers are not added to the pileup loop's
[[maybe_unused]] __device__ __attribute__((noinline)) void interp_finish_wave(int mode, int L, int n, double* x, const int32_t* nb_pos,
                                                             const double* spl_tb, double* out, size_t ld) {
    const WaveTeam tm;
    tm.sync();
    interp_finish_team(tm, mode, L, n, x, nb_pos, spl_tb, out, ld);
}

}  // namespace
