// rcp_rng.h -- R's default RNG as splitVector uses it (product side, host only).
//
// splitVector (R/util.R:74-80) lays bins out with `set.seed(42); add <- sample(1:n, dif)`
// and the neighborhood interpolation (R/util.R:53-58) with
// `set.seed(42); sort(sample(3:(n-2), L-4))`.  Because the seed is reset on every call the
// layout depends only on (n, dif) -- the plan builder computes each distinct layout once.
//
// Restated from R's public sources (src/main/RNG.c, src/main/random.c): set.seed ->
// 50 LCG scrambles + 625 LCG words (mti = 624), MT19937 with R's tempering, unif_rand
// fixup into (0, 1), R_unif_index (sample.kind "Rejection" since R 3.6.0 -- rbits in
// 16-bit chunks -- or the older "Rounding"), sample.int without replacement by
// partial Fisher-Yates on 0..n-1.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

namespace rcp {

class RRng {
  public:
    explicit RRng(uint32_t seed) { set_seed(seed); }

    void set_seed(uint32_t seed) {
        for (int j = 0; j < 50; ++j) seed = 69069u * seed + 1u;
        for (int j = 0; j < kN + 1; ++j) {
            seed = 69069u * seed + 1u;
            state_[j] = seed;
        }
        state_[0] = kN;  // mti = N: regenerate on the first draw
    }

    double unif_rand() {
        const double v = genrand();
        constexpr double i2_32m1 = 2.328306437080797e-10;
        if (v <= 0.0) return 0.5 * i2_32m1;
        if (1.0 - v <= 0.0) return 1.0 - 0.5 * i2_32m1;
        return v;
    }

    double unif_index(double dn, bool rounding) {
        if (rounding) return std::floor(dn * unif_rand());
        if (dn <= 0) return 0.0;
        const int bits = (int)std::ceil(std::log2(dn));
        double dv;
        do {
            int64_t v = 0;
            for (int n = 0; n <= bits; n += 16) {
                const int v1 = (int)std::floor(unif_rand() * 65536);
                v = 65536 * v + v1;
            }
            dv = (double)(v & ((int64_t(1) << bits) - 1));
        } while (dn <= dv);
        return dv;
    }

    // sample.int(n, k) without replacement; 1-based values in draw order.
    std::vector<int> sample_int(int n, int k, bool rounding) {
        std::vector<int> pool(n), out(k);
        for (int i = 0; i < n; ++i) pool[i] = i;
        int m = n;
        for (int i = 0; i < k; ++i) {
            const int j = (int)unif_index((double)m, rounding);
            out[i] = pool[j] + 1;
            pool[j] = pool[--m];
        }
        return out;
    }

    // sort(sample(n, k)) of the preprocessing steps (R/ranges.R:32-62), 1-based.  R's
    // sample.int switches to .Internal(sample2()) -- rejection of repeated unif_index draws --
    // when n > 1e7 and k <= n / 2; otherwise it is the partial Fisher-Yates of sample_int.
    // Returns false when k > n (R: "cannot take a sample larger than the population").
    bool sample_sorted(int64_t n, int64_t k, bool rounding, std::vector<int64_t>* out) {
        out->clear();
        if (k < 0 || k > n) return false;
        if (n > 10000000 && 2 * k <= n) {
            std::vector<uint64_t> seen((size_t)(n / 64 + 1), 0);
            for (int64_t got = 0; got < k;) {
                const int64_t v = (int64_t)unif_index((double)n, rounding);
                uint64_t& w = seen[(size_t)(v >> 6)];
                const uint64_t bit = uint64_t(1) << (v & 63);
                if (!(w & bit)) {
                    w |= bit;
                    ++got;
                }
            }
            out->reserve((size_t)k);
            for (size_t i = 0; i < seen.size(); ++i)
                for (uint64_t w = seen[i]; w; w &= w - 1) out->push_back((int64_t)(i * 64 + __builtin_ctzll(w)) + 1);
            return true;
        }
        std::vector<int64_t> pool((size_t)n);
        for (int64_t i = 0; i < n; ++i) pool[(size_t)i] = i;
        int64_t m = n;
        out->resize((size_t)k);
        for (int64_t i = 0; i < k; ++i) {
            const int64_t j = (int64_t)unif_index((double)m, rounding);
            (*out)[(size_t)i] = pool[(size_t)j] + 1;
            pool[(size_t)j] = pool[(size_t)--m];
        }
        std::sort(out->begin(), out->end());
        return true;
    }

  private:
    static constexpr int kN = 624;
    static constexpr int kM = 397;
    uint32_t state_[kN + 1];

    double genrand() {
        static constexpr uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
        uint32_t* mt = state_ + 1;
        uint32_t mti = state_[0];
        uint32_t y;
        if (mti >= (uint32_t)kN) {
            int kk = 0;
            for (; kk < kN - kM; ++kk) {
                y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
                mt[kk] = mt[kk + kM] ^ (y >> 1) ^ mag01[y & 1u];
            }
            for (; kk < kN - 1; ++kk) {
                y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
                mt[kk] = mt[kk + (kM - kN)] ^ (y >> 1) ^ mag01[y & 1u];
            }
            y = (mt[kN - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
            mt[kN - 1] = mt[kM - 1] ^ (y >> 1) ^ mag01[y & 1u];
            mti = 0;
        }
        y = mt[mti++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        state_[0] = mti;
        return (double)y * 2.3283064365386963e-10;
    }
};

// Prefix counts of the enlarged bins of splitVector's layout for (n, dif):
// cnt[k] = #{ bins j < k : j in sample(1:n, dif) }, k = 0..n.  Bin k then spans
// [bs*k + cnt[k], bs*(k+1) + cnt[k+1]).
inline std::vector<int32_t> bin_layout_counts(int n, int dif, bool rounding) {
    RRng rng(42);
    std::vector<uint8_t> big(n, 0);
    if (dif > 0)
        for (int a : rng.sample_int(n, dif, rounding)) big[a - 1] = 1;
    std::vector<int32_t> cnt(n + 1, 0);
    for (int k = 0; k < n; ++k) cnt[k + 1] = cnt[k] + big[k];
    return cnt;
}

// orig.pos of the neighborhood interpolation: sort(sample(3:(n-2), L-4)) (1-based).
// Returns false where R itself raises an error.
inline bool neighborhood_positions(int n, int L, bool rounding, std::vector<int32_t>* out) {
    if (L < 4 || n < 5) return false;
    const int k = L - 4;
    const int pool = n - 4;  // length(3:(n-2))
    RRng rng(42);
    std::vector<int> pos;
    if (pool == 1) {
        // sample(x = 3, k): a length-one numeric x >= 1 is sample.int(3, k)
        if (k > 3) return false;
        pos = rng.sample_int(3, k, rounding);
    } else {
        if (k > pool) return false;
        pos = rng.sample_int(pool, k, rounding);
        for (int& p : pos) p += 2;
    }
    std::sort(pos.begin(), pos.end());
    out->assign(pos.begin(), pos.end());
    return true;
}

}  // namespace rcp
