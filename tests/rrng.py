"""R's random number generator restated in pure Python, independently of the two C copies
(oracle/rcp_oracle.c for the checker, recoup_amd/csrc/rcp_rng.h for the product): test
infrastructure only.

splitVector's bin layouts (R/util.R:74-80: set.seed(seed); sample(1:n, dif)) and its
neighborhood positions (R/util.R:26, :56: sort(sample(3:(n - 2), length(x) - 4))), and the
downsample / sampleto draws of preprocessRanges (R/ranges.R:32-62), come from R's default RNG:

  * set.seed(seed), RNGkind "Mersenne-Twister" (R src/main/RNG.c, RNG_Init + FixupSeeds): the
    seed is scrambled by 50 steps of seed = 69069 * seed + 1, the next 625 steps fill the
    generator's state (word 0 is the position `mti`, reset to 624), all modulo 2^32;
  * unif_rand (MT_genrand): MT19937 with R's tempering, y * 2.3283064365386963e-10, kept inside
    (0, 1) by `fixup`;
  * sample.int (src/main/random.c do_sample, R >= 3.6 sample.kind = "Rejection"): a partial
    Fisher-Yates over 0..n-1 whose index is R_unif_index(n) = rbits(ceil(log2 n)) drawn 16 bits
    per unif_rand until below n; sample.kind = "Rounding" takes floor(n * unif_rand()); for
    n > 1e7 and size <= n / 2 sample.int uses .Internal(sample2()), R_unif_index until `size`
    distinct values (a hash set).
"""
import math

N, M = 624, 397
MATRIX_A, UPPER, LOWER = 0x9908B0DF, 0x80000000, 0x7FFFFFFF
I2_32M1 = 2.328306437080797e-10  # 1 / (2^32 - 1)


class RRng:
    def __init__(self, seed, kind="Rejection"):
        s = seed & 0xFFFFFFFF
        for _ in range(50):
            s = (69069 * s + 1) & 0xFFFFFFFF
        words = []
        for _ in range(N + 1):
            s = (69069 * s + 1) & 0xFFFFFFFF
            words.append(s)
        self.mt = words[1:]
        self.mti = N  # FixupSeeds(initial = 1): dummy[0] = 624
        self.kind = kind

    def _genrand(self):
        mt = self.mt
        if self.mti >= N:
            for kk in range(N - M):
                y = (mt[kk] & UPPER) | (mt[kk + 1] & LOWER)
                mt[kk] = mt[kk + M] ^ (y >> 1) ^ (MATRIX_A if y & 1 else 0)
            for kk in range(N - M, N - 1):
                y = (mt[kk] & UPPER) | (mt[kk + 1] & LOWER)
                mt[kk] = mt[kk + (M - N)] ^ (y >> 1) ^ (MATRIX_A if y & 1 else 0)
            y = (mt[N - 1] & UPPER) | (mt[0] & LOWER)
            mt[N - 1] = mt[M - 1] ^ (y >> 1) ^ (MATRIX_A if y & 1 else 0)
            self.mti = 0
        y = mt[self.mti]
        self.mti += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y * 2.3283064365386963e-10

    def unif_rand(self):
        x = self._genrand()
        if x <= 0.0:
            return 0.5 * I2_32M1
        if 1.0 - x <= 0.0:
            return 1.0 - 0.5 * I2_32M1
        return x

    def runif(self, k):
        return [self.unif_rand() for _ in range(k)]

    def unif_index(self, n):
        if self.kind == "Rounding":
            return math.floor(n * self.unif_rand())
        if n <= 0:
            return 0
        bits = math.ceil(math.log2(n))
        while True:
            v = 0
            for _ in range(0, bits + 1, 16):
                v = 65536 * v + math.floor(self.unif_rand() * 65536)
            v &= (1 << bits) - 1
            if v < n:
                return v

    def sample_int(self, n, k):
        """sample.int(n, k) without replacement (1-based), R's own draw order."""
        if k > n:
            raise ValueError("cannot take a sample larger than the population")
        if n > 1e7 and k <= n / 2:  # .Internal(sample2(n, k))
            seen, out = set(), []
            while len(out) < k:
                v = self.unif_index(n) + 1
                if v not in seen:
                    seen.add(v)
                    out.append(v)
            return out
        x = list(range(n))
        out = []
        for _ in range(k):
            j = self.unif_index(n)
            out.append(x[j] + 1)
            n -= 1
            x[j] = x[n]
        return out
