// rcp_divrn.h -- correctly rounded division by a bin width through its reciprocal (device and host)
#pragma once
#ifndef __HIPCC__
#ifndef __host__
#define __host__
#define __device__
#endif
#endif

// RN(a / d) without a division: rd = RN(1 / d), the correctly rounded reciprocal (an IEEE
// division, made once per divisor, not per bin).  q0 = RN(a rd), the residual a - d q0 is exact
// with one FMA, and RN(q0 + (a - d q0) rd) corrects q0 (Markstein's final correction step).  The
// textbook proof of that step assumes q0 within one ulp of a / d; q0 = RN(a RN(1/d)) is only
// guaranteed within about 1.5 ulp, so equality with the IEEE division a / d is EMPIRICALLY
// checked, not proven: tests/native/div_rn_check.c (run by tests/test_host.py) compares it
// exhaustively on every numerator < 2^18 over widths 1..600, and on random numerators < 2^32
// over widths < 2^20 unscaled, with a uniform scale in (0, 1), and with linear normalisation
// factors min(lib) / lib (R/util.R:349-362) of random library sizes.  Three FMA-class
// instructions instead of the ten of the hardware division sequence.
__host__ __device__ inline double rcp_div_rn(double a, double d, double rd) {
    const double q0 = a * rd;
    const double r = __builtin_fma(-q0, d, a);
    return __builtin_fma(r, rd, q0);
}

