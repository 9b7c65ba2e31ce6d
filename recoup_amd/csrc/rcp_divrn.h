// rcp_divrn.h -- correctly rounded division by a bin width through its reciprocal (device and host)
#pragma once
#ifndef __HIPCC__
#ifndef __host__
#define __host__
#define __device__
#endif
#endif

// RN(a / d) without a division: rd = RN(1 / d), the correctly rounded reciprocal (an IEEE
// division, made once per divisor, not per bin).  q0 = RN(a rd) is within one ulp of a / d, the
// residual a - d q0 is exact with one FMA, and RN(q0 + (a - d q0) rd) is RN(a / d) (Markstein's
// correction theorem: rd within half an ulp of 1 / d, q0 within one ulp of a / d; no overflow or
// underflow for bin numerators and widths).  Three FMA-class instructions instead of the ten of
// the hardware division sequence; bit-equal to a / d (tests/test_host.py checks it exhaustively
// on small numerators and widths and on random large ones).
__host__ __device__ inline double rcp_div_rn(double a, double d, double rd) {
    const double q0 = a * rd;
    const double r = __builtin_fma(-q0, d, a);
    return __builtin_fma(r, rd, q0);
}

