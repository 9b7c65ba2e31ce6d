/* Checks rcp_div_rn (recoup_amd/csrc/rcp_divrn.h) against IEEE division: exhaustively for
 * numerators 0 .. 2^NBITS - 1 and widths 1 .. DMAX, then on random (numerator < 2^32,
 * width < 2^20, scale factor: none, uniform (0, 1) or min(lib) / lib) triples.  Test infrastructure (tests/test_host.py). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include "rcp_divrn.h"

static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}

int main(int argc, char** argv) {
    const int nbits = argc > 1 ? atoi(argv[1]) : 16, dmax = argc > 2 ? atoi(argv[2]) : 1024;
    const long nrand = argc > 3 ? atol(argv[3]) : 1000000;
    long bad = 0;
    for (int d = 1; d <= dmax; ++d) {
        const double dd = (double)d, rd = 1.0 / dd;
        for (uint32_t n = 0; n < (1u << nbits); ++n) {
            const double a = (double)n;
            if (rcp_div_rn(a, dd, rd) != a / dd) ++bad;
        }
    }
    for (long i = 0; i < nrand; ++i) {
        const double n = (double)(uint32_t)xr();
        const double dd = (double)(1 + (xr() & 0xFFFFF));
        double sc = 1.0;
        if (i % 3 == 1) sc = (double)(xr() >> 11) / 9007199254740992.0;
        if (i % 3 == 2) {  /* calcLinearFactors: min(lib) / lib of library sizes up to 2^31 */
            const double lib = (double)(1 + (xr() & 0x7FFFFFFF)), mn = (double)(1 + (uint64_t)(lib * ((double)(xr() >> 11) / 9007199254740992.0)));
            sc = mn / lib;
        }
        const double a = n * sc;
        if (rcp_div_rn(a, dd, 1.0 / dd) != a / dd) ++bad;
    }
    printf("%ld\n", bad);
    return bad != 0;
}
