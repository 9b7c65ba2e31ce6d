/* CPU check of the packed transfers' host encoders (recoup_amd/csrc/rcp_pack.h) against their
 * definitions: every strand byte value in every position of an 8-code group, random groups; blocks
 * of values decoded back (base + offset) equal to the input, and refused exactly when no base fits.
 * Prints the number of failures. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "rcp_pack.h"

static uint64_t rng = 88172645463325252ull;
static uint64_t next(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
}

int main(void) {
    long bad = 0;
    for (long t = 0; t < 3000000; ++t) {
        int8_t c[8];
        uint64_t r = next();
        memcpy(c, &r, 8);
        if (t < 8 * 256) c[t % 8] = (int8_t)(t / 8);
        if (t % 3 == 0)
            for (int u = 0; u < 8; ++u) c[u] = (int8_t)((uint8_t)c[u] % 4);
        uint64_t w;
        memcpy(&w, c, 8);
        uint32_t exp = 0;
        for (int u = 0; u < 8; ++u) exp |= (uint32_t)((c[u] >= 0 && c[u] <= 2) ? c[u] : 3) << (2 * u);
        bad += rcp_pack_strand8(w) != exp;
    }
    int32_t v[1024];
    uint16_t off[1024];
    for (int t = 0; t < 20000; ++t) {
        const int len = 1 + (int)(next() % 1024);
        const int kind = t % 4;
        int32_t x = (int32_t)(next() % 4000000000u) - 2000000000;
        for (int j = 0; j < len; ++j) {
            if (kind == 0) x += (int32_t)(next() % 64);                    /* sorted, dense */
            else if (kind == 1) x = (int32_t)(next() % 65536) - 32768;     /* spread 2^16 */
            else if (kind == 2) x = (int32_t)(next() % 70000);             /* may not fit */
            else x = (int32_t)next();                                      /* any */
            v[j] = x;
        }
        int64_t lo = v[0], hi = v[0];
        for (int j = 1; j < len; ++j) {
            lo = v[j] < lo ? v[j] : lo;
            hi = v[j] > hi ? v[j] : hi;
        }
        int32_t base = 0;
        const int fits = rcp_pack_block16(v, len, off, &base);
        if (fits != (hi - lo <= 65535)) { ++bad; continue; }
        if (fits)
            for (int j = 0; j < len; ++j) bad += (int32_t)((uint32_t)base + off[j]) != v[j];
    }
    /* chromosome codes one byte each: in-range codes as themselves, any other as 255 (the
     * device's -1: the read is dropped, as the code would drop it) */
    for (int32_t nc = 1; nc <= 255; nc += 17)
        for (long t = 0; t < 20000; ++t) {
            const int32_t c = t < 600 ? (int32_t)t - 300 : (int32_t)next();
            const uint8_t b = rcp_pack_code8(c, nc);
            const int32_t back = b == 255 ? -1 : (int32_t)b;
            bad += (c >= 0 && c < nc) ? back != c : back != -1;
        }
    printf("%ld\n", bad);
    return bad != 0;
}
