// rcp_pack.h -- host-side packing of the packed transfers (rcp_stage.cpp; decoded on the device by
// rcp_kernels.hip rcp_unpack_*): plain C, shared with the CPU check tests/native/pack_check.c.
#pragma once
#include <stdint.h>

// eight strand codes (int8, little-endian in w) -> 16 bits, two per code: the code when it is
// 0..2, else 3 (the device restores -1 for it: the read is dropped).  Per byte: bit 7 set, or
// bits 0..6 + 125 carrying into bit 7, is a code outside 0..2; then the 2-bit fields gathered.
static inline uint32_t rcp_pack_strand8(uint64_t w) {
    const uint64_t k7F = 0x7F7F7F7F7F7F7F7Full, k80 = 0x8080808080808080ull, k03 = 0x0303030303030303ull;
    const uint64_t inv = (((w & k7F) + 0x7D7D7D7D7D7D7D7Dull) | w) & k80;
    uint64_t x = (w & k03) | ((inv >> 7) * 3);
    x = (x | (x >> 6)) & 0x000F000F000F000Full;
    x = (x | (x >> 12)) & 0x000000FF000000FFull;
    x = (x | (x >> 24)) & 0xFFFFull;
    return (uint32_t)x;
}

// one block of int32 values as 16-bit offsets from their minimum when the block spans < 2^16
// (coordinate-sorted starts, chromosome codes, read widths: nearly every block); 0: the block
// does not fit (sent raw).  Two passes: the min / max reduction, then the offsets.
static inline int rcp_pack_block16(const int32_t* v, int len, uint16_t* off, int32_t* base) {
    int32_t lo = v[0], hi = v[0];
    for (int j = 1; j < len; ++j) {
        lo = v[j] < lo ? v[j] : lo;
        hi = v[j] > hi ? v[j] : hi;
    }
    if ((int64_t)hi - (int64_t)lo > 65535) return 0;
    for (int j = 0; j < len; ++j) off[j] = (uint16_t)((uint32_t)v[j] - (uint32_t)lo);
    *base = lo;
    return 1;
}

// chromosome codes one byte each: a code in [0, n_codes) as itself, any other (R's NA from
// match(), a level the readset does not hold) as 255 -- the device restores -1 for it, which
// drops the read as the code did (n_codes <= 255)
static inline uint8_t rcp_pack_code8(int32_t c, int32_t n_codes) {
    return (uint32_t)c < (uint32_t)n_codes ? (uint8_t)c : (uint8_t)255;
}
