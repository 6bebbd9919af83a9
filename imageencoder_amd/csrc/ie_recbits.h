// ie_recbits.h -- which bit positions of a record stream can start a record, 32 positions at once.
//
// A record (Block::streamEncoded / loadFromStream, Block.cpp:406-472) opens with 4 bits bl, then --
// with RLE -- the value count Lw in bl bits; the parse accepts a header when bl != 0 and Lw <= N*N
// (rec_len_head in ie_decode.hip).  valid_mask32 evaluates that test for the 32 headers that
// start at positions p0 .. p0+31 of a 64-bit MSB-first window `v` (bit 63 = position p0; a
// header needs at most 4 + 15 = 19 bits, so position p0+31 still fits) with bitwise operations
// on shifted copies of the window: X_k holds, in bit (31 - q), the bit at position p0 + q + k.
// For bl = b > s (N*N = 2^s) the count fits iff its top b - s bits are zero (Lw < 2^s), or they
// are 0...01 followed by s zero bits (Lw == 2^s).  Returns bit q set iff a record can start at
// p0 + q (LSB-first, as the walk's bitmap reads it).  Host and device: tests/test_recbits builds
// it against the per-position test.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define IE_HD __host__ __device__ __forceinline__
#else
#define IE_HD inline
#endif

IE_HD uint32_t ie_bitrev32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bitreverse32(x);
#else
    x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
    x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
    x = ((x >> 8) & 0x00FF00FFu) | ((x & 0x00FF00FFu) << 8);
    return (x >> 16) | (x << 16);
#endif
}

template <int N>
IE_HD uint32_t valid_mask32(uint64_t v, int rle) {
    constexpr int S = (N == 4) ? 4 : 6;  // N*N = 2^S
    uint32_t X[19];
#pragma unroll
    for (int k = 0; k < 19; k++) X[k] = uint32_t((v << k) >> 32);
    const uint32_t nz = X[0] | X[1] | X[2] | X[3];  // bl != 0
    if (!rle) return ie_bitrev32(nz);
    // bl in [1, S]: any count fits.  S = 4: bl < 8 and bl != 0, minus 5..7 (0101, 0110, 0111):
    // X0 = 0 and (X1 = 0 or X2 = X3 = 0).  S = 6: bl < 8 minus 7, or... (bl <= 6): X0 = 0 and not
    // (X1 & X2 & X3).
    uint32_t ok = (S == 4) ? (~X[0] & (~X[1] | ~(X[2] | X[3])) & nz) : (~X[0] & ~(X[1] & X[2] & X[3]) & nz);
    uint32_t orTop = 0;  // X4 | ... | X(3 + t - 1): the count's top bits before bit t
#pragma unroll
    for (int b = S + 1; b <= 15; b++) {
        const int t = b - S;  // bits above 2^S in a b-bit count
        uint32_t z = 0;       // the S bits below the 2^S bit: X(4 + t) .. X(3 + b)
#pragma unroll
        for (int k = 4 + t; k <= 3 + b; k++) z |= X[k];
        const uint32_t okb = ~(orTop | (X[3 + t] & z));
        const uint32_t m0 = (b & 8) ? X[0] : ~X[0], m1 = (b & 4) ? X[1] : ~X[1];
        const uint32_t m2 = (b & 2) ? X[2] : ~X[2], m3 = (b & 1) ? X[3] : ~X[3];
        ok |= m0 & m1 & m2 & m3 & okb;
        orTop |= X[3 + t];
    }
    return ie_bitrev32(ok);
}
