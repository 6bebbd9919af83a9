// valid_mask32 (imageencoder_amd/csrc/ie_recbits.h) against the per-position header test
// (rec_len_head, ie_decode.hip: bl != 0 and, with RLE, the bl-bit count <= N*N), on random,
// sparse and dense 64-bit windows, both block sizes, RLE on and off.
#include <cstdio>
#include <random>

#include "ie_recbits.h"

template <int N>
static bool head_ok(uint64_t v, int q, int rle) {
    const uint32_t head = uint32_t((v << q) >> 44);  // 20 bits from position q
    const uint32_t bl = head >> 16;
    if (!bl) return false;
    if (!rle) return true;
    const uint32_t lw = (head & 0xFFFFu) >> (16 - bl);
    return lw <= uint32_t(N * N);
}

template <int N>
static long check(uint64_t v, int rle) {
    const uint32_t m = valid_mask32<N>(v, rle);
    long bad = 0;
    for (int q = 0; q < 32; q++) bad += (((m >> q) & 1u) != 0) != head_ok<N>(v, q, rle);
    return bad;
}

int main() {
    std::mt19937_64 g(12345);
    long bad = 0, n = 0;
    for (int i = 0; i < 2000000; i++) {
        uint64_t v = g();
        if (i % 3 == 1) v &= g() & g() & g();  // sparse: long zero runs, counts near 0 and 2^S
        if (i % 3 == 2) v |= g() | g();        // dense
        for (int rle = 0; rle < 2; rle++) {
            bad += check<4>(v, rle) + check<8>(v, rle);
            n += 64;
        }
    }
    // every header value at position 0, with every 16-bit tail
    for (uint64_t h = 0; h < (1u << 20); h++)
        for (int rle = 0; rle < 2; rle++) bad += check<4>(h << 44, rle) + check<8>(h << 44, rle);
    printf("checked %ld positions, %ld mismatches\n", n, bad);
    return bad != 0;
}
