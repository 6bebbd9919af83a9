// imageencoder_amd/csrc/ie_encode.hip -- the block encoder for gfx950 (MI355X).
//
// One launch encodes a batch of frames.  Work decomposition:
//   lane      = one "group" of BPT horizontally adjacent N x N blocks (4 x 4x4 or 1 x 8x8), so a
//               wave reads 64 x 16 B (or 64 x 8 B) contiguous bytes per pixel row;
//   workgroup = one tile of kTPB groups (<= 1024 blocks), never straddling a frame.
// Per tile, in one pass over the pixels (each input byte is read from HBM once, each output word
// written once):
//   1. level shift + forward DCT + quantise every block (Block.cpp:139-153, algo.cpp:309-331):
//      FAST = the butterfly FP32 DCT of ie_dct.h, whose error the host bounds rigorously;
//      coefficients whose quotient lies within that bound of a rounding tie are re-evaluated in
//      the reference's exact FP64 operation order.  EXACT = every coefficient in FP64 order.
//   2. zig-zag RLE sizing (Block.cpp:186-232, :383-397): bl, Lw, record length;
//   3. workgroup exclusive scan of record lengths; the records are written MSB-first into an
//      LDS image of the tile's bit stream (Block.cpp:372-413, BitStream.cpp:61-77);
//   4. decoupled look-back over the preceding tiles of the chain for the tile's global bit offset
//      (the whole workgroup reads 1024 predecessor states per round trip);
//   5. funnel-shifted, coalesced store of the LDS image into the output words.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ie_common.hpp"
#include "ie_dct.h"
#include "ie_device.h"

namespace ie {

template <int N> struct ZigZag;
template <> struct ZigZag<4> {
    static constexpr int idx[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
};
template <> struct ZigZag<8> {
    static constexpr int idx[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
};

// pos[k] = zig-zag position of natural index k (inverse of ZigZag<N>::idx)
template <int N> struct ZigZagInv;
template <> struct ZigZagInv<4> {
    static constexpr int pos[16] = {0, 1, 5, 6, 2, 4, 7, 12, 3, 8, 11, 13, 9, 10, 14, 15};
};
template <> struct ZigZagInv<8> {
    static constexpr int pos[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                                    3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                                    10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                                    21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};
};

#ifndef IE_PX_AUX8
#define IE_PX_AUX8 2  // cache-policy bits of encode_kernel<8>'s pixel DMA: nt (HBM-resident C3 141.7 against 143.1 us)
#endif
#ifndef IE_PROFILE
#define IE_PROFILE 0
#endif
#ifndef IE_BPT4
#define IE_BPT4 4
#endif
#ifndef IE_WAVES4
#define IE_WAVES4 5
#endif
#ifndef IE_WAVES8
#define IE_WAVES8 4
#endif
// Threads per tile (= per workgroup).  256 (four waves, 1024 4x4 blocks); 64 makes every wave an
// independent tile (no workgroup barriers, 16 tiles per CU) but quadruples the look-backs, which
// measured slower.
#ifndef IE_TPB
#define IE_TPB 256
#endif
constexpr int kEncTPB = IE_TPB;
template <int N> struct Geo;
template <> struct Geo<4> {  // IE_BPT4 blocks side by side: 4 * IE_BPT4 bytes per pixel row per lane
    static constexpr int BPT = IE_BPT4;
    static constexpr int WAVES = IE_WAVES4;  // __launch_bounds__ occupancy hint (waves per SIMD)
};
template <> struct Geo<8> {  // one block: 8 bytes per pixel row per lane
    static constexpr int BPT = 1;
    static constexpr int WAVES = IE_WAVES8;  // 4: <= 128 registers
};

// The tile's LDS bit image: kEncTPB * BPT records of at most rec_bits bits (the matrix's bound,
// ie_capi.cpp build_tables), plus slack for the zero pairs emit_block2 may OR in past the last
// record (<= 16 * N*N bits) and the store's look-ahead word; at least the fix-up's scratch.
// Sized per launch (dynamic LDS): a smaller image measured faster at equal occupancy.
constexpr int image_words_for(int n, int bpt, int rec_bits) {
    return ((kEncTPB * bpt * rec_bits + 31) / 32 + 4 + (n * n + 3) + 3) / 4 * 4;  // keeps misc 16-B aligned
}

// Structural fix-up compaction (FAST 4x4): per-wave LDS task slots in the (not yet built) tile
// image, after the pixel area.
#ifndef IE_FIX_UNROLL
#define IE_FIX_UNROLL 16
#endif
// FAST 4x4: the tile's pixels go straight from HBM into LDS (global_load_lds_dwordx4, no VGPR
// destination) in the fix-up's pixel area, laid out per wave as [row r][lane][4 words] (block b
// of a lane = word b of each row), and every block reads its four rows back when it is
// transformed: no pixel registers live across the tile's phases.
constexpr int kFixPix = 0;  // [BPT][TPB] x 4 words: the pixels
template <int B> constexpr int fix_tasks() { return kFixPix + B * kEncTPB * 4; }  // per wave: [64] tasks, [64] results
template <int B> constexpr int fix_words() { return fix_tasks<B>() + (kEncTPB / 64) * 128; }  // the image is never smaller
// 8x8: one 16-word block per lane at a 20-word stride (16-byte writes land on distinct banks)
constexpr int kFix8Stride = 20;
constexpr int kFix8Tasks = kFix8Stride * kEncTPB;
constexpr int kNsStage = 4;  // non-structural rows staged per pass, per wave
constexpr int kFix8Stage = kFix8Tasks + (kEncTPB / 64) * 128;
constexpr int kFix8Words = kFix8Stage + (kEncTPB / 64) * kNsStage * 64 * 2;

template <int WPR>
__device__ __forceinline__ uint32_t pix(const uint32_t (&row)[WPR], int byte) {
    return (row[byte >> 2] >> (8 * (byte & 3))) & 0xFFu;
}

// The pixel bytes of one block, packed four to a word (row-major): the argument of the
// out-of-line FP64 path, passed in registers.
template <int N> struct BlockPx {
    uint32_t w[N * N / 4];
};

// Exact coefficient in the reference's FP64 order (algo.cpp:314-325, Block.cpp:149-152):
//   acc = 0; for i, j: acc = acc + P[uv][ij] * x[ij];  D = acc * (C(u)C(v));  round(D / q)
// with x[ij] = double(p) - 128 (Block.cpp:141-143).  This file is compiled with
// -ffp-contract=off, so every product and sum is rounded separately as in the reference; the
// division is IEEE (a multiply by the exact reciprocal when q is a power of two); the rounding is
// half away from zero (std::round).  Out of line: it runs only for the few coefficients whose
// FP32 quotient lies near a rounding tie, and must not inflate the hot path's registers.
template <int N>
__device__ __forceinline__ int exact_coef_inl(const EncTables* __restrict__ tab, int k, BlockPx<N> px) {
    constexpr int NN = N * N;
    const double* P = &tab->P[k * NN];
    double acc = 0.0;
#pragma unroll
    for (int ij = 0; ij < NN; ij++) {
        const double x = double(int((px.w[ij >> 2] >> (8 * (ij & 3))) & 0xFFu) - 128);  // == double(p) + (-128.0), exactly
        acc = acc + P[ij] * x;
    }
    const double D = acc * tab->S[k];
    const double rq = tab->rq[k];
    const double t = (rq != 0.0) ? D * rq : D / tab->qd[k];
    double r = trunc(t);
    if (fabs(t - r) >= 0.5) r += copysign(1.0, t);
    return int(r);
}

// The same evaluation with the coefficient's row of P and its scalars taken from an LDS copy.
// (The row is walked four terms at a time so the compiler does not hoist all NN LDS loads and
// conversions at once: the caller's packed coefficients stay live around it.)
template <int N>
__device__ __forceinline__ int exact_coef_row(const double* P, double S, double rq, double qd, const BlockPx<N>& px) {
    constexpr int NN = N * N;
    double acc = 0.0;
#pragma unroll IE_FIX_UNROLL
    for (int ij = 0; ij < NN; ij++) {
        const double x = double(int((px.w[ij >> 2] >> (8 * (ij & 3))) & 0xFFu) - 128);  // == double(p) + (-128.0), exactly
        acc = acc + P[ij] * x;
    }
    const double D = acc * S;
    const double t = (rq != 0.0) ? D * rq : D / qd;
    double r = trunc(t);
    if (fabs(t - r) >= 0.5) r += copysign(1.0, t);
    return int(r);
}

// exact_coef_row for a fix-up task: the block's pixel words are read from their LDS slot pw
// (4 pixels per word) and the row through a generic pointer P (the LDS copy of a structural row or
// the table in global memory), one pixel word per step of a loop the compiler need not unroll --
// a register copy of the pixels indexed by a loop counter would live in scratch memory.
template <int N>
__device__ __forceinline__ int exact_coef_task(const double* P, double S, double rq, double qd, const uint32_t* pw) {
    constexpr int NN = N * N;
    double acc = 0.0;
    for (int w = 0; w < NN / 4; w++) {
        const uint32_t px4 = pw[w];
        double pr[4];
#pragma unroll
        for (int e = 0; e < 4; e++) pr[e] = P[4 * w + e];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const double x = double(int((px4 >> (8 * e)) & 0xFFu) - 128);
            acc = acc + pr[e] * x;
        }
    }
    const double D = acc * S;
    const double t = (rq != 0.0) ? D * rq : D / qd;
    double r = trunc(t);
    if (fabs(t - r) >= 0.5) r += copysign(1.0, t);
    return int(r);
}

// exact_coef_task for a 4x4 block whose pixel rows are 256 words apart (encode4w_kernel's LDS
// layout), one row per step of a loop left rolled: few registers live beside the caller's.
__device__ __forceinline__ int exact_coef_rows4(const double* P, double S, double rq, double qd, const uint32_t* pw) {
    double acc = 0.0;
#pragma unroll 1
    for (int w = 0; w < 4; w++) {
        const uint32_t px4 = pw[w * 256];
        double pr[4];
#pragma unroll
        for (int e = 0; e < 4; e++) pr[e] = P[4 * w + e];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const double x = double(int((px4 >> (8 * e)) & 0xFFu) - 128);  // == double(p) + (-128.0), exactly
            acc = acc + pr[e] * x;
        }
    }
    const double D = acc * S;
    const double t = (rq != 0.0) ? D * rq : D / qd;
    double r = trunc(t);
    if (fabs(t - r) >= 0.5) r += copysign(1.0, t);
    return int(r);
}

// exact_coef_task for an 8x8 block in encode_kernel<8>'s LDS pixel layout (row r = words
// r*128, r*128 + 1 from pw): the pixel words come from LDS one at a time (a register copy of the
// block indexed by the loop counter would live in scratch memory).
__device__ __forceinline__ int exact_coef_rows8(const double* P, double S, double rq, double qd, const uint32_t* pw) {
    double acc = 0.0;
#pragma unroll 2
    for (int w = 0; w < 16; w++) {
        const uint32_t px4 = pw[(w >> 1) * 128 + (w & 1)];
        double pr[4];
#pragma unroll
        for (int e = 0; e < 4; e++) pr[e] = P[4 * w + e];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const double x = double(int((px4 >> (8 * e)) & 0xFFu) - 128);  // == double(p) + (-128.0), exactly
            acc = acc + pr[e] * x;
        }
    }
    const double D = acc * S;
    const double t = (rq != 0.0) ? D * rq : D / qd;
    double r = trunc(t);
    if (fabs(t - r) >= 0.5) r += copysign(1.0, t);
    return int(r);
}

// Out-of-line copy for the EXACT mode's per-coefficient loop.
template <int N>
__device__ __noinline__ int exact_coef(const EncTables* __restrict__ tab, int k, BlockPx<N> px) {
    return exact_coef_inl<N>(tab, k, px);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Load the pixel rows of one group: seg[r][m] = bytes [4m, 4m+4) of the group's row r.
template <int N, int WPR, int BPT = Geo<N>::BPT>
__device__ __forceinline__ void load_group(const EncArgs& a, const uint8_t* base, int nblk, uint32_t (&seg)[N][WPR]) {
    if (a.vec_ok && nblk == BPT) {
#pragma unroll
        for (int r = 0; r < N; r++) {
            const uint8_t* p = base + size_t(r) * a.stride;
            if constexpr (WPR == 4) {
                const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
                seg[r][0] = v.x; seg[r][1] = v.y; seg[r][2] = v.z; seg[r][3] = v.w;
            } else if constexpr (WPR == 2) {
                const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
                seg[r][0] = v.x; seg[r][1] = v.y;
            } else {
                seg[r][0] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p));
            }
        }
    } else {
#pragma unroll
        for (int r = 0; r < N; r++) {
            const uint8_t* p = base + size_t(r) * a.stride;
#pragma unroll
            for (int m = 0; m < WPR; m++) {
                uint32_t wv = 0;
                if (m * 4 < nblk * N) {
#pragma unroll
                    for (int e = 0; e < 4; e++) wv |= uint32_t(p[m * 4 + e]) << (8 * e);
                }
                seg[r][m] = wv;
            }
        }
    }
}

template <int N> struct Packed {
    uint32_t w[N * N / 2];  // zig-zag order, two int16 per word: z[2j] in the low half
};

constexpr float kMagic = 12582912.0f;  // 1.5 * 2^23: t + kMagic rounds t (|t| < 2^22) to an integer

// The "structural" coefficients (0,N/2), (N/2,0), (N/2,N/2): their reference value is, up to
// FP64 rounding, a rational multiple of an integer pixel sum (every c[u][i]c[v][j] is +-1/2 or
// +-sqrt(1/2)), so their quotients land EXACTLY on rounding ties for 1/(4q) of all blocks, where
// only the reference's own FP64 rounding decides.  They are flagged per coefficient and
// re-evaluated alone; the other coefficients reach a tie only within the FP32 error bound.
template <int N> struct Structural {
    static constexpr int k[3] = {N / 2, (N / 2) * N, (N / 2) * N + N / 2};
    static constexpr int zpos(int s) { return ZigZagInv<N>::pos[k[s]]; }
};

// Round the FP32 quotients t[] to int16 (zig-zag packed).  y = t + 1.5*2^23 leaves
// int16(rint(t)) in y's low 16 bits and |t - (y - 1.5*2^23)| is the rounding residual.  Returns
// the largest residual of the ordinary (non-structural, non-exact) coefficients -- >= lim_ord means
// the block may hold a tie within the error bound -- and in *sflags bit s a possible tie of
// structural coefficient s.
template <int N>
__device__ __forceinline__ float round_block(const EncTables* __restrict__ tab, const float (&t)[N * N],
                                             uint32_t (&zp)[N * N / 2], uint32_t* sflags) {
    constexpr int NN = N * N;
    uint32_t yb[NN];
    float e[NN];
#pragma unroll
    for (int k = 0; k < NN; k++) {
        const float y = t[k] + kMagic;
        e[k] = fabsf(t[k] - (y - kMagic));
        yb[k] = __float_as_uint(y);
    }
    // t[0] exact (q[0] a power of two): std::round's half-away-from-zero directly
    const uint32_t dc = uint32_t(int(truncf(t[0] + copysignf(0.5f, t[0]))));
    const bool dcx = tab->dc_exact != 0;
    yb[0] = dcx ? dc : yb[0];
    float emax = dcx ? 0.0f : e[0];
#pragma unroll
    for (int k = 1; k < NN; k++) {
        if (k == Structural<N>::k[0] || k == Structural<N>::k[1] || k == Structural<N>::k[2]) continue;
        emax = fmaxf(emax, e[k]);
    }
    uint32_t sf = 0;
#pragma unroll
    for (int s = 0; s < 3; s++) sf |= (e[Structural<N>::k[s]] >= tab->lim[Structural<N>::k[s]]) ? (1u << s) : 0u;
    *sflags = sf;
#pragma unroll
    for (int j = 0; j < NN / 2; j++)
        zp[j] = __builtin_amdgcn_perm(yb[ZigZag<N>::idx[2 * j + 1]], yb[ZigZag<N>::idx[2 * j]], 0x05040100u);
    return emax;
}

// 8x8: round as above, but flag every coefficient on its own (bit k of the returned mask: its
// residual reaches lim[k]).  The fix-up then re-evaluates single coefficients and never
// recomputes a whole 8x8 block, whose 64 live quotients would spill next to the 32 packed words.
template <int N>
__device__ __forceinline__ uint64_t round_block_mask(const EncTables* __restrict__ tab, const float (&t)[N * N],
                                                     uint32_t (&zp)[N * N / 2]) {
    constexpr int NN = N * N;
    static_assert(NN <= 64, "one mask bit per coefficient");
    uint32_t yb[NN];
    uint64_t near = 0;
#pragma unroll
    for (int k = 0; k < NN; k++) {
        const float y = t[k] + kMagic;
        const float e = fabsf(t[k] - (y - kMagic));
        yb[k] = __float_as_uint(y);
        near |= uint64_t(e >= tab->lim[k]) << k;
    }
    if (tab->dc_exact) {
        yb[0] = uint32_t(int(truncf(t[0] + copysignf(0.5f, t[0]))));
        near &= ~1ull;
    }
#pragma unroll
    for (int j = 0; j < NN / 2; j++)
        zp[j] = __builtin_amdgcn_perm(yb[ZigZag<N>::idx[2 * j + 1]], yb[ZigZag<N>::idx[2 * j]], 0x05040100u);
    return near;
}

// round_block_mask for 8x8 with each zig-zag pair rounded and packed (and pinned) in turn: never
// 64 magic-added quotients live beside the 64 quotients.  Same results bit for bit.
__device__ __forceinline__ uint64_t round_block_mask_lean8(const EncTables* __restrict__ tab, const float (&t)[64],
                                                         uint32_t (&zp)[32]) {
    uint64_t near = 0;
    const bool dcx = tab->dc_exact != 0;
#pragma unroll
    for (int j = 0; j < 32; j++) {
        uint32_t yb[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int k = ZigZag<8>::idx[2 * j + h];
            const float y = t[k] + kMagic;
            const float e = fabsf(t[k] - (y - kMagic));
            yb[h] = __float_as_uint(y);
            if (k == 0) {
                yb[h] = dcx ? uint32_t(int(truncf(t[0] + copysignf(0.5f, t[0])))) : yb[h];
                near |= (!dcx && e >= tab->lim[0]) ? 1ull : 0ull;
            } else {
                near |= uint64_t(e >= tab->lim[k]) << k;
            }
        }
        zp[j] = __builtin_amdgcn_perm(yb[1], yb[0], 0x05040100u);
        asm volatile("" : "+v"(zp[j]));
    }
    return near;
}

template <int N, int WPR>
__device__ __forceinline__ void block_pixels(const uint32_t (&seg)[N][WPR], int b, float (&x)[N * N]) {
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
        for (int j = 0; j < N; j++) x[i * N + j] = float(pix<WPR>(seg[i], b * N + j));
}

template <int N>
__device__ __forceinline__ void quotients(const EncTables* __restrict__ tab, float (&x)[N * N]) {
    if constexpr (N == 4) quot4(x, tab->plan4, FloatOp());
    else quot8(x, tab->dct, tab->g, FloatOp());
}

// The FP64 fix-up of one flagged block, all in line (a call would make the caller spill its
// live coefficient registers around it): the same FP32 quotients rounded into the task's LDS
// result slot, then every coefficient whose residual reaches its own lim[k] re-evaluated in the
// reference's FP64 order and patched in place (a runtime position: LDS, not a register array).
template <int N>
__device__ __forceinline__ void fix_block(const EncTables* __restrict__ tab, const BlockPx<N>& px, uint32_t* res) {
    constexpr int NN = N * N;
    float x[NN];
#pragma unroll
    for (int k = 0; k < NN; k++) x[k] = float((px.w[k >> 2] >> (8 * (k & 3))) & 0xFFu);
    quotients<N>(tab, x);
    uint32_t yb[NN];
    uint64_t near = 0;
#pragma unroll
    for (int k = 0; k < NN; k++) {
        const float y = x[k] + kMagic;
        const float e = fabsf(x[k] - (y - kMagic));
        yb[k] = __float_as_uint(y);
        if (k == 0 && tab->dc_exact) yb[0] = uint32_t(int(truncf(x[0] + copysignf(0.5f, x[0]))));
        else near |= uint64_t(e >= tab->lim[k]) << k;
    }
#pragma unroll
    for (int j = 0; j < NN / 2; j++)
        res[j] = __builtin_amdgcn_perm(yb[ZigZag<N>::idx[2 * j + 1]], yb[ZigZag<N>::idx[2 * j]], 0x05040100u);
    while (near) {
        const int k = __ffsll((unsigned long long)near) - 1;
        near &= near - 1;
        const int kz = ZigZagInv<N>::pos[k];
        const uint32_t v = uint32_t(exact_coef_inl<N>(tab, k, px)) & 0xFFFFu;
        const uint32_t w = res[kz >> 1];  // same-type read-modify-write (no uint16 aliasing)
        res[kz >> 1] = (kz & 1) ? ((w & 0xFFFFu) | (v << 16)) : ((w & 0xFFFF0000u) | v);
    }
}

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Packed int16 helpers (the compiler otherwise splits them into per-half compares).
// (Constants go in a register: an inline constant of a packed op feeds the low half only.)
__device__ __forceinline__ uint32_t pk_min1_u16(uint32_t w) {  // per half: min(h, 1) = (h != 0)
    uint32_t r;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(w), "s"(0x00010001u));
    return r;
}
__device__ __forceinline__ uint32_t pk_sign_i16(uint32_t w) {  // per half: h >> 15 (arithmetic)
    uint32_t r;
    asm("v_pk_ashrrev_i16 %0, %1, %2" : "=v"(r) : "s"(0x000F000Fu), "v"(w));
    return r;
}

// Zig-zag RLE sizing of one packed block (Block.cpp:186-232, :383-397), two coefficients per
// packed-int16 instruction.  Returns bl | Lw << 8 and the record length in bits.  In the RLE
// truncation case (L == N*N, z[N*N-2] == 0: the reference drops the last coefficient,
// Block.cpp:388-390) z[N*N-1] is cleared, so every coefficient at or past Lw is zero.
// 4x4 form with 32-bit masks throughout (the 64-bit nz mask cost 64-bit compares and moves), the
// pair masks merged by shift-or and the widest value by one three-input op per word.
__device__ __forceinline__ uint32_t size_block4(uint32_t (&zp)[8], int rle, uint32_t* bits) {
    uint32_t M = 0, mo = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t w = zp[j];
        M = (pk_min1_u16(w) << (2 * j)) | M;  // v_lshl_or_b32
        mo = (w ^ pk_sign_i16(w)) | mo;  // one v_bitop3 (the compiler's table: a hand-written one had the operands swapped)
    }
    const uint32_t nz = (M & 0x5555u) | ((M >> 15) & 0xAAAAu);  // bit kz: z[kz] != 0
    mo = (mo | (mo >> 16)) & 0xFFFFu;
    const int maxb = 33 - __clz(mo);
    const int L = 32 - __clz(nz);                       // 0 for nz == 0
    const int ffsL = L ? 32 - __clz(uint32_t(L)) : 1;  // utils.hpp:210-216, with ffs(0) == 1
    const int bl = max(maxb, ffsL);
    int lw;
    if (!rle) {
        lw = 16;
    } else if (L == 16 && !((nz >> 14) & 1u)) {
        lw = 32 - __clz(nz & 0x7FFFu);  // drop the last element (Block.cpp:388-390)
        zp[7] &= 0xFFFFu;
    } else {
        lw = L;
    }
    *bits = __umul24(uint32_t(bl), uint32_t(lw + rle)) + 4u;
    return uint32_t(bl) | (uint32_t(lw) << 8);
}

template <int N>
__device__ __forceinline__ uint32_t size_block(uint32_t (&zp)[N * N / 2], int rle, uint32_t* bits) {
    constexpr int NN = N * N;
    constexpr int NP = NN / 2;
    uint64_t nz = 0;  // bit kz set iff z[kz] != 0
    uint32_t mo = 0;  // OR of v ^ (v >> 15) per half: its bit length + 1 is the widest bits_needed
#pragma unroll
    for (int g = 0; g < NP / 8; g++) {
        uint32_t M = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t w = zp[g * 8 + j];
            M |= pk_min1_u16(w) << (2 * j);
            mo |= w ^ pk_sign_i16(w);  // one v_bitop3
        }
        const uint32_t nz16 = (M & 0x5555u) | ((M >> 15) & 0xAAAAu);
        nz |= uint64_t(nz16) << (16 * g);
    }
    mo = (mo | (mo >> 16)) & 0xFFFFu;
    const int maxb = 33 - __clz(mo);  // bits_needed (utils.hpp:226-243) of the widest value
    const int L = nz ? 64 - __clzll((long long)nz) : 0;
    const int ffsL = L ? 32 - __clz(L) : 1;  // utils.hpp:210-216, with ffs(0) == 1
    const int bl = max(maxb, ffsL);
    int lw;
    if (!rle) {
        lw = NN;
    } else if (L == NN && !((nz >> (NN - 2)) & 1ull)) {
        const uint64_t m = nz & ((1ull << (NN - 1)) - 1);  // drop the last element (Block.cpp:388-390)
        lw = m ? 64 - __clzll((long long)m) : 0;
        zp[NP - 1] &= 0xFFFFu;
    } else {
        lw = L;
    }
    *bits = __umul24(uint32_t(bl), uint32_t(lw + rle)) + 4u;  // (a 64-bit v_mad otherwise)
    return uint32_t(bl) | (uint32_t(lw) << 8);
}

// OR the low `len` bits of v (MSB first) into the LDS bit image at bit p (len + p%32 <= 64).
__device__ __forceinline__ void scatter_bits(uint32_t* img, uint32_t p, uint32_t v, uint32_t len) {
    // The image is the dynamic LDS area at LDS byte address 0 (the encode kernels allocate no static
    // LDS; tools/asmcheck.py checks their group_segment_fixed_size): the word pair's byte address
    // straight from p, the second word through the instruction's offset field.  The field is
    // left-aligned once, then funnel-shifted into the pair (-2.7 % against a 64-bit shift).
    (void)img;
    const uint32_t a = (p >> 3) & ~3u;
    const uint32_t s = p & 31u;
    const uint32_t u = v << (32u - len);  // the field left-aligned (len <= 32)
    const uint32_t hi = u >> s;
    const uint32_t lo = __builtin_amdgcn_alignbit(u, 0u, s);  // u << (32 - s), 0 for s = 0
    // (two ds_or_b32, never one ds_or_b64: the address is only 4-byte aligned, and a 64-bit LDS
    // atomic there raises a memory violation -- tools/asmcheck.py rejects 64-bit DS atomics)
    asm volatile("ds_or_b32 %0, %1\n\tds_or_b32 %0, %2 offset:4" ::"v"(a), "v"(hi), "v"(lo) : "memory");
}

// Branch-free variant: every pair is written (past Lw the packed coefficients are zero, so
// those ORs are no-ops) and the wave leaves the loop once no lane has a pair left: no per-lane
// exec-mask juggling per pair.  The zero pairs may land up to 2 * 16 * N*N/2 bits past the
// record: the image keeps that much slack.
template <int N>
__device__ __forceinline__ void emit_block2(uint32_t* img, uint32_t p, const uint32_t (&zp)[N * N / 2], uint32_t blw,
                                            int rle) {
    const uint32_t bl = blw & 0xFFu, lw = blw >> 8;
    if (rle) {
        scatter_bits(img, p, ((bl & 0xFu) << bl) | lw, 4u + bl);
        p += 4u + bl;
    } else {
        scatter_bits(img, p, bl & 0xFu, 4u);
        p += 4u;
    }
    const uint32_t m = (1u << bl) - 1u;
#pragma unroll
    for (int j = 0; j < N * N / 2; j++) {
        if (j > 0 && !__ballot(uint32_t(2 * j) < lw)) break;  // no lane has pair j
        const uint32_t v = ((zp[j] & m) << bl) | __builtin_amdgcn_ubfe(zp[j], 16u, bl);
        scatter_bits(img, p, v, 2u * bl);
        p += 2u * bl;
    }
}

// Every triple is ORed in, without a wave-wide "any lane still has one" exit per field (past Lw
// the coefficients are zero): the v_cmp + branch per field cost more than the skipped fields save
// unless every lane of the wave has a short record (measured -2 % on C2).
// 4x4 RLE records when every bl of the matrix is <= 10 (EncArgs::tri: the host's launch_chain
// sets it when (rec_bits - 4) / 17 <= 10): the header, Lw and z0 in one field of 4 + 2*bl <= 24
// bits, then the coefficients THREE at a time (3*bl <= 30 bits: the field is built in a 32-bit
// v), each ORed through scatter_bits' 64-bit window: 6 fields per block instead of 9.  Past Lw
// the packed coefficients are zero, so a trailing triple only ORs zeros.
__device__ __forceinline__ void emit_block3(uint32_t* img, uint32_t p, const uint32_t (&zp)[8], uint32_t blw) {
    const uint32_t bl = blw & 0xFFu, lw = blw >> 8;
    auto z = [&](int k) -> uint32_t {  // low bl bits of zig-zag coefficient k
        return __builtin_amdgcn_ubfe(zp[k >> 1], (k & 1) ? 16u : 0u, bl);
    };
    scatter_bits(img, p, ((((bl & 0xFu) << bl) | lw) << bl) | z(0), 4u + 2u * bl);
    p += 4u + 2u * bl;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t v = (((z(3 * j + 1) << bl) | z(3 * j + 2)) << bl) | z(3 * j + 3);
        scatter_bits(img, p, v, 3u * bl);
        p += 3u * bl;
    }
}

// Where tile t sits: its chain (frame / whole batch), its position in it and this thread's
// group of blocks.
struct TileGeo {
    int frame, tif, step, chain_pos;
    int nblk, byi, bx0;  // blocks of this thread's group (nblk = 0: none)
};

template <int N, int BPT = Geo<N>::BPT, int TG = kEncTPB, class Args = EncArgs>
__device__ __forceinline__ TileGeo tile_geo(const Args& a, int t, int tid) {
    TileGeo g;
    // Independent images interleave their tiles (frame = t % nframes), so every frame's chain
    // advances together; a concatenated stream keeps chain order = tile order.
    // (wave-uniform divisions by launch constants: multiply-highs, FastDiv)
    if (a.segmented) {
        g.tif = int(fdiv(uint32_t(t), a.div_frames.mul, a.div_frames.shr));
        g.frame = t - g.tif * a.nframes;
        g.step = a.nframes;
    } else {
        g.frame = int(fdiv(uint32_t(t), a.div_tpf.mul, a.div_tpf.shr));
        g.tif = t - g.frame * a.tiles_per_frame;
        g.step = 1;
    }
    g.chain_pos = a.segmented ? g.tif : t;  // tiles before this one in its chain
    // group gi = base + tid: the division by gpr is split into a wave-uniform (scalar) part and a
    // per-lane remainder r < gpr + kEncTPB, divided by a multiply-high with ceil(2^32 / gpr)
    const int base = g.tif * TG;  // (TG groups per tile; tid: the thread's group within it)
    const int q0 = int(fdiv(uint32_t(base), a.div_gpr.mul, a.div_gpr.shr)), r0 = base - q0 * a.gpr;
    const uint32_t r = uint32_t(r0 + tid);
    const uint32_t dq = (a.gpr == 1) ? r : __umulhi(r, a.gpr_magic);  // (2^32 does not fit the magic)
    const int gi = base + tid;
    g.nblk = g.byi = g.bx0 = 0;
    if (gi < a.groups_per_frame) {
        g.byi = q0 + int(dq);
        g.bx0 = int(r - dq * uint32_t(a.gpr)) * BPT;
        g.nblk = min(BPT, a.bx - g.bx0);
    }
    return g;
}

// The launch fields a tile's geometry and pixel loads need (EncArgs' first 27 words), read from
// the kernel-argument segment in ONE scalar round trip (two s_load_dwordx16).  Read field by field,
// the compiler sinks each load into the branch that uses it: a chain of ~6 dependent round trips
// (≈1.1 µs under load, measured by stamps) before a tile's first pixel load and again at its start.
struct GeoArgs {
    const uint8_t* y;
    uint64_t stride, frame_pitch;
    int nframes, bx, by, gpr;
    uint32_t gpr_magic;
    int groups_per_frame, tiles_per_frame, ntiles;
    FastDiv div_frames, div_tpf, div_gpr;
    int segmented;
};
template <class KA>
__device__ __forceinline__ GeoArgs load_geo(KA* ka) {
    typedef uint32_t u16v __attribute__((ext_vector_type(16)));
    using P = const __attribute__((address_space(4))) u16v;
    u16v A = ((P*)ka)[0], B = ((P*)ka)[1];
    asm volatile("" : "+s"(A), "+s"(B));  // both loaded here, before any use
    auto w = [&](size_t off) -> uint32_t { return off < 64 ? A[off / 4] : B[off / 4 - 16]; };
    auto d = [&](size_t off) -> uint64_t { return uint64_t(w(off)) | (uint64_t(w(off + 4)) << 32); };
    auto fd = [&](size_t off) { return FastDiv{w(off), w(off + 4), w(off + 8)}; };
    static_assert(offsetof(EncArgs, segmented) + 4 <= 128, "geometry fields in the first 128 bytes");
    GeoArgs g;
    g.y = reinterpret_cast<const uint8_t*>(d(offsetof(EncArgs, y)));
    g.stride = d(offsetof(EncArgs, stride));
    g.frame_pitch = d(offsetof(EncArgs, frame_pitch));
    g.nframes = int(w(offsetof(EncArgs, nframes)));
    g.bx = int(w(offsetof(EncArgs, bx)));
    g.by = int(w(offsetof(EncArgs, by)));
    g.gpr = int(w(offsetof(EncArgs, gpr)));
    g.gpr_magic = w(offsetof(EncArgs, gpr_magic));
    g.groups_per_frame = int(w(offsetof(EncArgs, groups_per_frame)));
    g.tiles_per_frame = int(w(offsetof(EncArgs, tiles_per_frame)));
    g.ntiles = int(w(offsetof(EncArgs, ntiles)));
    g.div_frames = fd(offsetof(EncArgs, div_frames));
    g.div_tpf = fd(offsetof(EncArgs, div_tpf));
    g.div_gpr = fd(offsetof(EncArgs, div_gpr));
    g.segmented = int(w(offsetof(EncArgs, segmented)));
    return g;
}

template <int N, int WPR, int BPT = Geo<N>::BPT>
__device__ __forceinline__ void load_tile(const EncArgs& a, const TileGeo& g, uint32_t (&seg)[N][WPR]) {
    if (g.nblk) {
        const uint8_t* base =
            a.y + size_t(g.frame) * a.frame_pitch + size_t(g.byi) * N * a.stride + size_t(g.bx0) * N;
        load_group<N, WPR, BPT>(a, base, g.nblk, seg);
    } else {
#pragma unroll
        for (int r = 0; r < N; r++)
#pragma unroll
            for (int m = 0; m < WPR; m++) seg[r][m] = 0;
    }
}

// Profiling stamps (IE_STAMPS): thread 0's s_memtime at the phase boundaries of each tile.
#define STAMP(i)                                                                                  \
    do {                                                                                          \
        if (stamps && tid == 0) stamps[size_t(t) * kStamps + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)

// Occupancy hint: __launch_bounds__'s second argument (Geo<N>::WAVES; stating it as
// amdgpu_waves_per_eu instead measured slower).
// The EXACT 4x4 kernel (FP64 for every coefficient) keeps four waves per SIMD.
template <int N, bool EXACT> constexpr int enc_waves() { return (N == 4 && EXACT) ? 4 : Geo<N>::WAVES; }
#define IE_ENC_BOUNDS(N, EXACT) __launch_bounds__(kEncTPB, (enc_waves<N, EXACT>()))
// HIST: count the stored bytes into a per-tile LDS histogram (256 words after the misc area),
// merged into a.hist[frame] at the end: the Huffman pass's histogram without re-reading the stream.
// R > 1: R copies of each bin, bin b of lane l at b * R + l % R (the same byte in several lanes of
// one ds_add no longer serialises on one address)
template <int R = 1>
struct HistCountT {
    uint32_t* hl;
    uint64_t limit;  // bytes at stream positions >= limit are padding (the chain's last word)
    uint32_t lo = 0;  // l % R
    __device__ __forceinline__ void add(uint32_t b) const { atomicAdd(&hl[b * R + lo], 1u); }
    __device__ __forceinline__ void operator()(uint64_t gw, uint32_t v) const {
        if (limit == ~0ull) {  // (wave-uniform) not the chain's last tile: every byte counts
#pragma unroll
            for (int k = 0; k < 4; k++) add((v >> (8 * k)) & 0xFFu);
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (4 * gw + k < limit) add((v >> (8 * k)) & 0xFFu);
        }
    }
};
using HistCount = HistCountT<1>;

// BB: blocks per thread (4x4: 4; the LDS pixel layout also takes 1 -- measured on one 4K frame,
// 2 025 tiles of one block per lane took 36 us against 20 us for 506 tiles of four: the longer
// look-back chain costs more than the shorter tiles save)
template <int N, bool EXACT, bool HIST = false, int BB = Geo<N>::BPT>
__global__ IE_ENC_BOUNDS(N, EXACT) void encode_kernel(EncArgs a, const EncTables* __restrict__ tab) {
    constexpr int NN = N * N;
    constexpr int NP = NN / 2;
    constexpr int BPT = BB;
    constexpr int WPR = BPT * N / 4;
    constexpr int TPB = kEncTPB;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];  // [a.img_words + 32]
    // Dynamic LDS: [tile image: img_words][misc: 32 words][HIST: 256 words][srow]; the image at
    // LDS address 0, so its addresses need no base.
    uint32_t* img = smem;
    uint32_t* misc = smem + a.img_words;  // [0..15] scan scratch (one word per wave)
    uint32_t* ctl = misc + 16;     // [4] ticket, [5..6] exclusive prefix, [7] predecessor tail
    // FAST mode: the structural coefficients' FP64 rows (P[3][NN], then S[3], rq[3], qd[3])
    double* const srow = reinterpret_cast<double*>(misc + 32 + (HIST ? 256 : 0));
    // 4x4 FAST: all NN rows of P, then S, rq, qd of every coefficient (kRowDoubles); 8x8: the three
    // structural rows, then their S, rq, qd (3 * NN + 9)
    constexpr bool kFullRows = N == 4 && !EXACT;
    constexpr int kRowDoubles = kFullRows ? NN * NN + 3 * NN : 3 * NN + 9;
    // row / S / rq / qd of structural coefficient s (kFullRows: of coefficient k = s)
    auto rowP = [&](int k) -> const double* { return kFullRows ? srow + k * NN : srow + k * NN; };
    auto rowS = [&](int k) { return kFullRows ? srow[NN * NN + k] : srow[3 * NN + k]; };
    auto rowRq = [&](int k) { return kFullRows ? srow[NN * NN + NN + k] : srow[3 * NN + 3 + k]; };
    auto rowQd = [&](int k) { return kFullRows ? srow[NN * NN + 2 * NN + k] : srow[3 * NN + 6 + k]; };
    (void)kRowDoubles;

    const int tid = threadIdx.x;
    // Profiling hooks (IE_ABLATE / IE_STAMPS) exist only in IE_PROFILE builds (tools/variants.sh):
    // in the product build they are constants, so they hold no scalar registers.  (Round 3 kept them
    // live in the 8x8 kernel to dodge a spill; with its pixels in LDS and the fix-up reading them
    // from there the 8x8 kernel has no scratch without that.)
    constexpr bool kProf = IE_PROFILE != 0;
    const int ablate = kProf ? a.ablate : 0;
    uint64_t* const stamps = kProf ? a.stamps : nullptr;
    // Tile order = dispatch order.  Workgroups are dispatched in increasing blockIdx, so every
    // chain predecessor of a resident tile is resident or done and the look-back cannot
    // deadlock; the bounded spins report (never hang) should that ever not hold, and the host
    // then re-runs with an atomic ticket (a.ticket != nullptr), which orders tiles explicitly.
    int t;
    if (a.ticket) {
        if (tid == 0) ctl[4] = uint32_t(atomicAdd(a.ticket, 1ull) - a.ticket_base);
        lds_barrier();
        t = __builtin_amdgcn_readfirstlane(int(ctl[4]));  // uniform: tile geometry stays in SGPRs
        if (t >= a.ntiles) return;  // ticket desync (a failed earlier launch): never touch memory
    } else {
        t = int(blockIdx.x);
    }
    STAMP(0);
    uint32_t* const hl = misc + 32;  // HIST: the tile's byte histogram
    if constexpr (HIST)
        for (int i = tid; i < 256; i += TPB) hl[i] = 0u;  // (visible after the scan's barriers)
    if constexpr (kFullRows) {
        // 4x4: every coefficient's FP64 row P[k][*] and its S, rq, qd (304 doubles): the fix-up's
        // structural AND whole-block evaluations read them from LDS, never from global memory
        for (int i = tid; i < kRowDoubles; i += TPB)
            srow[i] = (i < NN * NN) ? tab->P[i] : (i < NN * NN + NN) ? tab->S[i - NN * NN]
                    : (i < NN * NN + 2 * NN) ? tab->rq[i - NN * NN - NN] : tab->qd[i - NN * NN - 2 * NN];
    } else if constexpr (!EXACT) {
        // issued before the pixel loads, so waiting for it does not wait for them
        for (int i = tid; i < 3 * NN + 9; i += TPB) srow[i] = tab->srow[i];
    }
    const TileGeo g = tile_geo<N, BPT>(a, t, tid);
    // the chain's first bit: the host's value, or (streamed video, ie_vstream_*) the previous
    // launch's chain end on the device, written before this launch started (stream order)
    const uint64_t start_bit = a.start_dev ? *a.start_dev : a.start_bit;
    const int frame = g.frame, tif = g.tif, step = g.step, chain_pos = g.chain_pos;
    const int nblk = g.nblk, byi = g.byi, bx0 = g.bx0;
    constexpr bool kLdsPix = N == 4 && !EXACT;
    // 8x8 FAST: the pixels in LDS too, [8 rows][64 lanes][2 words] per wave (block row r of lane l
    // = words r*128 + 2l, 2l+1): no pixel registers live through the transform and the fix-up
    constexpr bool kLdsPix8 = N == 8 && !EXACT;
    // kLdsPix: this wave's [4 rows][64 lanes][BPT] words; block b of a lane = word b of each row
    constexpr int kRowW = (N == 8) ? 128 : 64 * BPT;
    uint32_t* const pwave = img + kFixPix + (tid >> 6) * (N * kRowW);
    const int lane = tid & 63;
    uint32_t seg[N][WPR];
    if constexpr (kLdsPix8) {
        // DMA when the wave's blocks pair up within rows (even bx): lanes 0-31 fetch row r, lanes
        // 32-63 row r+1, 16 bytes = the row pieces of blocks 2c, 2c+1 (c = lane & 31) each
        const int wfirst = tif * TPB + (tid & ~63);                          // the wave's first block
        const int nwb = min(64, max(0, a.groups_per_frame - wfirst));        // its blocks in this frame
        if (a.vec_ok && !(a.bx & 1) && nwb > 0) {
            const int c = lane & 31, half = lane >> 5;
            const int bi = wfirst + 2 * c;                                    // block of this lane's piece
            const bool live = 2 * c < nwb;
            const int by_ = bi / a.bx, bx_ = bi - by_ * a.bx;
            const uint8_t* src = a.y + size_t(frame) * a.frame_pitch + size_t(by_) * N * a.stride + size_t(bx_) * N;
#pragma unroll
            for (int r = 0; r < N; r += 2)
                if (live)
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + size_t(r + half) * a.stride),
                                                     (__attribute__((address_space(3))) void*)(pwave + r * kRowW), 16, 0, IE_PX_AUX8);
        } else {  // odd bx / unaligned rows: through registers
            load_tile<N, WPR, BPT>(a, g, seg);
#pragma unroll
            for (int r = 0; r < N; r++) {
                u32x2 v;
                v.x = seg[r][0];
                v.y = seg[r][1];
                *reinterpret_cast<u32x2*>(pwave + r * kRowW + 2 * lane) = v;
            }
        }
    } else if constexpr (kLdsPix) {
        static_assert((BPT == 4 || BPT == 1) && WPR == BPT && TPB % 64 == 0, "LDS pixel layout: 4 * BPT bytes per lane per row");
        if (ablate & 4096) {
            // profiling: no pixel loads at all (the LDS holds whatever the previous tile left)
        } else if (!__ballot(!(a.vec_ok && nblk == BPT))) {  // every group of the wave is whole: DMA
            const uint8_t* base =
                a.y + size_t(frame) * a.frame_pitch + size_t(byi) * N * a.stride + size_t(bx0) * N;
#pragma unroll
            for (int r = 0; r < N; r++)
                if constexpr (BPT == 4)
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + size_t(r) * a.stride),
                                                     (__attribute__((address_space(3))) void*)(pwave + r * kRowW), 16, 0, 0);
                else
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + size_t(r) * a.stride),
                                                     (__attribute__((address_space(3))) void*)(pwave + r * kRowW), 4, 0, 0);
        } else {  // ragged (frame edge, unaligned rows): through registers
            load_tile<N, WPR, BPT>(a, g, seg);
#pragma unroll
            for (int r = 0; r < N; r++) {
                if constexpr (BPT == 4) {
                    u32x4 v;
                    v.x = seg[r][0]; v.y = seg[r][1]; v.z = seg[r][2]; v.w = seg[r][3];
                    *reinterpret_cast<u32x4*>(pwave + r * kRowW + lane * 4) = v;
                } else {
                    pwave[r * kRowW + lane] = seg[r][0];
                }
            }
        }
    } else if (ablate & 128) {  // profiling: no pixel loads (synthetic pixels from the thread id)
#pragma unroll
        for (int r = 0; r < N; r++)
#pragma unroll
            for (int m = 0; m < WPR; m++) seg[r][m] = (uint32_t(tid) * 0x9E3779B1u + uint32_t(t) * 0x85EBCA77u) ^ (r * 0x27D4EB2Fu + m);
    } else {
        load_tile<N, WPR, BPT>(a, g, seg);
    }
    if constexpr (!EXACT) lds_barrier();  // srow visible (the pixel loads stay in flight)
    if constexpr (kLdsPix || kLdsPix8) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pixels landed

    asm volatile("; PHASE load_done" ::: "memory");
    if (ablate & 512) return;  // profiling: instruction count of the prologue + load alone
    if (stamps) {  // profiling: wait for the pixels so the stamp marks their arrival
        uint32_t acc = 0;
#pragma unroll
        for (int r = 0; r < N; r++)
#pragma unroll
            for (int m = 0; m < WPR; m++) acc ^= seg[r][m];
        if (acc == 0x9E3779B9u) a.err[1] = acc;
    }
    STAMP(2);
    // ---------------------------------------------------------------- 1. transform + quantise
    uint32_t zp[BPT][NP];
    // fix-up requests, 4 bits per block: bits 0-2 structural coefficient s, bit 3 the whole block
    uint32_t flags = 0;
    uint64_t near8 = 0;  // 8x8: per-coefficient requests of the lane's one block
    uint32_t pix_next[N];  // the odd block's rows, read with the even block's
    (void)pix_next;
#pragma unroll
    for (int b = 0; b < BPT; b++) {
#if !IE_NO_SCHED_BARRIER
        __builtin_amdgcn_sched_barrier(0);  // one block at a time: keeps the live set small
#endif
        if constexpr (EXACT) {
            BlockPx<N> px;
#pragma unroll
            for (int i = 0; i < N; i++)
#pragma unroll
                for (int m = 0; m < N / 4; m++) px.w[i * (N / 4) + m] = seg[i][(b * N) / 4 + m];
            uint32_t yb[NN];
            for (int k = 0; k < NN; k++) yb[k] = uint32_t(exact_coef<N>(tab, k, px));
#pragma unroll
            for (int j = 0; j < NP; j++)
                zp[b][j] = __builtin_amdgcn_perm(yb[ZigZag<N>::idx[2 * j + 1]], yb[ZigZag<N>::idx[2 * j]], 0x05040100u);
        } else {
            float x[NN];
            if constexpr (kLdsPix8) {
                uint32_t rows[N][2];
#pragma unroll
                for (int r = 0; r < N; r++) {
                    const u32x2 v = *reinterpret_cast<const u32x2*>(pwave + r * kRowW + 2 * lane);
                    rows[r][0] = v.x;
                    rows[r][1] = v.y;
                }
                block_pixels<N, 2>(rows, 0, x);
            } else if constexpr (kLdsPix) {
                uint32_t rows[N][1];
                // two blocks' rows per 8-byte read (2-way instead of 4-way bank conflicts: -0.6 %)
                if constexpr (BPT % 2 == 0) {
                    if (b % 2 == 0) {
#pragma unroll
                        for (int r = 0; r < N; r++) {
                            const u32x2 v = *reinterpret_cast<const u32x2*>(pwave + r * kRowW + lane * BPT + b);
                            rows[r][0] = v.x;
                            pix_next[r] = v.y;
                        }
                    } else {
#pragma unroll
                        for (int r = 0; r < N; r++) rows[r][0] = pix_next[r];
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < N; r++) rows[r][0] = pwave[r * kRowW + lane * BPT + b];
                }
                block_pixels<N, 1>(rows, 0, x);
            } else {
                block_pixels<N, WPR>(seg, b, x);
            }
            if (!(ablate & 16)) quotients<N>(tab, x);
            if constexpr (N == 8) {
                static_assert(BPT == 1, "8x8: one block per lane");
                near8 = round_block_mask<N>(tab, x, zp[b]);
                if (b >= nblk || (ablate & 1)) near8 = 0;
#pragma unroll
                for (int j = 0; j < NP; j++) asm volatile("" : "+v"(zp[b][j]));  // packed here, not at first use
                continue;
            }
            uint32_t sf;
            const float emax = round_block<N>(tab, x, zp[b], &sf);
            uint32_t fb = (emax >= tab->lim_min) ? 8u : sf;  // a whole-block fix covers s
            if (ablate & 32) fb &= 7u;   // profiling: drop whole-block fixes
            if (ablate & 64) fb &= 8u;   // profiling: drop structural fixes
            if (b < nblk && !(ablate & 1)) flags |= fb << (4 * b);
        }
    }
    asm volatile("; PHASE quant_done" ::: "memory");
    if (ablate & 1024) {  // profiling: ... + transform + rounding (keep the results live)
        uint32_t acc = flags;
#pragma unroll
        for (int b = 0; b < BPT; b++)
#pragma unroll
            for (int j = 0; j < NP; j++) acc ^= zp[b][j];
        if (acc == 0x9E3779B9u) a.err[1] = acc;
        return;
    }
    STAMP(3);

    // ---------------------------------------------------------------- 1b. FP64 fix-up
    // Requests compacted per wave into an LDS task list, evaluated one per lane in the
    // reference's FP64 order, patched back by their owners (below: 8x8, then 4x4).
    if constexpr (!EXACT && N == 8) {
        // 8x8: one task per flagged coefficient, compacted per wave as for 4x4: the lane's block
        // (16 words) goes to an LDS slot, lane i evaluates task i in FP64 -- the structural
        // coefficients' rows from the LDS copy, any other row from the (L2-resident) table --
        // and the owners patch their results in.
        const unsigned nfix = unsigned(__popcll(near8));
        if (__ballot(near8 != 0)) {
            const uint32_t cnt = nfix;
            uint32_t pre = 0, total = 0;
#pragma unroll
            for (int k = 0; k < 7; k++) {  // cnt <= 64
                const uint64_t bm = __ballot((cnt >> k) & 1u);
                pre += __builtin_amdgcn_mbcnt_hi(uint32_t(bm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(bm), 0u)) << k;
                total += uint32_t(__popcll(bm)) << k;
            }
            uint32_t* task = img + kFix8Tasks + (tid >> 6) * 128;  // [64] tasks, then [64] results
            uint32_t* res = task + 64;
            for (uint32_t r0 = 0; r0 < total; r0 += 64) {
                uint64_t m = near8;
                uint32_t i = pre - r0;
                while (m) {
                    const int k = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    if (i < 64u) task[i] = (uint32_t(tid) << 6) | uint32_t(k);
                    i++;
                }
                wave_sync();
                const bool busy = uint32_t(lane) < total - r0;
                const uint32_t tk = busy ? task[lane] : 0u;
                const int k = int(tk & 63u), owner = int(tk >> 6);
                const int s = (k == Structural<N>::k[0]) ? 0 : (k == Structural<N>::k[1]) ? 1
                            : (k == Structural<N>::k[2]) ? 2 : -1;
                // Structural rows come from the LDS copy; any other task's row (rare) is staged
                // through LDS by the whole wave first, kNsStage rows per pass (one coalesced row
                // per load), so no dependent add of the FP64 chain waits on global memory.
                uint64_t ns = __ballot(busy && s < 0);
                bool done = !busy;
                double* stage = reinterpret_cast<double*>(img + kFix8Stage) + (tid >> 6) * (kNsStage * NN);
                do {
                    int slot = -1;
                    for (int r = 0; r < kNsStage && ns; r++) {
                        const int L = __ffsll((unsigned long long)ns) - 1;
                        ns &= ns - 1;
                        const int kr = __builtin_amdgcn_readlane(k, L);
                        stage[r * NN + lane] = tab->P[kr * NN + lane];  // NN = 64 = one double per lane
                        if (lane == L) slot = r;
                    }
                    wave_sync();
                    if (!done && (s >= 0 || slot >= 0)) {
                        const double* P = (s >= 0) ? srow + s * NN : stage + slot * NN;
                        const double S = (s >= 0) ? srow[3 * NN + s] : tab->S[k];
                        const double rq = (s >= 0) ? srow[3 * NN + 3 + s] : tab->rq[k];
                        const double qd = (s >= 0) ? srow[3 * NN + 6 + s] : tab->qd[k];
                        res[lane] = uint32_t(exact_coef_rows8(P, S, rq, qd, pwave + 2 * (owner & 63))) & 0xFFFFu;
                        done = true;
                    }
                    wave_sync();  // the next pass rewrites the staged rows
                } while (ns);
                wave_sync();
                m = near8;
                i = pre - r0;
                while (m) {
                    const int k = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    if (i < 64u) {
                        const uint32_t v = res[i];
                        const int kz = ZigZagInv<N>::pos[k];
#pragma unroll
                        for (int j = 0; j < NP; j++)
                            if ((kz >> 1) == j)
                                zp[0][j] = (kz & 1) ? ((zp[0][j] & 0xFFFFu) | (v << 16)) : ((zp[0][j] & 0xFFFF0000u) | v);
                    }
                    i++;
                }
                wave_sync();  // the next round rewrites the task list
            }
        }
        const unsigned wsum = unsigned(wave_sum64(nfix));
        if ((tid & 63) == 0) a.wave_fix[size_t(t) * (TPB / 64) + (tid >> 6)] = wsum;
    } else if constexpr (!EXACT) {
        // Structural requests, compacted per wave: the wave's pixels go to LDS (so the pixel
        // registers die here), every request gets a task number (a 4-plane ballot prefix), lane i
        // evaluates task i in FP64 and the owners patch their results in.  One FP64 evaluation
        // per 64 requests instead of one per lane per request.
        if (__ballot(flags != 0)) {
            // the pixels of block b of thread `owner` (of this wave): the tile's LDS pixel layout
            auto block_px = [&](int b, int owner) {
                BlockPx<N> px;
#pragma unroll
                for (int r = 0; r < N; r++) px.w[r] = pwave[r * kRowW + (owner & 63) * BPT + b];
                return px;
            };
            const uint32_t sf = flags & (0x77777777u >> (32 - 4 * BPT));
            const uint32_t cnt = __popc(sf);
            uint32_t pre = 0, total = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {  // cnt <= 3 * BPT <= 12
                const uint64_t bm = __ballot((cnt >> k) & 1u);
                pre += __builtin_amdgcn_mbcnt_hi(uint32_t(bm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(bm), 0u)) << k;
                total += uint32_t(__popcll(bm)) << k;
            }
            uint32_t* task = img + fix_tasks<BPT>() + (tid >> 6) * 128;  // [64] tasks, then [64] results
            uint32_t* res = task + 64;
            for (uint32_t r0 = 0; r0 < total; r0 += 64) {
                uint32_t m = sf, i = pre - r0;
                while (m) {
                    const int bit = __ffs(m) - 1;
                    m &= m - 1;
                    if (i < 64u) task[i] = (uint32_t(tid) << 4) | uint32_t(bit);
                    i++;
                }
                wave_sync();
                if (uint32_t(lane) < total - r0) {
                    const uint32_t tk = task[lane];
                    const int s = int(tk & 3u), b = int((tk >> 2) & 3u), owner = int(tk >> 4);
                    const BlockPx<N> px = block_px(b, owner);
                    const int ks = kFullRows ? Structural<N>::k[0] * (s == 0) + Structural<N>::k[1] * (s == 1) +
                                                   Structural<N>::k[2] * (s == 2)
                                             : s;
                    res[lane] = (ablate & 256) ? (px.w[0] & 0xFFFFu)  // profiling: no FP64 arithmetic
                                                 : uint32_t(exact_coef_row<N>(rowP(ks), rowS(ks), rowRq(ks),
                                                                              rowQd(ks), px)) & 0xFFFFu;
                }
                wave_sync();
                m = sf;
                i = pre - r0;
                while (m) {
                    const int bit = __ffs(m) - 1;
                    m &= m - 1;
                    if (i < 64u) {
                        const uint32_t v = res[i];
                        const int b = bit >> 2, s = bit & 3;
#pragma unroll
                        for (int bb = 0; bb < BPT; bb++)
#pragma unroll
                            for (int ss = 0; ss < 3; ss++) {
                                const int zpos = Structural<N>::zpos(ss);
                                if (b == bb && s == ss)
                                    zp[bb][zpos >> 1] = (zpos & 1) ? ((zp[bb][zpos >> 1] & 0xFFFFu) | (v << 16))
                                                                   : ((zp[bb][zpos >> 1] & 0xFFFF0000u) | v);
                            }
                    }
                    i++;
                }
                wave_sync();  // the next round rewrites the task list
            }
            // Whole-block requests (rare: an ordinary coefficient near a tie): all NN coefficients
            // of the block are re-evaluated in FP64, one per lane, four blocks per round.
            const uint32_t wf = flags & (0x88888888u >> (32 - 4 * BPT));
            if (__ballot(wf != 0)) {
                const uint32_t nb = __popc(wf);
                uint32_t pb = 0, tb = 0;
#pragma unroll
                for (int k = 0; k < 3; k++) {  // nb <= BPT <= 4
                    const uint64_t bm = __ballot((nb >> k) & 1u);
                    pb += __builtin_amdgcn_mbcnt_hi(uint32_t(bm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(bm), 0u)) << k;
                    tb += uint32_t(__popcll(bm)) << k;
                }
                for (uint32_t r0 = 0; r0 < tb; r0 += 4) {
                    uint32_t m = wf, j = pb - r0;
                    while (m) {
                        const int b = (__ffs(m) - 1) >> 2;
                        m &= m - 1;
                        if (j < 4u) task[j] = (uint32_t(tid) << 4) | uint32_t(b);
                        j++;
                    }
                    wave_sync();
                    if (uint32_t(lane >> 4) < tb - r0) {
                        const uint32_t tk = task[lane >> 4];
                        const int b = int(tk & 3u), owner = int(tk >> 4), k = lane & 15;
                        const BlockPx<N> px = block_px(b, owner);
                        res[lane] = uint32_t(kFullRows ? exact_coef_row<N>(rowP(k), rowS(k), rowRq(k), rowQd(k), px)
                                                       : exact_coef_row<N>(tab->P + k * NN, tab->S[k], tab->rq[k],
                                                                           tab->qd[k], px)) & 0xFFFFu;
                    }
                    wave_sync();
                    m = wf;
                    j = pb - r0;
                    while (m) {
                        const int b = (__ffs(m) - 1) >> 2;
                        m &= m - 1;
                        if (j < 4u) {
                            const uint32_t* rr = res + 16 * j;
#pragma unroll
                            for (int jj = 0; jj < NP; jj++) {
                                const uint32_t w = rr[ZigZag<N>::idx[2 * jj]] | (rr[ZigZag<N>::idx[2 * jj + 1]] << 16);
#pragma unroll
                                for (int bb = 0; bb < BPT; bb++) zp[bb][jj] = (b == bb) ? w : zp[bb][jj];
                            }
                        }
                        j++;
                    }
                    wave_sync();
                }
            }
        }
        const unsigned wsum = unsigned(wave_sum64(__popc(flags)));
        if ((tid & 63) == 0) a.wave_fix[size_t(t) * (TPB / 64) + (tid >> 6)] = wsum;
    }
    asm volatile("; PHASE fix_done" ::: "memory");
    STAMP(4);

    // ---------------------------------------------------------------- 1c. zig-zag RLE sizing
    uint32_t blw[BPT];  // bl | Lw << 8
    uint32_t rbits[BPT];
    uint32_t mybits = 0;
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        if (a.coef && b < nblk) {
            int16_t* dst = a.coef + (size_t(frame) * a.by * a.bx + size_t(byi) * a.bx + bx0 + b) * NN;
#pragma unroll
            for (int k = 0; k < NN; k++) {
                const int kz = ZigZagInv<N>::pos[k];
                dst[k] = int16_t(kz & 1 ? (zp[b][kz >> 1] >> 16) : (zp[b][kz >> 1] & 0xFFFFu));
            }
        }
        blw[b] = size_block<N>(zp[b], a.rle, &rbits[b]);
        rbits[b] = (b < nblk) ? rbits[b] : 0u;
        mybits += rbits[b];
    }
    asm volatile("; PHASE size_done" ::: "memory");
    if (ablate & 2048) {  // profiling: ... + FP64 fix-up + sizing
        uint32_t acc = mybits;
#pragma unroll
        for (int b = 0; b < BPT; b++)
#pragma unroll
            for (int j = 0; j < NP; j++) acc ^= zp[b][j] + blw[b];
        if (acc == 0x9E3779B9u) a.err[1] = acc;
        return;
    }
    STAMP(5);
    // (the fix-up slots alias the tile image: the scan's barrier below orders them before the
    // image is zeroed)

    // ---------------------------------------------------------------- 2. tile scan + LDS image
    uint32_t A;
    const uint32_t off = block_excl_scan<TPB>(mybits, misc, &A);
    if (tid == 0) chain_publish_count(a.st, t, chain_pos, a.tag, A);  // successors may resolve now
    Probe pr{0, 0, 0};
    if (tid < 64 && chain_pos != 0 && !(ablate & 4)) pr = probe_issue(a.st, t, chain_pos, step, 0, kProbe0);  // in flight during emission
    const uint32_t nw = (A + 31) >> 5;
    for (uint32_t w = 4 * tid; w < nw + 2; w += 4 * TPB) *reinterpret_cast<u32x4*>(img + w) = u32x4{0u, 0u, 0u, 0u};
    lds_barrier();
    asm volatile("; PHASE scan_done" ::: "memory");
    STAMP(6);
    if (!(ablate & 2)) {  // the records: header + Lw + z0 and coefficient triples, or pairs
        uint32_t p = off;
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            if (N == 4 && a.tri && a.rle) {
                if constexpr (N == 4)
                    if (rbits[b]) emit_block3(img, p, zp[b], blw[b]);
            } else {
                if (rbits[b]) emit_block2<N>(img, p, zp[b], blw[b], a.rle);
            }
            p += rbits[b];
        }
    }
    lds_barrier();
    asm volatile("; PHASE emit_done" ::: "memory");
    STAMP(7);

    // ---------------------------------------------------------------- 3. look-back
    const bool chain_last = a.segmented ? (tif == a.tiles_per_frame - 1) : (t == a.ntiles - 1);
    uint32_t* out = a.out + (a.segmented ? uint64_t(frame) * a.out_pitch_words : 0ull);
    uint64_t excl;
    if (ablate & 4) {
        if (tid == 0) {
            publish(a.st, t, 1, a.tag, A);
            ctl[7] = 0;
            ctl[8] = 0;
        }
        lds_barrier();
        excl = uint64_t(tif) * (110u * TPB);
    } else {
        excl = chain_resolve(a.st, t, chain_pos, step, a.tag, img, A, out, start_bit, a.err, ctl, pr,
                             stamps ? &stamps[size_t(t) * kStamps + 1] : nullptr, true, a.deep_lb != 0);
    }
    if (tid == 0) {
        const uint64_t P = start_bit + excl;
        if (tif == 0) a.frame_start[frame] = P;
        if (chain_last) a.chain_end[a.segmented ? frame : 0] = P + A;
    }
    asm volatile("; PHASE lookback_done" ::: "memory");
    STAMP(8);

    // ---------------------------------------------------------------- 4. store
    if constexpr (HIST) {
        if (tif == 0)  // the words before the first record word hold only the caller's header
            for (uint32_t i = tid; i < uint32_t(start_bit >> 5); i += TPB) {
                const uint32_t v = out[i];
#pragma unroll
                for (int k = 0; k < 4; k++) atomicAdd(&hl[(v >> (8 * k)) & 0xFFu], 1u);
            }
        const uint64_t end = start_bit + excl + A;
        const HistCount cnt{hl, chain_last ? (end + 7) / 8 : ~0ull};
        store_tile<TPB>(out, img, A, start_bit + excl, ctl, chain_last, a.st, t - step, a.tag, a.err, cnt);
        lds_barrier();
        for (int i = tid; i < 256; i += TPB)
            if (hl[i]) atomicAdd(&a.hist[size_t(frame) * 256 + i], hl[i]);
    } else if (!(ablate & 8)) {
        store_tile<TPB>(out, img, A, start_bit + excl, ctl, chain_last, a.st, t - step, a.tag, a.err);
    }
    STAMP(9);
}

// round_block<4> with the rounding done pair by pair in zig-zag order and each packed word
// pinned as soon as it exists: the 16 magic-added quotients never live at once (register
// pressure of encode4w_kernel's fourth slot).  Same results bit for bit.
__device__ __forceinline__ float round_block_lean4(const EncTables* __restrict__ tab, const float (&t)[16],
                                                   uint32_t (&zp)[8], uint32_t* sflags) {
    constexpr int S0 = Structural<4>::k[0], S1 = Structural<4>::k[1], S2 = Structural<4>::k[2];
    const bool dcx = tab->dc_exact != 0;
    float emax = 0.0f;
    uint32_t sf = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        uint32_t yb[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int k = ZigZag<4>::idx[2 * j + h];
            const float y = t[k] + kMagic;
            const float e = fabsf(t[k] - (y - kMagic));
            yb[h] = __float_as_uint(y);
            if (k == 0) {
                const uint32_t dc = uint32_t(int(truncf(t[0] + copysignf(0.5f, t[0]))));
                yb[h] = dcx ? dc : yb[h];
                emax = dcx ? emax : fmaxf(emax, e);
            } else if (k == S0) {
                sf |= (e >= tab->lim[S0]) ? 1u : 0u;
            } else if (k == S1) {
                sf |= (e >= tab->lim[S1]) ? 2u : 0u;
            } else if (k == S2) {
                sf |= (e >= tab->lim[S2]) ? 4u : 0u;
            } else {
                emax = fmaxf(emax, e);
            }
        }
        zp[j] = __builtin_amdgcn_perm(yb[1], yb[0], 0x05040100u);
        asm volatile("" : "+v"(zp[j]));
        if (j & 1) __builtin_amdgcn_sched_barrier(0);
    }
    *sflags = sf;
    return emax;
}

// =============================================================================================
// encode4w_kernel -- the 4x4 FAST encoder with WAVE-LOCAL emission.
//
// Same tile (1024 blocks, 256 threads, one chain element, the same chain granules) and the same
// arithmetic as encode_kernel<4, false> (quot4 + round_block + the compacted FP64 fix-up, so the
// Trk exactness argument carries over unchanged), laid out so that a wave needs its workgroup
// only twice:
//   * wave w owns the tile's blocks [256w, 256w + 256) (64 groups of four, raster order); lane l
//     computes block 64b + l of that run in SLOT b = 0..3, so a slot is 64 consecutive blocks of
//     the stream and one wave scan (DPP) places every record inside its slot;
//   * the pixels land in the wave's own LDS region by DMA as [row][256 blocks] words (a slot
//     reads them conflict-free, no other wave touches them); after the fix-up the same region
//     holds two slot images in turn: slots 0 and 1 are emitted while wave 0 resolves the tile's
//     look-back, then each slot is stored as soon as its image is complete and its buffer takes
//     slot b + 2;
//   * a word shared by two waves of the tile is written by the earlier wave, which ORs in the
//     later wave's first bits (its head word, saved in LDS before the look-back barrier); a word
//     shared with the predecessor tile is completed with that tile's tail granule as in
//     encode_kernel.
// LDS per tile 20.5 KB (encode_kernel<4>: ~27 KB), so up to seven tiles per CU.
// Preconditions (launch_encode checks them): whole 16-byte groups (vec_ok, bx % 4 == 0), at
// least 8 groups in every tile (groups_per_frame % 8 == 0: every wave segment >= 160 bits) and
// slot images that fit half a region (rec_bits <= 252).
// =============================================================================================
// Look-back windows after the first probe, for launches that fill the chip (one small window at a
// time: the nearest inclusive prefix is seldom far, and each probed predecessor is an uncached
// load -- C4's one 8 128-tile chain: 2 windows of 64 108.6 us, 1 of 64 102.4, 1 of 32 101.1, 1 of
// 16 104.4 us per 64-frame launch; C2 and one 4K frame unchanged; tools/ab.py, round 6)
#ifndef IE_W_AHEAD
#define IE_W_AHEAD 1  // windows per round trip (each holds 4 VGPRs live beside slots 2-3)
#endif
#ifndef IE_W_LBW
#define IE_W_LBW 32  // predecessors per window
#endif
#ifndef IE_W_WAVES
#define IE_W_WAVES 6  // __launch_bounds__ occupancy hint (waves per SIMD): 76 VGPRs, no scratch (7 spills)
#endif
constexpr int kWReg = 1024;  // words per wave region: [4 rows][64 NS blocks] pixels, then the slot-pair images in turn
constexpr int kWTask = 128;  // words per wave: fix-up tasks [64] + results [64]
constexpr int kWMisc = 32;   // [0..3] wave bits, [4..7] wave head words, [8..9] excl, [10] ptail, [11] tail pending, [12] ticket,
                             // [16..17] FP64 task counters, [18..25] small-launch window sums, [26..29] their found flags
// FP64 rows in LDS (doubles): P[16][16] then S, rq, qd of every coefficient (the structural
// three alone measured equal: the LDS they would free does not add a tile per CU at 78 VGPRs)
constexpr int kWRows = 16 * 16 + 3 * 16;
constexpr int kWLdsBytes = (4 * kWReg + 4 * kWTask + kWMisc) * 4 + kWRows * 8;
// HIST: copies of the byte histogram (tools/ab.py --op counted, 16 4K frames: counting costs 20.3 us
// over a launch without it at 1 copy, 15.8 at 4; 8 and 16 copies cost a tile per CU and are slower,
// two 16-bit bins per word slower still -- the LDS read-modify-write of 112 M byte-adds is the floor)
constexpr int kWHistRep = 4;

// Inclusive scan over the 64 lanes of a wave by DPP row shifts and row broadcasts (six VALU).
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xF, 0xF, true));   // row_shr:1
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xF, 0xF, true));   // row_shr:2
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xF, 0xF, true));   // row_shr:4
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xF, 0xF, true));   // row_shr:8
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xA, 0xF, false));  // row_bcast:15
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xC, 0xF, false));  // row_bcast:31
    return v;
}

// One slot image I (bit 0 at absolute stream bit X) to the output words, by one wave: words
// [r0, nw) counted from floor(X / 32), word r = alignbit(I[r - 1], I[r], X % 32) with I[-1] =
// prev (the 32 bits before X); the partial word nw is left to whoever writes the next bits.
template <typename Cnt = NoCount>
__device__ __forceinline__ void store_slot(uint32_t* __restrict__ out, const uint32_t* I, uint64_t X, uint32_t nw,
                                           uint32_t r0, uint32_t prev, int lane, const Cnt& cnt = Cnt{}) {
    if (nw <= r0) return;
    const uint64_t w0 = X >> 5;
    const uint32_t s = uint32_t(X) & 31u;
    auto word = [&](uint32_t r) -> uint32_t {
        const uint32_t am = I[max(r, 1u) - 1u];
        return bswap32(__builtin_amdgcn_alignbit(r ? am : prev, I[r], s));
    };
    uint32_t hd = min(nw - r0, uint32_t((4u - uint32_t((w0 + r0) & 3u)) & 3u));
    if (r0 + hd == 0u) hd = min(nw, 4u);  // (the quad loop needs I[r - 1]: word -1 is prev)
    if (uint32_t(lane) < hd) {
        const uint32_t v = word(r0 + lane);
        out[w0 + r0 + lane] = v;
        cnt(w0 + r0 + lane, v);
    }
    const uint32_t rq = r0 + hd, nq = (nw - rq) >> 2;
    // output quad q = words rq + 4q .. +3 (16-byte aligned in out) needs I[rq + 4q - 1 ..
    // rq + 4q + 3]: five words at offset d of the two 16-byte LDS quads from (rq - 1) / 4 + q,
    // read whole (consecutive lanes, consecutive quads: no bank conflicts), d wave-uniform
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const uint32_t d = (rq - 1u) & 3u;
    const v4u* I4 = reinterpret_cast<const v4u*>(I) + ((rq - 1u) >> 2);
    uint32_t* const ob = out + (w0 + rq);
    auto quads = [&](auto dc) {
        constexpr uint32_t D = decltype(dc)::value;
        for (uint32_t q = lane; q < nq; q += 64) {
            const v4u A = I4[q], B = I4[q + 1];
            const uint32_t W[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
            const v4u v = {bswap32(__builtin_amdgcn_alignbit(W[D], W[D + 1], s)), bswap32(__builtin_amdgcn_alignbit(W[D + 1], W[D + 2], s)),
                           bswap32(__builtin_amdgcn_alignbit(W[D + 2], W[D + 3], s)), bswap32(__builtin_amdgcn_alignbit(W[D + 3], W[D + 4], s))};
            __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(ob + 4u * q));
            cnt(w0 + rq + 4u * q, v.x);
            cnt(w0 + rq + 4u * q + 1u, v.y);
            cnt(w0 + rq + 4u * q + 2u, v.z);
            cnt(w0 + rq + 4u * q + 3u, v.w);
        }
    };
    if (d == 0u) quads(std::integral_constant<uint32_t, 0>{});
    else if (d == 1u) quads(std::integral_constant<uint32_t, 1>{});
    else if (d == 2u) quads(std::integral_constant<uint32_t, 2>{});
    else quads(std::integral_constant<uint32_t, 3>{});

    const uint32_t rt = rq + 4u * nq;
    if (uint32_t(lane) < nw - rt) {
        const uint32_t v = word(rt + lane);
        out[w0 + rt + lane] = v;
        cnt(w0 + rt + lane, v);
    }
}

// The last 32 bits of the stream up to the end of a slot image of n bits, given the 32 bits
// before it (prev).
__device__ __forceinline__ uint32_t slot_tail32(const uint32_t* I, uint32_t n, uint32_t prev) {
    if (n >= 32) return image_tail32(I, n);
    return n ? ((prev << n) | (I[0] >> (32u - n))) : prev;
}

// profiling builds (IE_PROFILE, IE_STAMPS set): lane 0 of each wave stamps s_memtime at its phase
// boundaries, [tile][wave][12] (tools/stamps_w.py)
#define WSTAMP(i)                                                                                                   \
    do {                                                                                                            \
        if (IE_PROFILE && a.stamps && lane == 0 && wv < 4) a.stamps[size_t(t) * kStamps + wv * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// the chip-wide 100 MHz clock (comparable across CUs and XCDs) at the wave's start (14) and end (15)
#define WRTSTAMP(i)                                                                                                 \
    do {                                                                                                            \
        if (IE_PROFILE && a.stamps && lane == 0 && wv < 4) a.stamps[size_t(t) * kStamps + wv * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

// HIST (ie_encode_images_counted): every stored byte also counted into a per-tile LDS histogram
// (256 words after misc), merged into a.hist[frame] at the end -- the Huffman pass's byte counts
// without reading the stream back.
template <bool HIST>
__global__ __launch_bounds__(256, IE_W_WAVES) void encode4w_kernel(EncArgs a, const EncTables* __restrict__ tab) {
    // (two slots per lane -- twice the tiles for small launches -- measured slower on a lone 4K
    // frame, 23.9 against 18.2 us: the phases are bound by the SIMDs' issue, not by one wave's
    // latency, and twice the tiles lengthen the look-back)
    constexpr int N = 4, NN = 16, NP = 8, TPB = 256, NS = 4;
    constexpr int GW = 16 * NS, BW = 64 * NS, TG = 4 * GW;  // groups / blocks per wave, groups per tile
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar registers
    uint32_t* const reg = smem + wv * kWReg;  // this wave's pixels, later its two slot images
    uint32_t* const task = smem + 4 * kWReg + wv * kWTask;
    uint32_t* const res = task + 64;
    uint32_t* const misc = smem + 4 * kWReg + 4 * kWTask;
    uint32_t* const hl = misc + kWMisc;  // HIST: the tile's byte histogram
    constexpr int HR = kWHistRep, HWORDS = 256 * HR;
    double* const srow = reinterpret_cast<double*>(misc + kWMisc + (HIST ? HWORDS : 0));

    int t;
    if (a.ticket) {
        if (tid == 0) misc[12] = uint32_t(atomicAdd(a.ticket, 1ull) - a.ticket_base);
        lds_barrier();
        t = __builtin_amdgcn_readfirstlane(int(misc[12]));
        if (t >= a.ntiles) return;
    } else {
        t = int(blockIdx.x);
    }
    WSTAMP(0);
    WRTSTAMP(14);
    asm volatile("; PHASE w0" ::: "memory");
    if constexpr (HIST)
        for (int i = tid; i < HWORDS; i += TPB) hl[i] = 0u;  // (visible after the first barrier)
    // the FP64 rows and their S, rq, qd: the fix-up reads them from LDS
    for (int i = tid; i < kWRows; i += TPB)
        srow[i] = (i < NN * NN) ? tab->P[i] : (i < NN * NN + NN) ? tab->S[i - NN * NN]
                : (i < NN * NN + 2 * NN) ? tab->rq[i - NN * NN - NN] : tab->qd[i - NN * NN - 2 * NN];
    const TileGeo g = tile_geo<4, 4, TG>(a, t, tid);  // lane l of wave w: group 64 w + l of the tile
    const uint64_t start_bit = a.start_dev ? *a.start_dev : a.start_bit;
    const int frame = g.frame, tif = g.tif, step = g.step, chain_pos = g.chain_pos;
    // groups in this tile / in this wave (>= 8 per tile: launch precondition)
    const int ng = min(TG, a.groups_per_frame - tif * TG);
    const int nbw = 4 * min(GW, max(0, ng - GW * wv));  // blocks of this wave
    const int wlast = (ng - 1) / GW;                    // the tile's last non-empty wave
    if (g.nblk) {
        // pixel row r of the wave's block j at reg[r BW + j]: a lane's 16 bytes are its group's row
        const uint8_t* base = a.y + size_t(frame) * a.frame_pitch + size_t(g.byi) * N * a.stride + size_t(g.bx0) * N;
#pragma unroll
        for (int r = 0; r < N; r++)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + size_t(r) * a.stride),
                                             (__attribute__((address_space(3))) void*)(reg + r * BW), 16, 0, 0);
    }
    lds_barrier();                                            // srow visible (the pixel DMA stays in flight)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pixels landed
    WSTAMP(1);
    asm volatile("; PHASE w1" ::: "memory");

    // ------------------------------------------------------------ transform + quantise, 4 slots
    uint32_t zp[NS][NP];
    uint32_t flags = 0;  // 4 bits per slot: structural s (bits 0-2), whole block (bit 3)
#pragma unroll
    for (int b = 0; b < NS; b++) {
        __builtin_amdgcn_sched_barrier(0);
        uint32_t rows[N][1];
#pragma unroll
        for (int r = 0; r < N; r++) rows[r][0] = reg[r * BW + 64 * b + lane];
        float x[NN];
        block_pixels<N, 1>(rows, 0, x);
        uint32_t sf;
        float emax;
        quotients<N>(tab, x);
        emax = round_block_lean4(tab, x, zp[b], &sf);
        const uint32_t fb = (emax >= tab->lim_min) ? 8u : sf;
        if (64 * b + lane < nbw) flags |= fb << (4 * b);
        // pin the packed words here: otherwise the packing sinks to its first use and the 16
        // unpacked quotients of every slot stay live across the slots (spills)
#pragma unroll
        for (int j = 0; j < NP; j++) asm volatile("" : "+v"(zp[b][j]));
        asm volatile("" : "+v"(flags));
    }

    WSTAMP(2);
    asm volatile("; PHASE w2" ::: "memory");
    // ------------------------------------------------------------ FP64 fix-up
    static_assert(Structural<4>::zpos(0) & Structural<4>::zpos(1) & Structural<4>::zpos(2) & 1,
                  "4x4 structural coefficients sit in high halves of the packed words");
    auto block_px = [&](int b, int owner) {
        BlockPx<N> px;
#pragma unroll
        for (int r = 0; r < N; r++) px.w[r] = reg[r * BW + 64 * b + owner];
        return px;
    };
    if (__ballot(flags != 0)) {
        const uint32_t sf = flags & 0x7777u;
        const uint32_t cnt = __popc(sf);
        uint32_t pre = 0, total = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {  // cnt <= 12
            const uint64_t bm = __ballot((cnt >> k) & 1u);
            pre += __builtin_amdgcn_mbcnt_hi(uint32_t(bm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(bm), 0u)) << k;
            total += uint32_t(__popcll(bm)) << k;
        }
        for (uint32_t r0 = 0; r0 < total; r0 += 64) {
            uint32_t m = sf, i = pre - r0;
            while (m) {
                const int bit = __ffs(m) - 1;
                m &= m - 1;
                if (i < 64u) task[i] = (uint32_t(lane) << 4) | uint32_t(bit);
                i++;
            }
            wave_sync();
            if (uint32_t(lane) < total - r0) {
                const uint32_t tk = task[lane];
                const int s = int(tk & 3u), b = int((tk >> 2) & 3u), owner = int(tk >> 4);
                const BlockPx<N> px = block_px(b, owner);
                const int k = Structural<N>::k[0] * (s == 0) + Structural<N>::k[1] * (s == 1) + Structural<N>::k[2] * (s == 2);
                const int y = exact_coef_row<N>(srow + k * NN, srow[NN * NN + k], srow[NN * NN + NN + k],
                                                srow[NN * NN + 2 * NN + k], px);
                res[lane] = uint32_t(y) & 0xFFFFu;
            }
            wave_sync();
            // the owners take their results back: the flagged positions in bit order, each a
            // constant register (the three structural coefficients are high halves of packed
            // words), so no per-request select over every slot and coefficient
            i = pre - r0;
#pragma unroll
            for (int b = 0; b < NS; b++)
#pragma unroll
                for (int ss = 0; ss < 3; ss++) {
                    if ((sf >> (4 * b + ss)) & 1u) {
                        const int zw = Structural<N>::zpos(ss) >> 1;
                        static_assert(Structural<4>::zpos(0) & Structural<4>::zpos(1) & Structural<4>::zpos(2) & 1,
                                      "4x4 structural coefficients sit in high halves");
                        if (i < 64u) zp[b][zw] = __builtin_amdgcn_perm(res[i], zp[b][zw], 0x05040100u);  // res low -> high half
                        i++;
                    }
                }
            wave_sync();
        }
        // whole-block requests (rare): all 16 coefficients in FP64, one per lane, four blocks a round
        const uint32_t wf = flags & 0x8888u;
        if (__ballot(wf != 0)) {
            const uint32_t nb = __popc(wf);
            uint32_t pb = 0, tb = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) {  // nb <= 4
                const uint64_t bm = __ballot((nb >> k) & 1u);
                pb += __builtin_amdgcn_mbcnt_hi(uint32_t(bm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(bm), 0u)) << k;
                tb += uint32_t(__popcll(bm)) << k;
            }
            for (uint32_t r0 = 0; r0 < tb; r0 += 4) {
                uint32_t m = wf, j = pb - r0;
                while (m) {
                    const int b = (__ffs(m) - 1) >> 2;
                    m &= m - 1;
                    if (j < 4u) task[j] = (uint32_t(lane) << 4) | uint32_t(b);
                    j++;
                }
                wave_sync();
                if (uint32_t(lane >> 4) < tb - r0) {
                    const uint32_t tk = task[lane >> 4];
                    const int b = int(tk & 3u), owner = int(tk >> 4), k = lane & 15;
                    const BlockPx<N> px = block_px(b, owner);
                    const int y = exact_coef_row<N>(srow + k * NN, srow[NN * NN + k], srow[NN * NN + NN + k],
                                                    srow[NN * NN + 2 * NN + k], px);
                    res[lane] = uint32_t(y) & 0xFFFFu;
                }
                wave_sync();
                m = wf;
                j = pb - r0;
                while (m) {
                    const int b = (__ffs(m) - 1) >> 2;
                    m &= m - 1;
                    if (j < 4u) {
                        const uint32_t* rr = res + 16 * j;
#pragma unroll
                        for (int jj = 0; jj < NP; jj++) {
                            const uint32_t w = rr[ZigZag<N>::idx[2 * jj]] | (rr[ZigZag<N>::idx[2 * jj + 1]] << 16);
#pragma unroll
                            for (int bb = 0; bb < NS; bb++) zp[bb][jj] = (b == bb) ? w : zp[bb][jj];
                        }
                    }
                    j++;
                }
                wave_sync();
            }
        }
    }
    {  // statistics: FP64 requests of this wave (one store)
        const uint32_t wsum = __builtin_amdgcn_readlane(wave_incl_scan_dpp(uint32_t(__popc(flags))), 63);
        if (lane == 0) a.wave_fix[size_t(t) * (TPB / 64) + wv] = wsum;
    }

    WSTAMP(3);
    asm volatile("; PHASE w3" ::: "memory");
    // ------------------------------------------------------------ sizing + the wave's offsets
    uint32_t blw[NS], rb[NS];
    const uint32_t k0 = uint32_t(tif * TG + GW * wv) * 4u;  // the wave's first block (frame raster order)
#pragma unroll
    for (int b = 0; b < NS; b++) {
        const bool valid = 64 * b + lane < nbw;
        if (a.coef && valid) {
            int16_t* dst = a.coef + (size_t(frame) * a.by * a.bx + k0 + 64 * b + lane) * NN;
#pragma unroll
            for (int k = 0; k < NN; k++) {
                const int kz = ZigZagInv<N>::pos[k];
                dst[k] = int16_t(kz & 1 ? (zp[b][kz >> 1] >> 16) : (zp[b][kz >> 1] & 0xFFFFu));
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        blw[b] = size_block<N>(zp[b], a.rle, &rb[b]);
        rb[b] = valid ? rb[b] : 0u;
        asm volatile("" : "+v"(blw[b]), "+v"(rb[b]));
#pragma unroll
        for (int j = 0; j < NP; j++) asm volatile("" : "+v"(zp[b][j]));
        __builtin_amdgcn_sched_barrier(0);
    }
    // slot pairs packed into 16-bit halves (a slot holds <= 64 * 252 bits)
    const uint32_t s01 = rb[0] | (rb[1] << 16), s23 = rb[2] | (rb[3] << 16);
    const uint32_t i01 = wave_incl_scan_dpp(s01), i23 = wave_incl_scan_dpp(s23);
    const uint32_t t01 = __builtin_amdgcn_readlane(i01, 63), t23 = __builtin_amdgcn_readlane(i23, 63);
    const uint32_t e01 = i01 - s01, e23 = i23 - s23;  // exclusive, per half (no borrow: each half >= 0)
    uint32_t T[NS], off[NS];
    T[0] = t01 & 0xFFFFu;
    T[1] = t01 >> 16;
    T[2] = t23 & 0xFFFFu;
    T[3] = t23 >> 16;
    off[0] = e01 & 0xFFFFu;
    off[1] = e01 >> 16;
    off[2] = e23 & 0xFFFFu;
    off[3] = e23 >> 16;
    const uint32_t S1 = T[0], S2 = S1 + T[1], S3 = S2 + T[2], Tw = S3 + T[3];
    if (lane == 0) misc[wv] = Tw;
    WSTAMP(4);
    asm volatile("; PHASE w4" ::: "memory");
    lds_barrier();  // ---- the tile's bit count and this wave's place in it
    WSTAMP(5);
    asm volatile("; PHASE w5" ::: "memory");

    uint32_t A = 0, W = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint32_t v = __builtin_amdgcn_readfirstlane(misc[w]);
        A += v;
        W += (w < wv) ? v : 0u;
    }
    if (tid == 0) chain_publish_count(a.st, t, chain_pos, a.tag, A);  // successors may resolve now
    // look-back probes, in flight while emitting.  A launch too small to fill the chip (deep_lb:
    // its tiles reach their look-back together, so a tile's nearest inclusive prefix is far away):
    // the four waves read predecessors [64 DW wv, 64 DW (wv + 1)) in DW windows each -- 256 DW in
    // one round trip; otherwise wave 0 reads the nearest kProbe0.
    constexpr int DW = 2;
    const bool deep = a.deep_lb != 0;
    Probe pr[DW];
#pragma unroll
    for (int i = 0; i < DW; i++) pr[i] = Probe{0, 0, 0};
    if (chain_pos != 0) {
        if (deep) {
#pragma unroll
            for (int i = 0; i < DW; i++) pr[i] = probe_issue(a.st, t, chain_pos, step, 64 * (DW * wv + i), 64);
        } else if (wv == 0) {
            pr[0] = probe_issue(a.st, t, chain_pos, step, 0, kProbe0);
        }
    }

    // slot-pair images: slots 0 and 1, then slots 2 and 3, each pair as ONE bit image from word 0
    // of the wave's region (a pair holds <= 2 * 64 * 252 bits = 1008 words); emission takes
    // absolute LDS bit addresses (scatter_bits' ds_or addresses LDS from byte 0)
    const uint32_t reg_bit0 = uint32_t(wv * kWReg) * 32u;
    const uint32_t Sb[NS] = {0u, S1, S2, S3};
    auto zero_img = [&](uint32_t bits) {
        const uint32_t nq = (bits + 127u) >> 7;  // 16-byte groups
        for (uint32_t q = lane; q < nq; q += 64) *reinterpret_cast<u32x4*>(reg + 4 * q) = u32x4{0u, 0u, 0u, 0u};
    };
    auto emit_slot = [&](int b) {  // slot b at its place in its pair's image
        if (rb[b]) {
            const uint32_t p = reg_bit0 + (Sb[b] - Sb[b & 2]) + off[b];
            if (a.tri && a.rle) emit_block3(smem, p, zp[b], blw[b]);
            else emit_block2<N>(smem, p, zp[b], blw[b], a.rle);
        }
    };
    zero_img(S2);
    wave_sync();
    emit_slot(0);
    emit_slot(1);
    wave_sync();
    WSTAMP(6);
    asm volatile("; PHASE w6" ::: "memory");
    if (lane == 0 && Tw) misc[4 + wv] = reg[0];  // the wave's first 32 bits

    // ------------------------------------------------------------ look-back (wave 0)
    const bool chain_last = a.segmented ? (tif == a.tiles_per_frame - 1) : (t == a.ntiles - 1);
    uint32_t* const out = a.out + (a.segmented ? uint64_t(frame) * a.out_pitch_words : 0ull);
    if (deep && chain_pos != 0) {
        // every wave sums its windows in order, up to the first with an inclusive prefix (read
        // again until every value it needs is published; its predecessors never wait on this
        // tile), for wave 0 to combine
        uint64_t sm = 0;
        bool found = false;
        unsigned spins = 0;
        for (;;) {
            bool ready = true;
            sm = 0;
            found = false;
#pragma unroll
            for (int i = 0; i < DW; i++) {
                const WinSum r = window_sum(pr[i], chain_pos, 64 * (DW * wv + i), 64, a.tag);
                if (!found) {
                    ready = ready && r.ready;
                    sm += r.sum;
                    found = r.found;
                }
            }
            if (ready) break;
            if (++spins > kSpinLimit) {
                if (lane == 0) atomicAdd(&a.err[0], 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int i = 0; i < DW; i++) pr[i] = probe_issue(a.st, t, chain_pos, step, 64 * (DW * wv + i), 64);
        }
        if (lane == 0) {
            misc[18 + 2 * wv] = uint32_t(sm);
            misc[19 + 2 * wv] = uint32_t(sm >> 32);
            misc[26 + wv] = found ? 1u : 0u;
        }
        lds_barrier();
    }
    if (wv == 0) {
        uint64_t excl = 0;
        uint32_t ptail = 0, pend = 0;
        if (chain_pos == 0) {
            // chain start: the bits before start_bit belong to the caller (header)
            const uint32_t s = uint32_t(start_bit & 31);
            ptail = s ? (bswap32(out[start_bit >> 5]) >> (32 - s)) : 0u;
        } else {
            bool done = false;
            if (deep) {  // the waves' sums in predecessor order, up to the first window with an inclusive prefix
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    if (!done) {
                        excl += uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(misc[18 + 2 * w]))) |
                                (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(misc[19 + 2 * w]))) << 32);
                        done = __builtin_amdgcn_readfirstlane(misc[26 + w]) != 0;
                    }
                }
                if (!done) excl = 0;  // more than 256 DW predecessors back: the wave-0 walk from the start
            }
            if (!done) {
                const Probe p0 = deep ? probe_issue(a.st, t, chain_pos, step, 0, kProbe0) : pr[0];
                excl = lookback_wave<IE_W_AHEAD, IE_W_LBW>(p0, a.st, t, chain_pos, step, a.tag, a.err, nullptr, deep);
            }
            const bool have = uint32_t(pr[0].gt >> 56) == a.tag;  // (lane 0's probe read the tail)
            const bool split = ((start_bit + excl) & 31) != 0;
            ptail = have ? uint32_t(pr[0].gt) : 0u;
            pend = (!have && split) ? 1u : 0u;
        }
        if (lane == 0) {
            if (chain_pos != 0) publish(a.st, t, 1, a.tag, excl + A);
            misc[8] = uint32_t(excl);
            misc[9] = uint32_t(excl >> 32);
            misc[10] = ptail;
            misc[11] = pend;
            const uint64_t P = start_bit + excl;
            if (tif == 0) a.frame_start[frame] = P;
            if (chain_last) a.chain_end[a.segmented ? frame : 0] = P + A;
        }
    }
    WSTAMP(7);
    asm volatile("; PHASE w7" ::: "memory");
    lds_barrier();  // ---- the tile's position
    WSTAMP(8);
    asm volatile("; PHASE w8" ::: "memory");

    // ------------------------------------------------------------ store, slot by slot
    if (Tw) {
        // (readfirstlane returns int: zero-extend each half, or a prefix of 2^31 bits or more
        // would sign-extend into the high word)
        const uint64_t excl = uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(misc[8]))) |
                              (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(misc[9]))) << 32);
        const uint64_t Xw = start_bit + excl + W;
        const bool pend = __builtin_amdgcn_readfirstlane(misc[11]) != 0u;
        // the wave's first word is written by the previous wave (or, pending, later by this one)
        const uint64_t skipw = ((Xw & 31) && (wv > 0 || pend)) ? (Xw >> 5) : ~0ull;
        uint32_t prev = (wv == 0) ? __builtin_amdgcn_readfirstlane(misc[10]) : 0u;
        // HIST: bytes at or past the chain's last byte are padding
        const HistCountT<HR> hc{hl, chain_last ? (start_bit + excl + A + 7) / 8 : ~0ull, uint32_t(lane % HR)};
        auto count = [&](uint64_t gw, uint32_t v) {
            if constexpr (HIST) hc(gw, v);
        };
        // pair 0 is stored as soon as the tile's position is known; the region then takes pair 1
        // (one wave's LDS operations complete in order)
        auto store_pair = [&](uint32_t S0, uint32_t n) {
            if (!n) return;
            const uint64_t Xb = Xw + S0;
            const uint32_t nw = uint32_t(((Xb + n) >> 5) - (Xb >> 5));
            if constexpr (HIST) store_slot(out, reg, Xb, nw, ((Xb >> 5) == skipw) ? 1u : 0u, prev, lane, hc);
            else store_slot(out, reg, Xb, nw, ((Xb >> 5) == skipw) ? 1u : 0u, prev, lane);
            prev = slot_tail32(reg, n, prev);
        };
        if constexpr (HIST) {
            if (wv == 0 && chain_pos == 0)  // the words before the first record word: the caller's header
                for (uint32_t i = lane; i < uint32_t(start_bit >> 5); i += 64) hc(i, out[i]);
        }
        store_pair(0u, S2);
        WSTAMP(9);
    asm volatile("; PHASE w9" ::: "memory");
        if (Tw > S2) {
            wave_sync();  // pair 0's image has been read
            zero_img(Tw - S2);
            wave_sync();
            emit_slot(2);
            emit_slot(3);
            wave_sync();
            store_pair(S2, Tw - S2);
        }
        const uint64_t E = Xw + Tw;
        const uint32_t e = uint32_t(E) & 31u;
        if (lane == 0) {
            if (e && (wv < wlast || chain_last)) {  // the wave's last, partial word
                const uint32_t v = bswap32((prev << (32u - e)) | (wv < wlast ? misc[4 + wv + 1] >> e : 0u));
                out[E >> 5] = v;
                count(E >> 5, v);
            }
            if (wv == wlast) publish(a.st, t, 2, a.tag, prev);  // the tile's last 32 bits
            if (wv == 0 && pend) {  // the first word, with the predecessor's tail
                const uint32_t pt = wait_tail(a.st, t - step, a.tag, a.err);
                const uint32_t s = uint32_t(Xw) & 31u;
                const uint32_t v = bswap32((pt << (32u - s)) | (misc[4] >> s));
                out[Xw >> 5] = v;
                count(Xw >> 5, v);
            }
        }
        WSTAMP(10);
        WRTSTAMP(15);
    asm volatile("; PHASE w10" ::: "memory");
    }
    if constexpr (HIST) {
        lds_barrier();  // every wave's bytes counted
        uint32_t c = 0;
#pragma unroll
        for (int r = 0; r < HR; r++) c += hl[tid * HR + r];
        if (c) atomicAdd(&a.hist[size_t(frame) * 256 + tid], c);
    }
}

// =============================================================================================
// encode4p_kernel -- encode4w_kernel's tile (wave-local slots, the same emission, look-back and
// store) with the integer half of the transform on the matrix pipe.  One workgroup per tile, the
// tiles in dispatch order (ticket mode, the host's fallback after a look-back timeout, runs
// encode4w_kernel).
//   * Matrix pipe: per slot (64 blocks of one wave), ONE v_mfma_i32_32x32x32_i8 forms the sixteen
//     integer basis sums J of every block (ie_dct.h quot4j: pixels as signed bytes x ^ 0x80, the
//     {-1,0,1} A fragment from EncTables::mfma_w), which replaces the 16 pixel unpacks and the
//     integer butterflies on the VALU; the FP32 stage (36 mul/fma) and the rounding follow, with
//     the tie limits of quot4j's own tracked run (lim4j).  The FP64 fix-up, sizing, emission and
//     store are encode4w_kernel's.
//   * Count by polling: each wave stores its bit count and a flag; wave 0 alone waits for the
//     four flags, publishes the tile aggregate and issues its look-back probe, while waves 1-3 go
//     straight on to their emission.  One workgroup barrier per tile (the position).
//   * Whole-wave images: when a wave's image fits its 4 KB region, all four slots are emitted
//     before the position barrier, beside wave 0's look-back; slot pairs in turn otherwise.
// Measured and not kept: a persistent grid walking the tiles -- by per-chain claim
// atomics (126.7 against 93.5 us) or in static order g, g + G, ... (110.3 against 88.4 us: a tile
// whose chain predecessor sits in a slower workgroup waits for it, where the dispatcher starts
// tiles in chain order as slots free) --, a software-pipelined persistent variant with two buffers
// per wave (126.7 against 93.6 us: four tiles per CU instead of six), an L2 prefetch of the tile
// about d dispatches later (neutral at d = 256-1024 on HBM-resident frames).
// =============================================================================================
constexpr int kPWfrag = 256;  // the matrix-pipe A fragments [64 lanes][4 words]
// encode4p_kernel's misc words: [0, 4) wave bit counts, H the waves' head words, E the tile's
// exclusive prefix (2), PT the tail before the chain start, PD the pending first word, F the
// count flags, D the deep look-back sums (2 per wave), FD their found flags
struct PMisc {
    static constexpr int H = 4, E = 8, PT = 10, PD = 11, F = 16, D = 20, FD = 28, S = 32;
    static_assert(FD + 4 <= S && F % 4 == 0, "misc layout");
};
constexpr int p_lds_bytes() { return (4 * 4 * 256 + 4 * kWTask + PMisc::S + kPWfrag) * 4 + kWRows * 8; }

typedef int v4i32 __attribute__((ext_vector_type(4)));
typedef int v16i32 __attribute__((ext_vector_type(16)));

// round_block_lean4 with the limits passed in (quot4j's own)
__device__ __forceinline__ float round_block_lean4j(const float (&t)[16], uint32_t (&zp)[8], uint32_t* sflags, bool dcx,
                                                    float l0, float l1, float l2) {
    constexpr int S0 = Structural<4>::k[0], S1 = Structural<4>::k[1], S2 = Structural<4>::k[2];
    float emax = 0.0f;
    uint32_t sf = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        uint32_t yb[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int k = ZigZag<4>::idx[2 * j + h];
            const float y = t[k] + kMagic;
            const float e = fabsf(t[k] - (y - kMagic));
            yb[h] = __float_as_uint(y);
            if (k == 0) {
                const uint32_t dc = uint32_t(int(truncf(t[0] + copysignf(0.5f, t[0]))));
                yb[h] = dcx ? dc : yb[h];
                emax = dcx ? emax : fmaxf(emax, e);
            } else if (k == S0) {
                sf |= (e >= l0) ? 1u : 0u;
            } else if (k == S1) {
                sf |= (e >= l1) ? 2u : 0u;
            } else if (k == S2) {
                sf |= (e >= l2) ? 4u : 0u;
            } else {
                emax = fmaxf(emax, e);
            }
        }
        zp[j] = __builtin_amdgcn_perm(yb[1], yb[0], 0x05040100u);
        asm volatile("" : "+v"(zp[j]));
    }
    *sflags = sf;
    return emax;
}

#ifndef IE_P_PXAUX
#define IE_P_PXAUX 2  // cache-policy bits of encode4p's pixel DMA: nt (pixels are read once; HBM-resident
                      // frames 98.2 against 101.1 us per 16-frame launch, MALL-resident 97.9 against 92.8)
#endif
#ifndef IE_P_WAVES
#define IE_P_WAVES 6  // __launch_bounds__ occupancy hint (waves per SIMD)
#endif
#ifndef IE_P_WAVES_HIST
#define IE_P_WAVES_HIST 6  // the counting instantiation (5: 89 VGPRs; measured 124.7 against 119.4 us)
#endif
#ifndef IE_P_ABL
#define IE_P_ABL 0  // (profiling builds) phases left out: 1 FP64 fix-up, 2 emission, 4 look-back, 8 store, 16 transform
#endif

template <bool HIST>
__global__ __launch_bounds__(256, HIST ? IE_P_WAVES_HIST : IE_P_WAVES) void encode4p_kernel(EncArgs a_, const EncTables* __restrict__ tab) {
    constexpr int N = 4, NN = 16, NP = 8, NS = 4, PS = 2;  // slots per lane, slots per pair
    constexpr int GW = 64, BW = 256, TG = 256;  // groups / blocks per wave, groups per tile
    constexpr int RW = 4 * BW;  // words per wave region
    using ML = PMisc;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int wv = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
    uint32_t* const reg = smem + wv * RW;  // this wave's pixels, later its slot images
    uint32_t* const task = smem + 4 * RW + wv * kWTask;
    uint32_t* const res = task + 64;
    uint32_t* const misc = smem + 4 * RW + 4 * kWTask;  // [ML::S]
    uint32_t* const wl = misc + ML::S;  // [64][4]: the matrix-pipe A fragment of every lane
    uint32_t* const hl = wl + kPWfrag;  // HIST: the tile's byte histogram
    constexpr int HR = kWHistRep, HWORDS = 256 * HR;
    double* const srow = reinterpret_cast<double*>(hl + (HIST ? HWORDS : 0));
    const int t = int(blockIdx.x);
    // The launch arguments are read through a pointer to the kernel-argument segment (constant
    // address space): the geometry words in one scalar round trip (load_geo), the rest where used.
    using KArgs = const __attribute__((address_space(4))) EncArgs;
    KArgs* ka = (KArgs*)(__builtin_amdgcn_kernarg_segment_ptr());
    const GeoArgs ga = load_geo(ka);
    if (t >= ga.ntiles) return;
    // The lane id is re-derived at every phase (fresh_lane): a lane-derived VGPR held across the
    // whole tile was spilled at higher occupancy.
    int lane = fresh_lane();
    // (profiling: the workgroup's entry on the chip-wide clock, wave 0's word 13)
    if (IE_PROFILE && a_.stamps && lane == 0) a_.stamps[size_t(t) * kStamps + wv * 16 + 13] = __builtin_amdgcn_s_memrealtime();
    const TileGeo g = tile_geo<4, 4, TG>(ga, t, GW * wv + lane);
    // the wave's pixel rows into its own region (row r of the wave's block j at reg[r BW + j]: a
    // lane's 16 bytes are its group's row)
    if (g.nblk) {
        const uint8_t* base = ga.y + size_t(g.frame) * ga.frame_pitch + size_t(g.byi) * N * ga.stride + size_t(g.bx0) * N;
#pragma unroll
        for (int r = 0; r < N; r++)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + size_t(r) * ga.stride),
                                             (__attribute__((address_space(3))) void*)(reg + r * BW), 16, 0, IE_P_PXAUX);
    }
    if (IE_PROFILE == 2 && a_.stamps && lane == 0) a_.stamps[size_t(t) * kStamps + wv * 16 + 1] = __builtin_amdgcn_s_memrealtime();
    // the FP64 rows (waves 0-2: 2432 bytes) and the matrix-pipe A fragments (wave 3; read back per
    // slot) by DMA too: no register round trip, one wait for everything
    {
        static_assert(kWRows * 8 == 2 * 1024 + 24 * 16, "rows: two full waves and 24 lanes of 16 bytes");
        if (wv < 2 || (wv == 2 && lane < 24))
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(&tab->rows4[wv * 128 + 2 * lane]),
                                             (__attribute__((address_space(3))) void*)(srow + wv * 128), 16, 0, 0);
        else if (wv == 3)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(&tab->mfma_w[lane][0]),
                                             (__attribute__((address_space(3))) void*)(wl), 16, 0, 0);
    }
    if constexpr (HIST)
        for (int i = 64 * wv + lane; i < HWORDS; i += 256) hl[i] = 0u;
    if (lane == 0) misc[ML::F + wv] = 0u;  // the waves' count flags
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the DMA above and this wave's pixels)
    if (IE_PROFILE && a_.stamps && lane == 0) a_.stamps[size_t(t) * kStamps + wv * 16 + 12] = __builtin_amdgcn_s_memrealtime();
    const uint64_t start_bit = a_.start_dev ? *a_.start_dev : a_.start_bit;
    const bool deep = a_.deep_lb != 0;
    lds_barrier();  // every wave's pixels, the rows, the A fragments (and the HIST bins) visible
    if (IE_PROFILE && a_.stamps && lane == 0) a_.stamps[size_t(t) * kStamps + wv * 16 + 11] = __builtin_amdgcn_s_memrealtime();
    KArgs& a = *ka;
    // (the tile's geometry is uniform: held in SGPRs, not in VGPRs the compiler would keep -- and
    // spill -- across the tile)
    const int frame = __builtin_amdgcn_readfirstlane(g.frame), tif = __builtin_amdgcn_readfirstlane(g.tif),
              step = __builtin_amdgcn_readfirstlane(g.step), chain_pos = __builtin_amdgcn_readfirstlane(g.chain_pos);
    const int ng = min(TG, ga.groups_per_frame - tif * TG);
    const int nbw = __builtin_amdgcn_readfirstlane(4 * min(GW, max(0, ng - GW * wv)));  // blocks of this wave
    const int wlast = (ng - 1) / GW;                    // the tile's last non-empty wave
    WSTAMP(0);
    WRTSTAMP(14);
    if (IE_PROFILE != 2) WSTAMP(1);
    asm volatile("; PHASE p1" ::: "memory");

    // ------------------------------------------------------------ transform + quantise, 4 slots
    using KTab = const __attribute__((address_space(4))) EncTables;
    KTab* tb = (KTab*)(tab);  // constant address space: scalar loads
    const bool dcx = tb->dc_exact4j != 0;
    const float lim_s0 = tb->lim4j[Structural<4>::k[0]], lim_s1 = tb->lim4j[Structural<4>::k[1]],
                lim_s2 = tb->lim4j[Structural<4>::k[2]], lim_min = tb->lim_min4j;
    uint32_t zp[NS][NP];
    uint32_t flags = 0;  // 4 bits per slot: structural s (bits 0-2), whole block (bit 3)
#pragma unroll
    for (int b = 0; b < NS; b++) {
        __builtin_amdgcn_sched_barrier(0);
        uint32_t sf;
        float emax;
        if (IE_P_ABL & 16) {  // (profiling) no transform: quotients = pixels / 64
            float x[NN];
#pragma unroll
            for (int k = 0; k < NN; k++) x[k] = float((reg[(k >> 2) * BW + 64 * b + lane] >> (8 * (k & 3))) & 0xFFu) * 0.015625f;
            emax = round_block_lean4j(x, zp[b], &sf, dcx, lim_s0, lim_s1, lim_s2);
        } else {
            v4i32 px;
#pragma unroll
            for (int r = 0; r < N; r++) px[r] = int(reg[r * BW + 64 * b + lane] ^ 0x80808080u);  // x - 128 as i8
            const v4i32 wfrag = *reinterpret_cast<const v4i32*>(wl + 4 * lane);
            const v16i32 Jc = __builtin_amdgcn_mfma_i32_32x32x32_i8(wfrag, px, v16i32{}, 0, 0, 0);
            float Jf[16], x[16];
#pragma unroll
            for (int k = 0; k < 16; k++) Jf[k] = float(Jc[k]);
            quot4j(Jf, x, tb->plan4j, FloatOp());
            emax = round_block_lean4j(x, zp[b], &sf, dcx, lim_s0, lim_s1, lim_s2);
        }
        const uint32_t fb = (emax >= lim_min) ? 8u : sf;
        if (64 * b + lane < nbw) flags |= fb << (4 * b);
#pragma unroll
        for (int j = 0; j < NP; j++) asm volatile("" : "+v"(zp[b][j]));
        asm volatile("" : "+v"(flags));
    }
    WSTAMP(2);
    asm volatile("; PHASE p2" ::: "memory");

    // ------------------------------------------------------------ FP64 fix-up (encode4w_kernel's)
    lane = fresh_lane();
    auto block_px = [&](int b, int owner) {
        BlockPx<N> px;
#pragma unroll
        for (int r = 0; r < N; r++) px.w[r] = reg[r * BW + 64 * b + owner];
        return px;
    };
    if (!(IE_P_ABL & 1) && __ballot(flags != 0)) {
        const uint32_t sf = flags & 0x7777u;
        const uint32_t cnt = __popc(sf);
        // the lanes' request counts placed by one DPP wave scan
        const uint32_t incl = wave_incl_scan_dpp(cnt);
        const uint32_t pre = incl - cnt;
        const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
        for (uint32_t r0 = 0; r0 < total; r0 += 64) {
            uint32_t m = sf, i = pre - r0;
            while (m) {
                const int bit = __ffs(m) - 1;
                m &= m - 1;
                if (i < 64u) task[i] = (uint32_t(lane) << 4) | uint32_t(bit);
                i++;
            }
            wave_sync();
            if (uint32_t(lane) < total - r0) {
                const uint32_t tk = task[lane];
                const int s = int(tk & 3u), b = int((tk >> 2) & 3u), owner = int(tk >> 4);
                const BlockPx<N> px = block_px(b, owner);
                const int k = Structural<N>::k[0] * (s == 0) + Structural<N>::k[1] * (s == 1) + Structural<N>::k[2] * (s == 2);
                const int y = (IE_P_ABL & 32) ? int(px.w[0] & 1u)  // (profiling) no FP64 arithmetic (a small value: records stay in bound)
                                              : exact_coef_row<N>(srow + k * NN, srow[NN * NN + k], srow[NN * NN + NN + k],
                                                                  srow[NN * NN + 2 * NN + k], px);
                res[lane] = uint32_t(y) & 0xFFFFu;
            }
            wave_sync();
            i = pre - r0;
#pragma unroll
            for (int b = 0; b < NS; b++)
#pragma unroll
                for (int ss = 0; ss < 3; ss++) {
                    if ((sf >> (4 * b + ss)) & 1u) {
                        const int zw = Structural<N>::zpos(ss) >> 1;
                        if (i < 64u) zp[b][zw] = __builtin_amdgcn_perm(res[i], zp[b][zw], 0x05040100u);  // res low -> high half
                        i++;
                    }
                }
            wave_sync();
        }
        const uint32_t wf = flags & 0x8888u;
        if (__ballot(wf != 0)) {
            const uint32_t nb = __popc(wf);
            uint32_t pb = 0, tb = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) {  // nb <= 4
                const uint64_t bm = __ballot((nb >> k) & 1u);
                pb += __builtin_amdgcn_mbcnt_hi(uint32_t(bm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(bm), 0u)) << k;
                tb += uint32_t(__popcll(bm)) << k;
            }
            for (uint32_t r0 = 0; r0 < tb; r0 += 4) {
                uint32_t m = wf, j = pb - r0;
                while (m) {
                    const int b = (__ffs(m) - 1) >> 2;
                    m &= m - 1;
                    if (j < 4u) task[j] = (uint32_t(lane) << 4) | uint32_t(b);
                    j++;
                }
                wave_sync();
                if (uint32_t(lane >> 4) < tb - r0) {
                    const uint32_t tk = task[lane >> 4];
                    const int b = int(tk & 3u), owner = int(tk >> 4), k = lane & 15;
                    const BlockPx<N> px = block_px(b, owner);
                    const int y = exact_coef_row<N>(srow + k * NN, srow[NN * NN + k], srow[NN * NN + NN + k],
                                                    srow[NN * NN + 2 * NN + k], px);
                    res[lane] = uint32_t(y) & 0xFFFFu;
                }
                wave_sync();
                m = wf;
                j = pb - r0;
                while (m) {
                    const int b = (__ffs(m) - 1) >> 2;
                    m &= m - 1;
                    if (j < 4u) {
                        const uint32_t* rr = res + 16 * j;
#pragma unroll
                        for (int jj = 0; jj < NP; jj++) {
                            const uint32_t w = rr[ZigZag<N>::idx[2 * jj]] | (rr[ZigZag<N>::idx[2 * jj + 1]] << 16);
#pragma unroll
                            for (int bb = 0; bb < NS; bb++) zp[bb][jj] = (b == bb) ? w : zp[bb][jj];
                        }
                    }
                    j++;
                }
                wave_sync();
            }
        }
    }
    {  // statistics: FP64 requests of this wave (one store)
        const uint32_t wsum = __builtin_amdgcn_readlane(wave_incl_scan_dpp(uint32_t(__popc(flags))), 63);
        if (lane == 0) a.wave_fix[size_t(t) * 4 + wv] = wsum;
    }
    WSTAMP(3);
    asm volatile("; PHASE p3" ::: "memory");

    // ------------------------------------------------------------ sizing + the wave's offsets
    lane = fresh_lane();
    uint32_t blw[NS], rb[NS];
    const uint32_t k0 = uint32_t(tif * TG + GW * wv) * 4u;  // the wave's first block (frame raster order)
#pragma unroll
    for (int b = 0; b < NS; b++) {
        const bool valid = 64 * b + lane < nbw;
        if (a.coef && valid) {
            int16_t* dst = a.coef + (size_t(frame) * a.by * a.bx + k0 + 64 * b + lane) * NN;
#pragma unroll
            for (int k = 0; k < NN; k++) {
                const int kz = ZigZagInv<N>::pos[k];
                dst[k] = int16_t(kz & 1 ? (zp[b][kz >> 1] >> 16) : (zp[b][kz >> 1] & 0xFFFFu));
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        blw[b] = size_block4(zp[b], a.rle, &rb[b]);
        rb[b] = valid ? rb[b] : 0u;
        asm volatile("" : "+v"(blw[b]), "+v"(rb[b]));
#pragma unroll
        for (int j = 0; j < NP; j++) asm volatile("" : "+v"(zp[b][j]));
        __builtin_amdgcn_sched_barrier(0);
    }
    uint32_t T[NS], off[NS];
#pragma unroll
    for (int h = 0; h < NS / 2; h++) {  // two slots per 32-bit scan (16-bit halves)
        const uint32_t sv = rb[2 * h] | (rb[2 * h + 1] << 16);
        const uint32_t iv = wave_incl_scan_dpp(sv);
        const uint32_t tv = __builtin_amdgcn_readlane(iv, 63), ev = iv - sv;
        T[2 * h] = tv & 0xFFFFu;
        T[2 * h + 1] = tv >> 16;
        off[2 * h] = ev & 0xFFFFu;
        off[2 * h + 1] = ev >> 16;
    }
    uint32_t Sb[NS];  // slot starts in the wave image
    Sb[0] = 0u;
#pragma unroll
    for (int b = 1; b < NS; b++) Sb[b] = Sb[b - 1] + T[b - 1];
    const uint32_t Tw = Sb[NS - 1] + T[NS - 1];
    const uint32_t S2 = Sb[2];  // the end of slot pair 0
    // The tile's bit count: wave 0 alone waits for the four waves' counts (their flags, cleared
    // before the tile) and publishes it; the other waves go on to their emission and learn their
    // place in the tile after the position barrier.  (A launch too small to fill the chip -- deep
    // look-back -- keeps a workgroup barrier here: all four waves read predecessor windows.)
    if (lane == 0) {
        misc[wv] = Tw;
        __hip_atomic_store(&misc[ML::F + wv], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    WSTAMP(4);
    asm volatile("; PHASE p4" ::: "memory");
    if (deep) {
        lds_barrier();
    } else if (wv == 0) {
        for (;;) {
            const u32x4 f = *reinterpret_cast<const volatile u32x4*>(misc + ML::F);
            if (__builtin_amdgcn_readfirstlane(f.x & f.y & f.z & f.w)) break;
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    WSTAMP(5);
    asm volatile("; PHASE p5" ::: "memory");

    lane = fresh_lane();
    uint32_t A = 0;  // (wave 0, or every wave in deep mode; the others after the position barrier)
#pragma unroll
    for (int w = 0; w < 4; w++) A += __builtin_amdgcn_readfirstlane(misc[w]);
    if (wv == 0 && lane == 0) chain_publish_count(a.st, t, chain_pos, a.tag, A);
    constexpr int DW = 2;
    Probe pr[DW];
#pragma unroll
    for (int i = 0; i < DW; i++) pr[i] = Probe{0, 0, 0};
    if (chain_pos != 0) {
        if (deep) {
#pragma unroll
            for (int i = 0; i < DW; i++) pr[i] = probe_issue(a.st, t, chain_pos, step, 64 * (DW * wv + i), 64);
        } else if (wv == 0 && !(IE_P_ABL & 4)) {  // (look-back left out: no probe either)
            pr[0] = probe_issue(a.st, t, chain_pos, step, 0, kProbe0);
        }
    }

    const uint32_t reg_bit0 = uint32_t(wv * RW) * 32u;
    auto zero_img = [&](uint32_t bits) {
        const uint32_t nq = (bits + 127u) >> 7;  // 16-byte groups
        uint32_t z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));  // (a hoisted zero vector was spilled)
        for (uint32_t q = lane; q < nq; q += 64) *reinterpret_cast<u32x4*>(reg + 4 * q) = u32x4{z, z, z, z};
    };
    // The wave's whole image fits its region (the last record's trailing zero fields reach at
    // most rec_bits past its start, plus the 64-bit window): all four slots are emitted before
    // the position barrier -- beside wave 0's look-back -- and stored in one pass after it.
    // Otherwise slot pairs in turn (pair 1 after pair 0 is stored).
    const bool whole = Tw + uint32_t(a.rec_bits) + 64u <= 32u * RW;
    auto emit_slot = [&](int b) {  // slot b at its place in the (whole or pair) image
        if (!(IE_P_ABL & 2) && rb[b]) {
            const uint32_t p = reg_bit0 + (whole ? Sb[b] : Sb[b] - Sb[(b / PS) * PS]) + off[b];
            if (a.tri && a.rle) emit_block3(smem, p, zp[b], blw[b]);
            else emit_block2<N>(smem, p, zp[b], blw[b], a.rle);
        }
    };
    zero_img(whole ? Tw : S2);
    wave_sync();
#pragma unroll
    for (int b = 0; b < PS; b++) emit_slot(b);
    if (whole) {
#pragma unroll
        for (int b = PS; b < NS; b++) emit_slot(b);
    }
    wave_sync();
    WSTAMP(6);
    asm volatile("; PHASE p6" ::: "memory");
    if (lane == 0 && Tw) misc[ML::H + wv] = reg[0];  // the wave's first 32 bits

    // ------------------------------------------------------------ look-back (wave 0)
    lane = fresh_lane();
    const bool chain_last = a.segmented ? (tif == a.tiles_per_frame - 1) : (t == a.ntiles - 1);
    uint32_t* const out = a.out + (a.segmented ? uint64_t(frame) * a.out_pitch_words : 0ull);
    if (deep && chain_pos != 0) {
        uint64_t sm = 0;
        bool found = false;
        unsigned spins = 0;
        for (;;) {
            bool ready = true;
            sm = 0;
            found = false;
#pragma unroll
            for (int i = 0; i < DW; i++) {
                const WinSum r = window_sum(pr[i], chain_pos, 64 * (DW * wv + i), 64, a.tag);
                if (!found) {
                    ready = ready && r.ready;
                    sm += r.sum;
                    found = r.found;
                }
            }
            if (ready) break;
            if (++spins > kSpinLimit) {
                if (lane == 0) atomicAdd(&a.err[0], 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int i = 0; i < DW; i++) pr[i] = probe_issue(a.st, t, chain_pos, step, 64 * (DW * wv + i), 64);
        }
        if (lane == 0) {
            misc[ML::D + 2 * wv] = uint32_t(sm);
            misc[ML::D + 2 * wv + 1] = uint32_t(sm >> 32);
            misc[ML::FD + wv] = found ? 1u : 0u;
        }
        lds_barrier();
    }
    if (wv == 0) {
        uint64_t excl = 0;
        uint32_t ptail = 0, pend = 0;
        if (chain_pos == 0) {
            const uint32_t s = uint32_t(start_bit & 31);
            ptail = s ? (bswap32(out[start_bit >> 5]) >> (32 - s)) : 0u;
        } else {
            bool done = false;
            if (deep) {
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    if (!done) {
                        excl += uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(misc[ML::D + 2 * w]))) |
                                (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(misc[ML::D + 2 * w + 1]))) << 32);
                        done = __builtin_amdgcn_readfirstlane(misc[ML::FD + w]) != 0;
                    }
                }
                if (!done) excl = 0;
            }
            if (!done) {
                const Probe p0 = deep ? probe_issue(a.st, t, chain_pos, step, 0, kProbe0) : pr[0];
                excl = (IE_P_ABL & 4) ? uint64_t(chain_pos) * 30000u
                                      : lookback_wave<IE_W_AHEAD, IE_W_LBW>(p0, a.st, t, chain_pos, step, a.tag, a.err, nullptr, deep);
            }
            const bool have = uint32_t(pr[0].gt >> 56) == a.tag;
            const bool split = ((start_bit + excl) & 31) != 0;
            ptail = have ? uint32_t(pr[0].gt) : 0u;
            pend = (!have && split) ? 1u : 0u;
        }
        if (lane == 0) {
            if (chain_pos != 0) publish(a.st, t, 1, a.tag, excl + A);
            misc[ML::E] = uint32_t(excl);
            misc[ML::E + 1] = uint32_t(excl >> 32);
            misc[ML::PT] = ptail;
            misc[ML::PD] = pend;
            const uint64_t P = start_bit + excl;
            if (tif == 0) a.frame_start[frame] = P;
            if (chain_last) a.chain_end[a.segmented ? frame : 0] = P + A;
        }
    }
    WSTAMP(7);
    asm volatile("; PHASE p7" ::: "memory");
    lds_barrier();  // ---- the tile's position
    WSTAMP(8);
    asm volatile("; PHASE p8" ::: "memory");
    lane = fresh_lane();
    uint32_t W = 0;
    A = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint32_t v = __builtin_amdgcn_readfirstlane(misc[w]);
        A += v;
        W += (w < wv) ? v : 0u;
    }

    // ------------------------------------------------------------ store, slot pair by slot pair
    if (Tw) {
        const uint64_t excl = uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(misc[ML::E]))) |
                              (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(misc[ML::E + 1]))) << 32);
        const uint64_t Xw = start_bit + excl + W;
        const bool pend = __builtin_amdgcn_readfirstlane(misc[ML::PD]) != 0u;
        const uint64_t skipw = ((Xw & 31) && (wv > 0 || pend)) ? (Xw >> 5) : ~0ull;
        uint32_t prev = (wv == 0) ? __builtin_amdgcn_readfirstlane(misc[ML::PT]) : 0u;
        const HistCountT<HR> hc{hl, chain_last ? (start_bit + excl + A + 7) / 8 : ~0ull, uint32_t(lane % HR)};
        auto count = [&](uint64_t gw, uint32_t v) {
            if constexpr (HIST) hc(gw, v);
        };
        auto store_pair = [&](uint32_t S0, uint32_t n) {
            if (!n || (IE_P_ABL & 8)) return;
            const uint64_t Xb = Xw + S0;
            const uint32_t nw = uint32_t(((Xb + n) >> 5) - (Xb >> 5));
            if constexpr (HIST) store_slot(out, reg, Xb, nw, ((Xb >> 5) == skipw) ? 1u : 0u, prev, lane, hc);
            else store_slot(out, reg, Xb, nw, ((Xb >> 5) == skipw) ? 1u : 0u, prev, lane);
            prev = slot_tail32(reg, n, prev);
        };
        if constexpr (HIST) {
            if (wv == 0 && chain_pos == 0)
                for (uint32_t i = lane; i < uint32_t(start_bit >> 5); i += 64) hc(i, out[i]);
        }
        const uint64_t E = Xw + Tw;
        const uint32_t e = uint32_t(E) & 31u;
        store_pair(0u, whole ? Tw : S2);
        WSTAMP(9);
        asm volatile("; PHASE p9" ::: "memory");
        if (!whole && Tw > S2) {
            wave_sync();  // pair 0's image has been read
            zero_img(Tw - S2);
            wave_sync();
#pragma unroll
            for (int b = PS; b < NS; b++) emit_slot(b);
            wave_sync();
            store_pair(S2, Tw - S2);
        }
        const uint32_t nexthead = (e && wv < wlast) ? misc[ML::H + wv + 1] : 0u;
        if (lane == 0) {
            if (e && (wv < wlast || chain_last)) {  // the wave's last, partial word
                const uint32_t v = bswap32((prev << (32u - e)) | (nexthead >> e));
                out[E >> 5] = v;
                count(E >> 5, v);
            }
            if (wv == wlast) publish(a.st, t, 2, a.tag, prev);  // the tile's last 32 bits
            if (wv == 0 && pend) {  // the first word, with the predecessor's tail
                const uint32_t pt = wait_tail(a.st, t - step, a.tag, a.err);
                const uint32_t s = uint32_t(Xw) & 31u;
                const uint32_t v = bswap32((pt << (32u - s)) | (misc[ML::H] >> s));
                out[Xw >> 5] = v;
                count(Xw >> 5, v);
            }
        }
        WSTAMP(10);
        asm volatile("; PHASE p10" ::: "memory");
        WRTSTAMP(15);
    }
    if constexpr (HIST) {
        lds_barrier();  // every wave's bytes counted
        uint32_t c = 0;
        const int th = 64 * wv + fresh_lane();
#pragma unroll
        for (int r = 0; r < HR; r++) c += hl[th * HR + r];
        if (c) atomicAdd(&a.hist[size_t(frame) * 256 + th], c);
    }
}

// Returns the FP64-statistics words per tile the launched kernel writes (its waves per tile).
int launch_encode4w(const EncArgs& a, hipStream_t s) {
    if (!a.ticket) {  // dispatch order: encode4p_kernel, one workgroup per tile
        const size_t lds = p_lds_bytes() + (a.hist ? 1024 * kWHistRep : 0);
        if (a.hist) hipLaunchKernelGGL(encode4p_kernel<true>, dim3(a.ntiles), dim3(256), lds, s, a, a.tab);
        else hipLaunchKernelGGL(encode4p_kernel<false>, dim3(a.ntiles), dim3(256), lds, s, a, a.tab);
        return 4;
    }
    // ticket mode (the host's redo after a look-back timeout): tiles in ticket order
    if (a.hist) hipLaunchKernelGGL(encode4w_kernel<true>, dim3(a.ntiles), dim3(256), kWLdsBytes + 1024 * kWHistRep, s, a, a.tab);
    else hipLaunchKernelGGL(encode4w_kernel<false>, dim3(a.ntiles), dim3(256), kWLdsBytes, s, a, a.tab);
    return 4;
}

// The streamed host path's per-image header words: word i (read from page-locked host memory
// the device maps, one PCIe read per image) to dst[i * pitch_words] -- instead of an SDMA copy
// that would queue behind the chunk's pixel upload on the copy engine.
__global__ void word_scatter_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint64_t pitch_words,
                                    int n) {
    const int i = int(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) dst[size_t(i) * pitch_words] = src[i];
}

void launch_word_scatter(const uint32_t* src, uint32_t* dst, uint64_t pitch_words, int n, hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(word_scatter_kernel, dim3(unsigned((n + 63) / 64)), dim3(64), 0, s, src, dst, pitch_words, n);
}

int encode_blocks_per_thread(int n) { return n == 4 ? Geo<4>::BPT : Geo<8>::BPT; }
#ifndef IE_SMALL_TILES
#define IE_SMALL_TILES 1024
#endif
int encode_small_tiles() {
    static const char* e = getenv("IE_SMALL_TILES");  // (A/B aid: 0 disables the small-launch geometry)
    static const int v = e ? atoi(e) : IE_SMALL_TILES;
    return v;
}

int encode_threads_per_tile() { return kEncTPB; }

int launch_encode4w(const EncArgs& a, hipStream_t s);

int launch_encode(const EncArgs& a0, int n, bool exact, hipStream_t s, int bpt) {
    EncArgs a = a0;
    // 4x4 FAST over whole 16-byte groups: the wave-local encoders (encode4p_kernel)
    if (n == 4 && !exact && bpt == 4 && a.vec_ok && a.bx % 4 == 0 &&
        a.groups_per_frame % 8 == 0 && a.rec_bits <= 252 && !a.ablate)
        return launch_encode4w(a, s);
    a.img_words = image_words_for(n, bpt, a.rec_bits);
    if (n == 4 && a.img_words < fix_words<4>()) a.img_words = fix_words<4>();
    if (n == 8 && a.img_words < kFix8Words) a.img_words = kFix8Words;
    const size_t rows = exact ? 0 : (n == 4 ? size_t(n * n * n * n + 3 * n * n) : size_t(3 * n * n + 9));
    const size_t lds = (size_t(a.img_words) + 32 + (a.hist ? 256 : 0)) * sizeof(uint32_t) + rows * sizeof(double);
    const dim3 grid(a.ntiles), block(kEncTPB);
    if (a.hist) {  // segmented 4x4 FAST launches only (ie_encode_images_counted; 8x8 would spill)
        hipLaunchKernelGGL((encode_kernel<4, false, true>), grid, block, lds, s, a, a.tab);
        return kEncTPB / 64;
    }
    if (n == 4) {
        if (exact) hipLaunchKernelGGL((encode_kernel<4, true>), grid, block, lds, s, a, a.tab);
        else hipLaunchKernelGGL((encode_kernel<4, false>), grid, block, lds, s, a, a.tab);
    } else {
        if (exact) hipLaunchKernelGGL((encode_kernel<8, true>), grid, block, lds, s, a, a.tab);
        else hipLaunchKernelGGL((encode_kernel<8, false>), grid, block, lds, s, a, a.tab);
    }
    return kEncTPB / 64;
}

}  // namespace ie
