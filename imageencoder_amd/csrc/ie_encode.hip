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

#include "ie_common.cuh"
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

template <int N> struct Geo;
template <> struct Geo<4> { static constexpr int BPT = 4; };  // 16 B per pixel row per lane
template <> struct Geo<8> { static constexpr int BPT = 1; };  //  8 B per pixel row per lane

// bits-in-tile upper bound: 4 + 16 * (N*N + 1) bits per block
template <int N> constexpr int image_words() {
    return ((kTPB * Geo<N>::BPT * (4 + 16 * (N * N + 1)) + 31) / 32 + 2 + 3) / 4 * 4;  // keeps misc 16-B aligned
}

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
__device__ __noinline__ int exact_coef(const EncTables* __restrict__ tab, int k, BlockPx<N> px) {
    constexpr int NN = N * N;
    const double* P = &tab->P[k * NN];
    double acc = 0.0;
#pragma unroll
    for (int ij = 0; ij < NN; ij++) {
        const double x = double(int((px.w[ij >> 2] >> (8 * (ij & 3))) & 0xFFu)) + (-128.0);
        acc = acc + P[ij] * x;
    }
    const double D = acc * tab->S[k];
    const double rq = tab->rq[k];
    const double t = (rq != 0.0) ? D * rq : D / tab->qd[k];
    double r = trunc(t);
    if (fabs(t - r) >= 0.5) r += copysign(1.0, t);
    return int(r);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Load the pixel rows of one group: seg[r][m] = bytes [4m, 4m+4) of the group's row r.
template <int N, int WPR>
__device__ __forceinline__ void load_group(const EncArgs& a, const uint8_t* base, int nblk, uint32_t (&seg)[N][WPR]) {
    constexpr int BPT = Geo<N>::BPT;
    if (a.vec_ok && nblk == BPT) {
#pragma unroll
        for (int r = 0; r < N; r++) {
            const uint8_t* p = base + size_t(r) * a.stride;
            if constexpr (WPR == 4) {
                const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
                seg[r][0] = v.x; seg[r][1] = v.y; seg[r][2] = v.z; seg[r][3] = v.w;
            } else {
                const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
                seg[r][0] = v.x; seg[r][1] = v.y;
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

// Quantise block b of the group into zp[] (zig-zag order, two int16 per word: z[2j] in the low
// half); returns the number of coefficients re-evaluated in FP64.  The values pass through the
// thread's private LDS slot `stage` (NN int16), so the rare FP64 re-evaluations patch them at a
// runtime index without forcing a register array into scratch memory.
template <int N> using NearMask = typename std::conditional<N == 4, uint32_t, uint64_t>::type;

template <int N, int WPR>
__device__ __forceinline__ NearMask<N> quantize_block(const EncTables* __restrict__ tab, const uint32_t (&seg)[N][WPR],
                                                      int b, uint32_t (&zp)[N * N / 2]) {
    constexpr int NN = N * N;
    using Mask = NearMask<N>;
    Mask need = 0;
    float x[NN];
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
        for (int j = 0; j < N; j++) x[i * N + j] = float(pix<WPR>(seg[i], b * N + j)) - 128.0f;
    dct2d<N>(x, tab->dct, FloatOp());
    // t = D * C(u)C(v)/q; y = t + 1.5*2^23 rounds t to the nearest integer (|t| < 2^22) and leaves
    // int16(rint(t)) in y's low 16 bits; |t - rint(t)| >= 0.5 - bound flags a possible tie.
    constexpr float kMagic = 12582912.0f;
    uint32_t yb[NN];
#pragma unroll
    for (int k = 0; k < NN; k++) {
        const float t = x[k] * tab->g[k];
        if (k == 0 && tab->thr[0] < 0.0f) {
            // t is exact here (integer sum times a power of two): round half away from zero
            yb[k] = uint32_t(int(truncf(t + copysignf(0.5f, t))));
        } else {
            const float y = t + kMagic;
            const float r = y - kMagic;
            need |= Mask(fabsf(t - r) >= tab->lim[k]) << k;
            yb[k] = __float_as_uint(y);
        }
    }
#pragma unroll
    for (int j = 0; j < NN / 2; j++)
        zp[j] = __builtin_amdgcn_perm(yb[ZigZag<N>::idx[2 * j + 1]], yb[ZigZag<N>::idx[2 * j]], 0x05040100u);
    return need;
}

// Replace zig-zag coefficient kz of a packed block by v (a runtime position: a select chain over
// the words, so the block stays in registers).
template <int NP>
__device__ __forceinline__ void patch(uint32_t (&zp)[NP], int kz, uint32_t v) {
    const int wsel = kz >> 1;
    const uint32_t lo = v & 0xFFFFu, hi = v << 16;
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const uint32_t w = zp[j];
        const uint32_t nw = (kz & 1) ? ((w & 0xFFFFu) | hi) : ((w & 0xFFFF0000u) | lo);
        zp[j] = (j == wsel) ? nw : w;
    }
}

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Zig-zag RLE sizing of one packed block (Block.cpp:186-232, :383-397), two coefficients per
// packed-int16 instruction.  Returns bl | Lw << 8 and the record length in bits.
template <int N>
__device__ __forceinline__ uint32_t size_block(const uint32_t (&zp)[N * N / 2], int rle, uint32_t* bits) {
    constexpr int NN = N * N;
    constexpr int NP = NN / 2;
    // nz: bit kz set iff z[kz] != 0 (min(u16, 1) per half, even kz in the low halves)
    uint64_t nz = 0;
    uint32_t mo = 0;  // OR of v ^ (v >> 15) per half: its bit length + 1 is the widest bits_needed
#pragma unroll
    for (int g = 0; g < NP / 8; g++) {
        uint32_t M = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t w = zp[g * 8 + j];
            const u16x2 m = __builtin_elementwise_min(__builtin_bit_cast(u16x2, w), u16x2{1, 1});
            M |= __builtin_bit_cast(uint32_t, m) << (2 * j);
            const s16x2 v = __builtin_bit_cast(s16x2, w);
            mo |= __builtin_bit_cast(uint32_t, v ^ (v >> s16x2{15, 15}));
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
    } else {
        lw = L;
    }
    *bits = 4u + uint32_t(bl) * uint32_t(lw + rle);
    return uint32_t(bl) | (uint32_t(lw) << 8);
}

template <int N, bool EXACT>
__global__ __launch_bounds__(kTPB, 4) void encode_kernel(EncArgs a, const EncTables* __restrict__ tab) {
    constexpr int NN = N * N;
    constexpr int BPT = Geo<N>::BPT;
    constexpr int WPR = BPT * N / 4;
    constexpr int IMGW = image_words<N>();
    __shared__ uint32_t smem[IMGW + 32];
    uint32_t* img = smem;
    uint32_t* misc = smem + IMGW;  // [0..3] scan, [4] ticket, [5..6] excl, [7] pred tail, [8..31] look-back

    const int tid = threadIdx.x;
    // Tile order = dispatch order.  Workgroups are dispatched in increasing blockIdx per XCD, so
    // every predecessor of a resident tile is resident or done and the look-back cannot deadlock;
    // the bounded spins report (never hang) should that ever not hold, and the host then re-runs
    // with an atomic ticket (a.ticket != nullptr), which orders tiles explicitly.
    int t;
    if (a.ticket) {
        if (tid == 0) misc[4] = uint32_t(atomicAdd(a.ticket, 1ull) - a.ticket_base);
        __syncthreads();
        t = int(misc[4]);
        if (t >= a.ntiles) return;  // ticket desync (a failed earlier launch): never touch memory
    } else {
        t = int(blockIdx.x);
    }
    // Independent images interleave their tiles in ticket order (frame = t % nframes), so every
    // frame's chain advances together; a concatenated stream keeps chain order = ticket order.
    int frame, tif, step;
    if (a.segmented) {
        frame = t % a.nframes;
        tif = t / a.nframes;
        step = a.nframes;
    } else {
        frame = t / a.tiles_per_frame;
        tif = t - frame * a.tiles_per_frame;
        step = 1;
    }
    const int chain_pos = a.segmented ? tif : t;  // tiles before this one in its chain

    // ---------------------------------------------------------------- 1. transform + quantise
    const int gi = tif * kTPB + tid;
    const bool active = gi < a.groups_per_frame;
    int nblk = 0, byi = 0, bx0 = 0;
    uint32_t seg[N][WPR];
    if (active) {
        byi = gi / a.gpr;
        bx0 = (gi - byi * a.gpr) * BPT;
        nblk = min(BPT, a.bx - bx0);
        const uint8_t* base = a.y + size_t(frame) * a.frame_pitch + size_t(byi) * N * a.stride + size_t(bx0) * N;
        load_group<N, WPR>(a, base, nblk, seg);
    } else {
#pragma unroll
        for (int r = 0; r < N; r++)
#pragma unroll
            for (int m = 0; m < WPR; m++) seg[r][m] = 0;
    }

    constexpr int NP = NN / 2;
    using Mask = NearMask<N>;
    uint32_t zp[BPT][NP];  // quantised coefficients, zig-zag order, two int16 per word
    Mask need[BPT];
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        __builtin_amdgcn_sched_barrier(0);  // one block at a time: keeps the live set small
        if constexpr (!EXACT) {
            if (a.ablate & 16) {
                need[b] = 0;
#pragma unroll
                for (int j = 0; j < NP; j++) zp[b][j] = seg[j % N][(j / N) % WPR] & 0x00FF00FFu;
            } else {
                need[b] = quantize_block<N, WPR>(tab, seg, b, zp[b]);
            }
        } else {
            need[b] = (NN == 64) ? ~Mask(0) : Mask((1ull << (NN & 63)) - 1);
#pragma unroll
            for (int j = 0; j < NP; j++) zp[b][j] = 0;
        }
        if (b >= nblk || (a.ablate & 1)) need[b] = 0;
    }

    // ---------------------------------------------------------------- 1b. FP64 re-evaluation
    // Coefficients flagged as possible ties (FAST) or all coefficients (EXACT) take the
    // reference's FP64 order.  FAST mode compacts a wave's flagged (lane, block, k) triples into
    // an LDS task list so that one exact evaluation per lane serves up to 64 of them.
    unsigned nfall = 0;
    const int lane = tid & 63, wid = tid >> 6;
    if constexpr (EXACT) {
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            BlockPx<N> px;
#pragma unroll
            for (int i = 0; i < N; i++)
#pragma unroll
                for (int m = 0; m < N / 4; m++) px.w[i * (N / 4) + m] = seg[i][(b * N) / 4 + m];
            Mask nd = need[b];
            while (nd) {
                const int k = (N == 4) ? (__ffs(uint32_t(nd)) - 1) : (__ffsll((unsigned long long)nd) - 1);
                nd &= nd - 1;
                patch<NP>(zp[b], ZigZagInv<N>::pos[k], uint32_t(exact_coef<N>(tab, k, px)));
            }
        }
    } else {
        uint32_t cnt = 0;
#pragma unroll
        for (int b = 0; b < BPT; b++) cnt += (N == 4) ? __popc(uint32_t(need[b])) : __popcll((unsigned long long)need[b]);
        if (__ballot(cnt != 0)) {
            // per-wave LDS region (the tile image is not built yet): pixels, tasks, results
            constexpr int WAVE_WORDS = (IMGW - 4) / (kTPB / 64);
            constexpr int PIXW = N * WPR;              // pixel words per lane (16 for both N)
            constexpr int CAP = (WAVE_WORDS - 64 * PIXW) / 2;
            static_assert(CAP >= 128, "LDS task list too small");
            uint32_t* wpix = img + wid * WAVE_WORDS;
            uint32_t* wtask = wpix + 64 * PIXW;
            int32_t* wres = reinterpret_cast<int32_t*>(wtask + CAP);
            const uint32_t incl = wave_incl_scan(cnt);
            const uint32_t off = incl - cnt;
            const uint32_t T = __shfl(incl, 63, 64);
            nfall = cnt;
#pragma unroll
            for (int i = 0; i < N; i++)
#pragma unroll
                for (int m = 0; m < WPR; m++) wpix[lane * PIXW + i * WPR + m] = seg[i][m];
            {
                uint32_t o = off;
#pragma unroll
                for (int b = 0; b < BPT; b++) {
                    Mask nd = need[b];
                    while (nd) {
                        const int k = (N == 4) ? (__ffs(uint32_t(nd)) - 1) : (__ffsll((unsigned long long)nd) - 1);
                        nd &= nd - 1;
                        if (o < CAP) wtask[o] = uint32_t(lane) | (uint32_t(b) << 6) | (uint32_t(k) << 8);
                        o++;
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t TT = min(T, uint32_t(CAP));
            for (uint32_t base = 0; base < TT; base += 64) {
                const uint32_t i = base + lane;
                if (i < TT) {
                    const uint32_t task = wtask[i];
                    const int o = int(task & 63), b = int((task >> 6) & 3), k = int(task >> 8);
                    BlockPx<N> px;
#pragma unroll
                    for (int r = 0; r < N; r++)
#pragma unroll
                        for (int m = 0; m < N / 4; m++) px.w[r * (N / 4) + m] = wpix[o * PIXW + r * WPR + (b * N) / 4 + m];
                    wres[i] = exact_coef<N>(tab, k, px);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (cnt) {
                uint32_t o = off;
#pragma unroll
                for (int b = 0; b < BPT; b++) {
                    Mask nd = need[b];
                    if (nd) {
                        BlockPx<N> px;
#pragma unroll
                        for (int i = 0; i < N; i++)
#pragma unroll
                            for (int m = 0; m < N / 4; m++) px.w[i * (N / 4) + m] = seg[i][(b * N) / 4 + m];
                        do {
                            const int k = (N == 4) ? (__ffs(uint32_t(nd)) - 1) : (__ffsll((unsigned long long)nd) - 1);
                            nd &= nd - 1;
                            // tasks beyond the list capacity are evaluated by their own lane
                            const int v = (o < CAP) ? wres[o] : exact_coef<N>(tab, k, px);
                            patch<NP>(zp[b], ZigZagInv<N>::pos[k], uint32_t(v));
                            o++;
                        } while (nd);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        const unsigned wsum = unsigned(wave_sum64(nfall));  // statistics: spread counters
        if (lane == 0 && wsum) atomicAdd(&a.err[2 + ((t * 4 + wid) & 63)], wsum);
    }

    // ---------------------------------------------------------------- 1c. zig-zag RLE sizing
    uint32_t blw[BPT];  // bl | Lw << 8
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
        uint32_t rb;
        blw[b] = size_block<N>(zp[b], a.rle, &rb);
        if (b < nblk) mybits += rb;
    }
    __syncthreads();  // the per-wave task areas alias the tile image

    // ---------------------------------------------------------------- 2. tile scan + LDS image
    uint32_t A;
    const uint32_t off = block_excl_scan(mybits, misc, &A);
    const uint32_t nw = (A + 31) >> 5;
    for (uint32_t w = tid; w < nw + 1; w += kTPB) img[w] = 0u;
    __syncthreads();
    if (mybits && !(a.ablate & 2)) {
        BitSink sink(img, off);
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            if (b < nblk) {
                const int bl = int(blw[b] & 0xFF), lw = int(blw[b] >> 8);
                const uint32_t m = (1u << bl) - 1u;
                if (a.rle) sink.put(4 + bl, ((uint32_t(bl) & 0xFu) << bl) | uint32_t(lw));
                else sink.put(4, uint32_t(bl) & 0xFu);
                // value fields in pairs: (z[2j], z[2j+1]) as one 2*bl-bit put
#pragma unroll
                for (int j = 0; j < NN / 2; j++) {
                    if (2 * j < lw) {
                        const uint32_t lo = zp[b][j] & m, hi = (zp[b][j] >> 16) & m;
                        if (2 * j + 1 < lw) sink.put(2 * bl, (lo << bl) | hi);
                        else sink.put(bl, lo);
                    }
                }
            }
        }
        sink.finish();
    }
    __syncthreads();

    // ---------------------------------------------------------------- 3. look-back
    const bool chain_last = a.segmented ? (tif == a.tiles_per_frame - 1) : (t == a.ntiles - 1);
    uint32_t* out = a.out + (a.segmented ? uint64_t(frame) * a.out_pitch_words : 0ull);
    if (tid == 0) {
        const uint32_t my_tail = image_tail32(img, A);
        if (chain_pos == 0) {
            // chain start: the bits before start_bit belong to the caller (header); keep them
            const uint64_t P = a.start_bit;
            const uint32_t s = uint32_t(P & 31);
            const uint32_t ptail = s ? (bswap32(out[P >> 5]) >> (32 - s)) : 0u;
            const uint32_t tl = (A >= 32) ? my_tail : ((A ? (ptail << A) : ptail) | my_tail);
            st_state(&a.st[2 * t], (uint64_t(a.tag) << 56) | (uint64_t(A) << 32) | tl);
            st_state(&a.st[2 * t + 1], (uint64_t(a.tag) << 56) | (uint64_t(A) & kMask56));
            misc[5] = 0;
            misc[6] = 0;
            misc[7] = ptail;
        } else if (A >= 32) {
            st_state(&a.st[2 * t], (uint64_t(a.tag) << 56) | (uint64_t(A) << 32) | my_tail);
        }
    }
    if (chain_pos != 0 && (a.ablate & 4)) {
        if (tid == 0) {
            st_state(&a.st[2 * t + 1], (uint64_t(a.tag) << 56) | (uint64_t(A) & kMask56));
            misc[5] = uint32_t(uint64_t(tif) * 110000u);
            misc[6] = 0;
            misc[7] = 0;
        }
    } else if (chain_pos != 0) {
        uint32_t ptail;
        const uint64_t excl = lookback_wg(a.st, t, chain_pos, step, a.tag, &ptail, a.err, misc + 8);
        if (tid == 0) {
            if (A < 32) {
                // a short tile publishes its tail only now: it must carry predecessor bits
                const uint32_t tl = (A ? (ptail << A) : ptail) | image_tail32(img, A);
                st_state(&a.st[2 * t], (uint64_t(a.tag) << 56) | (uint64_t(A) << 32) | tl);
            }
            st_state(&a.st[2 * t + 1], (uint64_t(a.tag) << 56) | ((excl + A) & kMask56));
            misc[5] = uint32_t(excl);
            misc[6] = uint32_t(excl >> 32);
            misc[7] = ptail;
        }
    }
    __syncthreads();
    const uint64_t excl = uint64_t(misc[5]) | (uint64_t(misc[6]) << 32);
    if (tid == 0) {
        const uint64_t P = a.start_bit + excl;
        if (tif == 0) a.frame_start[frame] = P;
        if (chain_last) a.chain_end[a.segmented ? frame : 0] = P + A;
    }

    // ---------------------------------------------------------------- 4. store
    if (!(a.ablate & 8)) store_image(out, img, A, a.start_bit + excl, misc[7], chain_last);
}

void launch_encode(const EncArgs& a, int n, bool exact, hipStream_t s) {
    const dim3 grid(a.ntiles), block(kTPB);
    if (n == 4) {
        if (exact) hipLaunchKernelGGL((encode_kernel<4, true>), grid, block, 0, s, a, a.tab);
        else hipLaunchKernelGGL((encode_kernel<4, false>), grid, block, 0, s, a, a.tab);
    } else {
        if (exact) hipLaunchKernelGGL((encode_kernel<8, true>), grid, block, 0, s, a, a.tab);
        else hipLaunchKernelGGL((encode_kernel<8, false>), grid, block, 0, s, a, a.tab);
    }
}

}  // namespace ie
