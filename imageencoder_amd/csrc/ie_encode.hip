// imageencoder_amd/csrc/ie_encode.hip -- the block encoder for gfx950 (MI355X).
//
// One launch encodes a batch of frames.  Work decomposition:
//   lane      = one "group" of BPT horizontally adjacent N x N blocks (4 x 4x4 or 1 x 8x8), so a
//               wave reads 64 x 16 B (or 64 x 8 B) contiguous bytes per pixel row;
//   workgroup = one tile of kTPB groups (<= 1024 blocks), never straddling a frame.
// Per tile, in one pass over the pixels (each byte is read from HBM once, each output word
// written once):
//   1. level shift + forward DCT + quantise every block (Block.cpp:139-153, algo.cpp:309-331):
//      FAST = separable FP32 with a rigorous error bound; coefficients whose quotient lies within
//      that bound of a rounding tie are re-evaluated in the reference's exact FP64 operation
//      order.  EXACT = every coefficient in FP64 reference order.
//   2. zig-zag RLE sizing (Block.cpp:186-232, :383-397): bl, Lw, record length;
//   3. workgroup exclusive scan of record lengths; the records are written MSB-first into an
//      LDS image of the tile's bit stream (Block.cpp:372-413, BitStream.cpp:61-77);
//   4. decoupled look-back over the preceding tiles of the chain for the tile's global bit offset;
//   5. funnel-shifted, coalesced store of the LDS image into the output words.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ie_common.cuh"
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

template <int N> struct Geo;
template <> struct Geo<4> { static constexpr int BPT = 4; };  // 16 B per pixel row per lane
template <> struct Geo<8> { static constexpr int BPT = 1; };  //  8 B per pixel row per lane

// bits-in-tile upper bound: 4 + 16 * (N*N + 1) bits per block
template <int N> constexpr int image_words() {
    return (kTPB * Geo<N>::BPT * (4 + 16 * (N * N + 1)) + 31) / 32 + 2;
}

// Exact coefficient in the reference's FP64 order (algo.cpp:314-325, Block.cpp:149-152):
//   acc = 0; for i, j: acc = acc + P[uv][ij] * x[ij];  D = acc * (C(u)C(v));  round(D / q)
// with x[ij] = double(p) - 128 (Block.cpp:141-143).  This file is compiled with
// -ffp-contract=off, so every product and sum is rounded separately as in the reference; the
// division is IEEE; the rounding is half away from zero (std::round).
template <int N, int WPR>
__device__ __forceinline__ int exact_coef(const EncTables* __restrict__ tab, int k, const uint32_t (&seg)[N][WPR],
                                          int b) {
    constexpr int NN = N * N;
    const double* P = &tab->P[k * NN];
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
        for (int j = 0; j < N; j++) {
            const int byte = b * N + j;
            const double x = double(int((seg[i][byte >> 2] >> (8 * (byte & 3))) & 0xFFu)) + (-128.0);
            acc = acc + P[i * N + j] * x;
        }
    const double D = acc * tab->S[k];
    const double t = D / tab->qd[k];
    double r = trunc(t);
    if (fabs(t - r) >= 0.5) r += copysign(1.0, t);
    return int(r);
}

// Load the pixel rows of one group: seg[r][m] = bytes [4m, 4m+4) of the group's row r.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

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

template <int N, bool EXACT>
__global__ __launch_bounds__(kTPB) void encode_kernel(EncArgs a) {
    constexpr int NN = N * N;
    constexpr int BPT = Geo<N>::BPT;
    constexpr int WPR = BPT * N / 4;
    constexpr int IMGW = image_words<N>();
    __shared__ uint32_t smem[IMGW + 16];
    uint32_t* img = smem;
    uint32_t* misc = smem + IMGW;  // [0..3] scan, [4] ticket, [5..6] excl lo/hi, [7] pred tail

    const int tid = threadIdx.x;
    if (tid == 0) misc[4] = uint32_t(atomicAdd(a.ticket, 1ull) - a.ticket_base);
    __syncthreads();
    const int t = int(misc[4]);
    if (t >= a.ntiles) return;  // ticket desync (a failed earlier launch): never touch memory
    const int frame = t / a.tiles_per_frame;
    const int tif = t - frame * a.tiles_per_frame;
    const EncTables* __restrict__ tab = a.tab;

    // ---------------------------------------------------------------- 1. transform + quantise
    const int gi = tif * kTPB + tid;
    const bool active = gi < a.groups_per_frame;
    int nblk = 0;
    uint32_t seg[N][WPR];
    if (active) {
        const int byi = gi / a.gpr, seg_i = gi - byi * a.gpr;
        const int bx0 = seg_i * BPT;
        nblk = min(BPT, a.bx - bx0);
        const uint8_t* base = a.y + size_t(frame) * a.frame_pitch + size_t(byi) * N * a.stride + size_t(bx0) * N;
        load_group<N, WPR>(a, base, nblk, seg);
    } else {
#pragma unroll
        for (int r = 0; r < N; r++)
#pragma unroll
            for (int m = 0; m < WPR; m++) seg[r][m] = 0;
    }

    int zq[BPT][NN];        // quantised coefficients, zig-zag order
    uint32_t blw[BPT];      // bl | Lw << 8
    uint32_t mybits = 0;
    unsigned nfall = 0;
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        float x[NN];
#pragma unroll
        for (int i = 0; i < N; i++)
#pragma unroll
            for (int j = 0; j < N; j++) {
                const int byte = b * N + j;
                x[i * N + j] = float((seg[i][byte >> 2] >> (8 * (byte & 3))) & 0xFFu) - 128.0f;
            }
        int zn[NN];  // natural order
        uint64_t need = 0;
        if constexpr (!EXACT) {
            // separable FP32: y[i][v] = sum_j cf[v][j] x[i][j];  D[u][v] = sum_i cf[u][i] y[i][v]
            float yv[NN];
#pragma unroll
            for (int i = 0; i < N; i++)
#pragma unroll
                for (int v = 0; v < N; v++) {
                    float acc = 0.0f;
#pragma unroll
                    for (int j = 0; j < N; j++) acc = __builtin_fmaf(tab->cf[v * N + j], x[i * N + j], acc);
                    yv[i * N + v] = acc;
                }
#pragma unroll
            for (int u = 0; u < N; u++)
#pragma unroll
                for (int v = 0; v < N; v++) {
                    float acc = 0.0f;
#pragma unroll
                    for (int i = 0; i < N; i++) acc = __builtin_fmaf(tab->cf[u * N + i], yv[i * N + v], acc);
                    const int k = u * N + v;
                    const float tq = acc * tab->g[k];
                    const float av = fabsf(tq);
                    const float fl = floorf(av);
                    const float fr = av - fl;
                    if (fabsf(fr - 0.5f) <= tab->thr[k]) need |= 1ull << k;
                    const int qi = int(fl) + (fr >= 0.5f ? 1 : 0);
                    zn[k] = tq < 0.0f ? -qi : qi;
                }
        } else {
            if constexpr (NN == 64) need = ~0ull;
            else need = (1ull << NN) - 1;
#pragma unroll
            for (int k = 0; k < NN; k++) zn[k] = 0;
        }
        // FP64 re-evaluation of flagged coefficients; the wave skips k that no lane flagged
#pragma unroll
        for (int k = 0; k < NN; k++) {
            const bool mine = (need >> k) & 1ull;
            if (__ballot(mine)) {
                if (mine && b < nblk) {
                    zn[k] = exact_coef<N, WPR>(tab, k, seg, b);
                    nfall++;
                }
            }
        }
        if (a.coef && b < nblk) {
            const int byi = gi / a.gpr, bxb = (gi - byi * a.gpr) * BPT + b;
            int16_t* dst = a.coef + (size_t(frame) * a.by * a.bx + size_t(byi) * a.bx + bxb) * NN;
#pragma unroll
            for (int k = 0; k < NN; k++) dst[k] = int16_t(zn[k]);
        }
        // zig-zag + RLE sizing
        uint64_t nz = 0;
        int maxb = 1;
#pragma unroll
        for (int kz = 0; kz < NN; kz++) {
            const int v = zn[ZigZag<N>::idx[kz]];
            zq[b][kz] = v;
            nz |= uint64_t(v != 0) << kz;
            const uint32_t s = uint32_t(v ^ (v >> 31));
            maxb = max(maxb, 33 - __clz(s));
        }
        const int L = nz ? 64 - __clzll((long long)nz) : 0;
        const int ffsL = L ? 32 - __clz(L) : 1;  // ffs(0) == 1 (utils.hpp:210-216)
        const int bl = max(maxb, ffsL);
        int lw;
        if (!a.rle) {
            lw = NN;
        } else if (L == NN && !((nz >> (NN - 2)) & 1ull)) {
            const uint64_t m = nz & ((1ull << (NN - 1)) - 1);  // drop the last element (Block.cpp:388-390)
            lw = m ? 64 - __clzll((long long)m) : 0;
        } else {
            lw = L;
        }
        blw[b] = uint32_t(bl) | (uint32_t(lw) << 8);
        if (b < nblk) mybits += 4u + uint32_t(bl) * uint32_t(lw + a.rle);
    }
    if (!EXACT && nfall) atomicAdd(&a.err[1], nfall);

    // ---------------------------------------------------------------- 2. tile scan + LDS image
    uint32_t A;
    const uint32_t off = block_excl_scan(mybits, misc, &A);
    const uint32_t nw = (A + 31) >> 5;
    for (uint32_t w = tid; w < nw + 1; w += kTPB) img[w] = 0u;
    __syncthreads();
    if (mybits) {
        BitSink sink(img, off);
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            if (b < nblk) {
                const int bl = int(blw[b] & 0xFF), lw = int(blw[b] >> 8);
                sink.put(4, uint32_t(bl) & 0xFu);
                if (a.rle) sink.put(bl, uint32_t(lw));
#pragma unroll
                for (int kz = 0; kz < NN; kz++)
                    if (kz < lw) sink.put(bl, uint32_t(zq[b][kz]));
            }
        }
        sink.finish();
    }
    __syncthreads();

    // ---------------------------------------------------------------- 3. look-back
    const int c0 = a.segmented ? frame * a.tiles_per_frame : 0;
    const bool chain_last = a.segmented ? (tif == a.tiles_per_frame - 1) : (t == a.ntiles - 1);
    uint32_t* out = a.out + (a.segmented ? uint64_t(frame) * a.out_pitch_words : 0ull);
    const uint32_t my_tail = (tid == 0) ? image_tail32(img, A) : 0u;
    if (tid == 0 && A >= 32) st_state(&a.st_agg[t], (uint64_t(a.tag) << 56) | (uint64_t(A) << 32) | my_tail);
    if (tid < 64) {
        uint64_t excl = 0;
        uint32_t ptail = 0;
        if (t == c0) {
            // chain start: the bits before start_bit belong to the caller (header); keep them
            const uint64_t P = a.start_bit;
            const uint32_t s = uint32_t(P & 31);
            ptail = s ? (bswap32(out[P >> 5]) >> (32 - s)) : 0u;
        } else {
            excl = lookback(a.st_agg, a.st_inc, t, c0, a.tag, &ptail, a.err);
        }
        if (tid == 0) {
            if (A < 32) {
                // a short tile publishes its tail only now: it must carry predecessor bits
                const uint32_t tl = (A ? (ptail << A) : ptail) | my_tail;
                st_state(&a.st_agg[t], (uint64_t(a.tag) << 56) | (uint64_t(A) << 32) | tl);
            }
            st_state(&a.st_inc[t], (uint64_t(a.tag) << 56) | ((excl + A) & kMask56));
            misc[5] = uint32_t(excl);
            misc[6] = uint32_t(excl >> 32);
            misc[7] = ptail;
            const uint64_t P = a.start_bit + excl;
            if (tif == 0) a.frame_start[frame] = P;
            if (chain_last) a.chain_end[a.segmented ? frame : 0] = P + A;
        }
    }
    __syncthreads();

    // ---------------------------------------------------------------- 4. store
    const uint64_t excl = uint64_t(misc[5]) | (uint64_t(misc[6]) << 32);
    store_image(out, img, A, a.start_bit + excl, misc[7], chain_last);
}

void launch_encode(const EncArgs& a, int n, bool exact, hipStream_t s) {
    const dim3 grid(a.ntiles), block(kTPB);
    if (n == 4) {
        if (exact) hipLaunchKernelGGL((encode_kernel<4, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((encode_kernel<4, false>), grid, block, 0, s, a);
    } else {
        if (exact) hipLaunchKernelGGL((encode_kernel<8, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((encode_kernel<8, false>), grid, block, 0, s, a);
    }
}

}  // namespace ie
