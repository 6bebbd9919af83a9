// imageencoder_amd/csrc/ie_pframe.hip -- P-frames of a gop > 1 video on gfx950 (§8f rank 4).
//
// A P-frame (Frame.cpp:160-243) is, per 16x16 macroblock: a SAD pattern search against the
// previous frame's buffer (Block.cpp:267-339 over the pattern tree of algo.cpp:119-139), the
// prediction error coded per 4x4 microblock through the FP64 forward DCT / quantiser and decoded
// back (ImageBase.cpp:266-306, Block.cpp:139-177), the reference block copied into the frame and
// the decoded error added back (Frame.cpp:220-242, Block.cpp:110-128).  The payload is the
// macroblocks' motion vectors followed by the covered microblocks' records in raster order.
//
// Layout of the work: one 256-thread workgroup per macroblock, one thread per pixel for the search
// (the nine candidates of a pattern level are summed together: nine wave reductions, one LDS
// exchange, every thread then picks the winner in the reference's order -- `<=`, later candidates
// win ties), one thread per coefficient for the DCT and one per pixel for the inverse, the 4x4
// microblocks' error staged in LDS as FP64.  The FP64 arithmetic is the reference's operation
// order (compiled with -ffp-contract=off).  The frame's first bit lives on the device (the
// previous frame's end), so consecutive frames chain without a host round trip; the records are
// placed by a two-level scan of their lengths and ORed into the zeroed stream.
#include <hip/hip_runtime.h>

#include "ie_device.h"

namespace ie {
namespace {

constexpr int kMB = 16;
constexpr int kPfTileBlocks = 2048;  // record-length tile of the scan: 256 threads x 8 blocks
__constant__ int kSx[9] = {0, 1, 1, 0, -1, -1, -1, 0, 1};  // algo.cpp:90-100
__constant__ int kSy[9] = {0, 0, 1, 1, 1, 0, -1, -1, -1};
__constant__ int kZz4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};  // algo.cpp:68-87

__device__ __forceinline__ int clamp16(int v, int hi) {  // std::clamp over int16_t (ImageBase.cpp:253-254)
    const int s = int(int16_t(v));
    return s < 0 ? 0 : (s > hi ? hi : s);
}

__device__ __forceinline__ int bits_needed16(int v) {  // utils.hpp:226-243 for an int16 value
    const int a = v < 0 ? ~v : v;
    return 33 - __clz(a) > 16 ? 16 : 33 - __clz(a);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// MSB-first bits ORed into the zeroed stream (words = stream bytes [4w, 4w + 4)).
struct BitOr {
    uint32_t* out;
    uint64_t w;
    uint32_t fill;
    uint64_t acc;
    __device__ BitOr(uint32_t* o, uint64_t pos) : out(o), w(pos >> 5), fill(uint32_t(pos & 31u)), acc(0) {}
    __device__ void put(int len, uint32_t v) {
        if (len <= 0) return;
        v &= (len >= 32) ? ~0u : ((1u << len) - 1u);
        acc |= uint64_t(v) << (64 - fill - uint32_t(len));
        fill += uint32_t(len);
        if (fill >= 32) {
            atomicOr(out + w, bswap32(uint32_t(acc >> 32)));
            acc <<= 32;
            fill -= 32;
            w++;
        }
    }
    __device__ void flush() {
        if (fill) atomicOr(out + w, bswap32(uint32_t(acc >> 32)));
    }
};

// bl | lw << 8 of a 4x4 block's record (Block.cpp:186-232 + the length rule of :383-397)
__device__ __forceinline__ uint32_t size4(const int16_t* c, int rle) {
    int L = 0, mb = 0, prev = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int v = c[kZz4[k]];
        if (v != 0) {
            if (k < 15) prev = k + 1;
            L = k + 1;
            mb = max(mb, bits_needed16(v));
        }
    }
    const int ffsL = L ? 32 - __clz(L) : 1;  // utils.hpp:210-216 (ffs(0) = 1 in every build)
    const int bl = max(mb, ffsL);
    const int lw = !rle ? 16 : ((L == 16 && c[kZz4[14]] == 0) ? prev : L);
    return uint32_t(bl) | (uint32_t(lw) << 8);
}

__device__ __forceinline__ uint32_t rec_len(uint32_t s, int rle) {
    const uint32_t bl = s & 0xFFu, lw = s >> 8;
    return 4u + (rle ? bl : 0u) + bl * lw;
}

template <int N>
__global__ __launch_bounds__(kTPB) void pf_macroblock_kernel(PfArgs a) {
    __shared__ uint32_t red[4][9];
    __shared__ double xs[256];
    __shared__ int16_t cq[256];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int mb = blockIdx.x;
    const int mx = (mb % a.mbx) * kMB, my = (mb / a.mbx) * kMB;
    const int py = t >> 4, px = t & 15;
    const int W16 = a.w - kMB, H16 = a.h - kMB;
    const int c = a.cur[size_t(my + py) * a.cs + mx + px];

    // ---- search (Block.cpp:272-329): the first best block is the one at ABSOLUTE (0, 0)
    int cx = 0, cy = 0, r = a.merange / 2;
    int bbx = 0, bby = 0;
    uint32_t best = 0xFFFFFFFFu;
    while (r != 0) {
        uint32_t d[9];
        int qx[9], qy[9];
#pragma unroll
        for (int p = 0; p < 9; p++) {
            qx[p] = clamp16(cx + kSx[p] * r + mx, W16);
            qy[p] = clamp16(cy + kSy[p] * r + my, H16);
            d[p] = uint32_t(abs(c - int(a.ref[size_t(qy[p] + py) * a.rs + qx[p] + px])));
        }
#pragma unroll
        for (int p = 0; p < 9; p++) {
            uint32_t v = d[p];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
            if (lane == 0) red[wv][p] = v;
        }
        __syncthreads();
        int np = -1, nbx = 0, nby = 0;
        uint32_t nd = best;
#pragma unroll
        for (int p = 0; p < 9; p++) {
            if (p > 0 && qx[p] == mx && qy[p] == my) continue;  // Block.cpp:297-301
            const uint32_t s = red[0][p] + red[1][p] + red[2][p] + red[3][p];
            if (s <= nd) {
                np = p;
                nd = s;
                nbx = qx[p];
                nby = qy[p];
            }
        }
        __syncthreads();  // red is rewritten by the next level
        if (np < 0) break;
        cx += kSx[np] * r;
        cy += kSy[np] * r;
        r /= 2;
        best = nd;
        bbx = nbx;
        bby = nby;
    }
    // the reference block at the motion vector (getCoordAfterMotion, Frame.cpp:221-224)
    const int ccx = clamp16(mx + cx, W16), ccy = clamp16(my + cy, H16);
    if (t == 0) {
        BitOr o(a.out, *a.start + uint64_t(mb) * 2u * uint32_t(a.mv_bits));  // streamMVec (Block.cpp:415-423)
        o.put(a.mv_bits, uint32_t(int32_t(int16_t(cx))));
        o.put(a.mv_bits, uint32_t(int32_t(int16_t(cy))));
        o.flush();
    }
    if constexpr (N != 4) {
        // micro_per_macro_row is 0 for 8x8 blocks (ImageBase.cpp:271): no error is coded and
        // expandDifferences adds the frame's own pixels to the copied reference block
        const int base = a.ref[size_t(ccy + py) * a.rs + ccx + px];
        a.rec[size_t(my + py) * a.w + mx + px] = uint8_t(min(base + c, 255));
        return;
    } else {
        const EncTables* T = a.tab;
        // ---- prediction error, microblock mi = (py/4, px/4), element k (expandDifferenceWith)
        const int rb = a.ref[size_t(bby + py) * a.rs + bbx + px];
        const int mi = (py >> 2) * 4 + (px >> 2);
        xs[mi * 16 + (py & 3) * 4 + (px & 3)] = (double(c) - double(rb)) + double(-128);
        __syncthreads();
        // ---- forward DCT + quantiser, thread = (microblock t/16, coefficient t%16) (Block.cpp:139-153)
        {
            const int m = t >> 4, uv = t & 15;
            const double* P = T->P + uv * 16;
            const double* x = xs + m * 16;
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < 16; k++) acc = acc + P[k] * x[k];
            const double D = acc * T->S[uv];
            cq[t] = int16_t(round(D / T->qd[uv]));
        }
        __syncthreads();
        const int m = t >> 4, e = t & 15;
        const int gb = (my / 4 + (m >> 2)) * a.bx + (mx / 4 + (m & 3));
        a.coef[size_t(gb) * 16 + e] = cq[t];
        if (e == 0) a.bits[gb] = rec_len(size4(cq + m * 16, a.rle), a.rle);
        // ---- inverse (Block.cpp:162-177), thread = (microblock t/16, pixel t%16), then
        // expandDifferences over the copied reference block (Block.cpp:110-119)
        double tt = 0.0;
#pragma unroll
        for (int uv = 0; uv < 16; uv++) tt = tt + T->R[uv * 16 + e] * (double(cq[m * 16 + uv]) * T->qd[uv]);
        const double ex = tt + double(128);
        const int ppy = (m >> 2) * 4 + (e >> 2), ppx = (m & 3) * 4 + (e & 3);
        const double v = double(a.ref[size_t(ccy + ppy) * a.rs + ccx + ppx]) + ex;
        a.rec[size_t(my + ppy) * a.w + mx + ppx] = uint8_t(v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v));
    }
}

// Pixels no macroblock covers (the right / bottom strips when W or H is not a multiple of 16):
// their microblocks keep the frame's own pixels as "error" and have no record, so
// expandDifferences doubles them (Block.cpp:52-55,110-119).
__global__ __launch_bounds__(kTPB) void pf_strip_kernel(PfArgs a) {
    const size_t i = size_t(blockIdx.x) * kTPB + threadIdx.x;
    if (i >= size_t(a.w) * a.h) return;
    const int x = int(i % size_t(a.w)), y = int(i / size_t(a.w));
    if (x < a.mbx * kMB && y < a.mby * kMB) return;
    const int c = a.cur[size_t(y) * a.cs + x];
    a.rec[i] = uint8_t(min(2 * c, 255));
}

// block-wide exclusive scan of one value per thread; returns the total in *tot
__device__ __forceinline__ uint64_t block_exscan(uint64_t v, uint64_t* sh, uint64_t* tot) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wv] = x;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int k = 0; k < kTPB / 64; k++) {
        if (k < wv) before += sh[k];
        all += sh[k];
    }
    __syncthreads();
    *tot = all;
    return before + x - v;
}

__global__ __launch_bounds__(kTPB) void pf_tile_sum_kernel(const uint32_t* bits, int nb, uint64_t* tsum) {
    __shared__ uint64_t sh[kTPB / 64];
    const int b0 = blockIdx.x * kPfTileBlocks + threadIdx.x * 8;
    uint64_t s = 0;
    for (int k = 0; k < 8; k++)
        if (b0 + k < nb) s += bits[b0 + k];
    uint64_t tot;
    block_exscan(s, sh, &tot);
    if (threadIdx.x == 0) tsum[blockIdx.x] = tot;
}

// one workgroup: exclusive prefix of the tile sums; the frame's end bit
__global__ __launch_bounds__(kTPB) void pf_tile_scan_kernel(uint64_t* tsum, int ntiles, uint64_t head_bits,
                                                            const uint64_t* start, uint64_t* end) {
    __shared__ uint64_t sh[kTPB / 64];
    uint64_t carry = 0;
    for (int t0 = 0; t0 < ntiles; t0 += kTPB) {
        const int i = t0 + threadIdx.x;
        const uint64_t v = (i < ntiles) ? tsum[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_exscan(v, sh, &tot);
        if (i < ntiles) tsum[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *end = *start + head_bits + carry;
}

__global__ __launch_bounds__(kTPB) void pf_emit_kernel(PfArgs a, int nb, const uint64_t* tpre, uint64_t head_bits) {
    __shared__ uint64_t sh[kTPB / 64];
    const int b0 = blockIdx.x * kPfTileBlocks + threadIdx.x * 8;
    uint64_t s = 0;
    for (int k = 0; k < 8; k++)
        if (b0 + k < nb) s += a.bits[b0 + k];
    uint64_t tot;
    const uint64_t ex = block_exscan(s, sh, &tot);
    if (s == 0) return;
    BitOr o(a.out, *a.start + head_bits + tpre[blockIdx.x] + ex);
    for (int k = 0; k < 8 && b0 + k < nb; k++) {
        if (!a.bits[b0 + k]) continue;  // no macroblock covered it: no record (Block.cpp:373-375)
        const int16_t* c = a.coef + size_t(b0 + k) * 16;
        const uint32_t sz = size4(c, a.rle);
        const int bl = int(sz & 0xFFu), lw = int(sz >> 8);
        o.put(4, uint32_t(bl));  // Block::streamEncoded (Block.cpp:372-413)
        if (a.rle) o.put(bl, uint32_t(lw));
        for (int i = 0; i < lw; i++) o.put(bl, uint32_t(int32_t(c[kZz4[i]])));
    }
    o.flush();
}

// the frame's end bit when it carries no records (8x8 blocks, or no macroblock)
__global__ void pf_end_kernel(const uint64_t* start, uint64_t* end, uint64_t head_bits) {
    if (threadIdx.x == 0) *end = *start + head_bits;
}

}  // namespace

void launch_pframe(const PfArgs& a, int n, uint64_t* tsum, hipStream_t s) {
    const int nmb = a.mbx * a.mby;
    const uint64_t head = uint64_t(nmb) * 2u * uint32_t(a.mv_bits);
    const int nb = a.bx * (a.h / n);
    if (nmb > 0) {
        if (n == 4) {
            // blocks no macroblock covers keep bits = 0 (no record)
            if (a.w % kMB || a.h % kMB) (void)hipMemsetAsync(a.bits, 0, size_t(nb) * sizeof(uint32_t), s);
            hipLaunchKernelGGL(pf_macroblock_kernel<4>, dim3(nmb), dim3(kTPB), 0, s, a);
        } else {
            hipLaunchKernelGGL(pf_macroblock_kernel<8>, dim3(nmb), dim3(kTPB), 0, s, a);
        }
    }
    if (a.w % kMB || a.h % kMB || nmb == 0) {
        const size_t px = size_t(a.w) * a.h;
        hipLaunchKernelGGL(pf_strip_kernel, dim3(unsigned((px + kTPB - 1) / kTPB)), dim3(kTPB), 0, s, a);
    }
    if (n == 4 && nmb > 0) {
        const int ntiles = (nb + kPfTileBlocks - 1) / kPfTileBlocks;
        hipLaunchKernelGGL(pf_tile_sum_kernel, dim3(ntiles), dim3(kTPB), 0, s, a.bits, nb, tsum);
        hipLaunchKernelGGL(pf_tile_scan_kernel, dim3(1), dim3(kTPB), 0, s, tsum, ntiles, head, a.start, a.end);
        hipLaunchKernelGGL(pf_emit_kernel, dim3(ntiles), dim3(kTPB), 0, s, a, nb, tsum, head);
    } else {
        hipLaunchKernelGGL(pf_end_kernel, dim3(1), dim3(64), 0, s, a.start, a.end, head);
    }
}

int pframe_tiles(int nb) { return (nb + kPfTileBlocks - 1) / kPfTileBlocks; }

}  // namespace ie
