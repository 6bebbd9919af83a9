// imageencoder_amd/csrc/ie_pframe.hip -- P-frames of a gop > 1 video on gfx950 (§8f rank 4).
//
// A P-frame (Frame.cpp:160-243) is, per 16x16 macroblock: a SAD pattern search against the
// previous frame's buffer (Block.cpp:267-339 over the pattern tree of algo.cpp:119-139), the
// prediction error coded per 4x4 microblock through the FP64 forward DCT / quantiser and decoded
// back (ImageBase.cpp:266-306, Block.cpp:139-177), the reference block copied into the frame and
// the decoded error added back (Frame.cpp:220-242, Block.cpp:110-128).  The payload is the
// macroblocks' motion vectors followed by the covered microblocks' records in raster order.
//
// Layout of the work: one wave per macroblock, four pixels per lane (a candidate's partial SAD is
// one v_sad_u8; the nine candidates of a pattern level are reduced across the wave by DPP and
// every lane applies the reference's rule -- `<=`, later candidates win ties -- so the search needs
// no LDS and no barrier), four coefficients per lane for the DCT and four pixels for the inverse,
// the 4x4 microblocks' error and the FP64 transform rows staged in LDS.  The FP64 arithmetic is the reference's operation
// order (compiled with -ffp-contract=off).  The frame's first bit lives on the device (the
// previous frame's end), so consecutive frames chain without a host round trip; the records are
// placed by a two-level scan of their lengths and ORed into the zeroed stream.
#include <hip/hip_runtime.h>

#include "ie_common.hpp"
#include "ie_device.h"

namespace ie {
namespace {

constexpr int kMB = 16;
#ifndef IE_PF_PER
#define IE_PF_PER 2
#endif
constexpr int kPfPer = IE_PF_PER;              // records per emitting thread
constexpr int kPfTileBlocks = kTPB * kPfPer;  // record-length tile of the scan
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

// Sum over the wave by DPP (quad permutes, row shifts, row broadcasts: no LDS traffic), the total
// read from lane 63 as a wave-uniform value.  Lanes whose DPP source is outside the row add 0.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    int x = int(v);
    x += __builtin_amdgcn_update_dpp(0, x, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    x += __builtin_amdgcn_update_dpp(0, x, 0x4e, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8 (row sum in lane 15)
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xf, 0xf, false);  // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xf, 0xf, false);  // row_bcast:31 (total in lane 63)
    return uint32_t(__builtin_amdgcn_readlane(x, 63));
}

// four horizontally adjacent pixels packed little-endian (byte j = pixel j), any alignment
__device__ __forceinline__ uint32_t load4(const uint8_t* p) {
    return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}

// Pixels no macroblock covers (the bottom strip, rows [16*mby, h), then the right strip of the
// covered rows, columns [16*mbx, w)): their microblocks keep the frame's own pixels as "error" and
// have no record (bits = 0, written here for 4x4 blocks), so expandDifferences doubles them
// (Block.cpp:52-55,110-119).
__device__ __forceinline__ void pf_strip_pixel(const PfArgs& a, int n, size_t i) {
    const int hc = a.mby * kMB, wc = a.mbx * kMB;
    const size_t nbot = size_t(a.h - hc) * a.w, nright = size_t(hc) * (a.w - wc);
    if (i >= nbot + nright) return;
    int x, y;
    if (i < nbot) {
        y = hc + int(i / size_t(a.w));
        x = int(i % size_t(a.w));
    } else {
        const size_t j = i - nbot;
        const int rw = a.w - wc;
        y = int(j / size_t(rw));
        x = wc + int(j % size_t(rw));
    }
    const int c = a.cur[size_t(y) * a.cs + x];
    a.rec[size_t(y) * a.w + x] = uint8_t(min(2 * c, 255));
    if (n == 4 && (x & 3) == 0 && (y & 3) == 0) a.bits[size_t(y / 4) * a.bx + x / 4] = 0u;
}

// One WAVE per macroblock (a 64-thread workgroup: its barriers cost nothing): lane l holds pixel row
// l/4, columns 4(l%4)..+3 of the macroblock, whose SAD against a candidate is one v_sad_u8.
constexpr int kMbTPB = 64;

// Workgroups past the macroblocks (64 pixels each) do the uncovered strips: they touch no pixel
// or record a macroblock does, so they share the launch.
template <int N>
__global__ __launch_bounds__(kMbTPB) void pf_macroblock_kernel(PfArgs a) {
    __shared__ double xs[256];
    __shared__ double Ps[256], Rs[256], qs[16], Ss[16];
    __shared__ int16_t cq[256];
    const int l = threadIdx.x;
    const int mb = blockIdx.x;
    if (mb >= a.mbx * a.mby) {
        const size_t i = size_t(mb - a.mbx * a.mby) * kMbTPB + size_t(l);
        const size_t npx = size_t(a.w) * a.h - size_t(a.mbx) * a.mby * kMB * kMB;
        if (i < npx) pf_strip_pixel(a, N, i);
        return;
    }
    const int mx = (mb % a.mbx) * kMB, my = (mb / a.mbx) * kMB;
    const int py = l >> 2, px = (l & 3) * 4;
    const int W16 = a.w - kMB, H16 = a.h - kMB;
    const uint32_t c4 = load4(a.cur + size_t(my + py) * a.cs + mx + px);
    if constexpr (N == 4) {  // the FP64 rows of the forward and inverse transforms (EncTables)
        for (int i = l; i < 256; i += kMbTPB) {
            Ps[i] = a.tab->P[i];
            Rs[i] = a.tab->R[i];
        }
        if (l < 16) {
            qs[l] = a.tab->qd[l];
            Ss[l] = a.tab->S[l];
        }
    }

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
            d[p] = __builtin_amdgcn_sad_u8(c4, load4(a.ref + size_t(qy[p] + py) * a.rs + qx[p] + px), 0u);
        }
#pragma unroll
        for (int p = 0; p < 9; p++) d[p] = wave_sum(d[p]);  // the candidate's SAD, wave-uniform
        int np = -1, nbx = 0, nby = 0;
        uint32_t nd = best;
#pragma unroll
        for (int p = 0; p < 9; p++) {
            if (p > 0 && qx[p] == mx && qy[p] == my) continue;  // Block.cpp:297-301
            if (d[p] <= nd) {
                np = p;
                nd = d[p];
                nbx = qx[p];
                nby = qy[p];
            }
        }
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
    if (l == 0) {
        BitOr o(a.out, *a.start + uint64_t(mb) * 2u * uint32_t(a.mv_bits));  // streamMVec (Block.cpp:415-423)
        o.put(a.mv_bits, uint32_t(int32_t(int16_t(cx))));
        o.put(a.mv_bits, uint32_t(int32_t(int16_t(cy))));
        o.flush();
    }
    if constexpr (N != 4) {
        // micro_per_macro_row is 0 for 8x8 blocks (ImageBase.cpp:271): no error is coded and
        // expandDifferences adds the frame's own pixels to the copied reference block
        const uint32_t b4 = load4(a.ref + size_t(ccy + py) * a.rs + ccx + px);
        uint8_t* o = a.rec + size_t(my + py) * a.w + mx + px;
#pragma unroll
        for (int j = 0; j < 4; j++) o[j] = uint8_t(min(int((b4 >> (8 * j)) & 255u) + int((c4 >> (8 * j)) & 255u), 255));
        return;
    } else {
        // ---- prediction error (expandDifferenceWith): the lane's row of microblock
        // (py/4, l%4), element row py%4
        const uint32_t r4 = load4(a.ref + size_t(bby + py) * a.rs + bbx + px);
        const int mi = (py >> 2) * 4 + (l & 3);
#pragma unroll
        for (int j = 0; j < 4; j++)
            xs[mi * 16 + (py & 3) * 4 + j] =
                (double(int((c4 >> (8 * j)) & 255u)) - double(int((r4 >> (8 * j)) & 255u))) + double(-128);
        __syncthreads();
        // ---- forward DCT + quantiser (Block.cpp:139-153): lane = (microblock l/4, coefficients
        // 4(l%4)..+3), each in the reference's k order
        const int m = l >> 2, g = (l & 3) * 4;
        {
            const double* x = xs + m * 16;
            double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const double xk = x[k];
#pragma unroll
                for (int j = 0; j < 4; j++) acc[j] = acc[j] + Ps[(g + j) * 16 + k] * xk;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) cq[m * 16 + g + j] = int16_t(round((acc[j] * Ss[g + j]) / qs[g + j]));
        }
        __syncthreads();
        const int gb = (my / 4 + (m >> 2)) * a.bx + (mx / 4 + (m & 3));
        {  // the lane's four coefficients in one 8-byte store (coef rows are 32-byte aligned)
            uint64_t c4 = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) c4 |= uint64_t(uint16_t(cq[m * 16 + g + j])) << (16 * j);
            *reinterpret_cast<uint64_t*>(a.coef + size_t(gb) * 16 + g) = c4;
        }
        if (g == 0) a.bits[gb] = rec_len(size4(cq + m * 16, a.rle), a.rle);
        // ---- inverse (Block.cpp:162-177): lane = (microblock l/4, pixel row l%4), uv ascending;
        // then expandDifferences over the copied reference block (Block.cpp:110-119)
        double tt[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int uv = 0; uv < 16; uv++) {
            const double yv = double(cq[m * 16 + uv]) * qs[uv];
#pragma unroll
            for (int j = 0; j < 4; j++) tt[j] = tt[j] + Rs[uv * 16 + g + j] * yv;
        }
        const int ppy = (m >> 2) * 4 + (l & 3), ppx = (m & 3) * 4;
        const uint32_t b4 = load4(a.ref + size_t(ccy + ppy) * a.rs + ccx + ppx);
        uint32_t o4 = 0;  // four reconstructed pixels, one 4-byte store (W % 4 == 0, mx + ppx % 4 == 0)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const double v = double(int((b4 >> (8 * j)) & 255u)) + (tt[j] + double(128));
            o4 |= uint32_t(uint8_t(v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v))) << (8 * j);
        }
        *reinterpret_cast<uint32_t*>(a.rec + size_t(my + ppy) * a.w + mx + ppx) = o4;
    }
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
    const int b0 = blockIdx.x * kPfTileBlocks + threadIdx.x * kPfPer;
    uint64_t s = 0;
    for (int k = 0; k < kPfPer; k++)
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

// A tile's records are ORed into an LDS bit image (the image starts at the tile's first bit rounded
// down to a word), then the image goes out in whole words: plain stores for the words the tile owns
// alone, global ORs only for its first and last word (shared with the neighbouring tiles).
constexpr int kPfImgWords = (kPfTileBlocks * 259 + 31) / 32 + 2;  // 259 = the longest 4x4 record
__global__ __launch_bounds__(kTPB) void pf_emit_kernel(PfArgs a, int nb, const uint64_t* tpre, uint64_t head_bits) {
    __shared__ uint64_t sh[kTPB / 64];
    __shared__ uint32_t img[kPfImgWords];
    const int t = threadIdx.x;
    const int b0 = blockIdx.x * kPfTileBlocks + t * kPfPer;
    uint64_t s = 0;
    for (int k = 0; k < kPfPer; k++)
        if (b0 + k < nb) s += a.bits[b0 + k];
    uint64_t tot;
    const uint64_t ex = block_exscan(s, sh, &tot);
    const uint64_t S = *a.start + head_bits + tpre[blockIdx.x];  // the tile's first bit
    const uint32_t o0 = uint32_t(S & 31u);
    const uint32_t nw = uint32_t((o0 + tot + 31) / 32);
    for (uint32_t i = t; i < nw; i += kTPB) img[i] = 0u;
    __syncthreads();
    if (s) {
        BitOr o(img, o0 + ex);
        for (int k = 0; k < kPfPer && b0 + k < nb; k++) {
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
    __syncthreads();
    uint32_t* g = a.out + (S >> 5);
    for (uint32_t i = t; i < nw; i += kTPB) {
        if (i == 0 || i == nw - 1) atomicOr(g + i, img[i]);
        else g[i] = img[i];
    }
}

// The scan fused into the emission: tile t of the frame's record tiles publishes its bit count,
// finds its first bit by a decoupled look-back over its predecessors (the encoder's chain
// protocol, ie_common.hpp: aggregate as soon as the count is known, inclusive once resolved; tiles
// run in dispatch order) and emits -- one launch instead of tile sums, tile scan and emission.
// The last tile writes the frame's end bit.
__global__ __launch_bounds__(kTPB) void pf_emit_chain_kernel(PfArgs a, int nb, int ntiles, uint64_t head_bits) {
    __shared__ uint64_t sh[kTPB / 64];
    __shared__ uint32_t img[kPfImgWords];
    __shared__ uint64_t sx;
    const int t = threadIdx.x, tile = blockIdx.x;
    const int b0 = tile * kPfTileBlocks + t * kPfPer;
    uint64_t s = 0;
    for (int k = 0; k < kPfPer; k++)
        if (b0 + k < nb) s += a.bits[b0 + k];
    uint64_t tot;
    const uint64_t ex = block_exscan(s, sh, &tot);
    if (t == 0) chain_publish_count(a.st, tile, tile, a.tag, uint32_t(tot));
    if (t < 64) {
        uint64_t excl = 0;
        if (tile > 0) {
            const Probe pr = probe_issue(a.st, tile, tile, 1, 0, kProbe0);
            excl = lookback_wave(pr, a.st, tile, tile, 1, a.tag, a.err, nullptr, true);
            if (t == 0) publish(a.st, tile, 1, a.tag, excl + tot);
        }
        if (t == 0) sx = excl;
    }
    __syncthreads();
    const uint64_t S = *a.start + head_bits + sx;  // the tile's first bit
    if (tile == ntiles - 1 && t == 0) *a.end = S + tot;
    const uint32_t o0 = uint32_t(S & 31u);
    const uint32_t nw = uint32_t((o0 + tot + 31) / 32);
    for (uint32_t i = t; i < nw; i += kTPB) img[i] = 0u;
    __syncthreads();
    if (s) {
        BitOr o(img, o0 + ex);
        for (int k = 0; k < kPfPer && b0 + k < nb; k++) {
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
    __syncthreads();
    uint32_t* g = a.out + (S >> 5);
    for (uint32_t i = t; i < nw; i += kTPB) {
        if (i == 0 || i == nw - 1) atomicOr(g + i, img[i]);
        else g[i] = img[i];
    }
}

// the frame's end bit when it carries no records (8x8 blocks, or no macroblock)
__global__ void pf_end_kernel(const uint64_t* start, uint64_t* end, uint64_t head_bits) {
    if (threadIdx.x == 0) *end = *start + head_bits;
}

// P-frame decode, first half: lane l copies row l/4, pixels 4(l%4)..+3 of the reference block
__global__ __launch_bounds__(kMbTPB) void pf_mvcopy_kernel(const uint8_t* in, uint64_t start_bit, const uint64_t* dstart,
                                                           uint64_t nbits, int mv, const uint8_t* ref, uint64_t rs,
                                                           uint8_t* out, uint64_t os, int w, int h, int mbx) {
    const int l = threadIdx.x, mb = blockIdx.x;
    const int mx = (mb % mbx) * kMB, my = (mb / mbx) * kMB;
    if (dstart) start_bit = min(*dstart, nbits);
    const uint64_t p = start_bit + uint64_t(mb) * 2u * uint32_t(mv);
    if (p + 2u * uint32_t(mv) > nbits) return;  // (a truncated stream: the host reports it)
    uint64_t win = 0;  // 64 stream bits from byte p/8 (2*mv <= 32 bits + 7 bits of offset)
#pragma unroll
    for (int k = 0; k < 8; k++) win = (win << 8) | in[(p >> 3) + k];
    const uint32_t s = uint32_t(p & 7u);
    const uint32_t rx = uint32_t(win >> (64 - s - uint32_t(mv))) & ((1u << mv) - 1u);
    const uint32_t ry = uint32_t(win >> (64 - s - 2u * uint32_t(mv))) & ((1u << mv) - 1u);
    const int vx = int(int16_t(uint16_t(rx << (16 - mv))) >> (16 - mv));  // shift_signed (utils.hpp:265-269)
    const int vy = int(int16_t(uint16_t(ry << (16 - mv))) >> (16 - mv));
    const int cx = clamp16(mx + vx, w - kMB), cy = clamp16(my + vy, h - kMB);
    const int py = l >> 2, px = (l & 3) * 4;
    const uint8_t* sp = ref + size_t(cy + py) * rs + cx + px;
    uint8_t* dp = out + size_t(my + py) * os + mx + px;
#pragma unroll
    for (int j = 0; j < 4; j++) dp[j] = sp[j];
}

}  // namespace

void launch_pframe_mvcopy(const uint8_t* stream, uint64_t start_bit, const uint64_t* dstart, uint64_t nbits, int mv_bits,
                          const uint8_t* ref, uint64_t rs, uint8_t* out, uint64_t os, int w, int h, hipStream_t s) {
    const int nmb = (w / kMB) * (h / kMB);
    if (nmb > 0)
        hipLaunchKernelGGL(pf_mvcopy_kernel, dim3(nmb), dim3(kMbTPB), 0, s, stream, start_bit, dstart, nbits, mv_bits, ref,
                           rs, out, os, w, h, w / kMB);
}

void launch_pframe(const PfArgs& a, int n, uint64_t* tsum, hipStream_t s) {
    const int nmb = a.mbx * a.mby;
    const uint64_t head = uint64_t(nmb) * 2u * uint32_t(a.mv_bits);
    const int nb = a.bx * (a.h / n);
    const size_t px = size_t(a.w) * a.h - size_t(nmb) * kMB * kMB;  // pixels no macroblock covers
    const unsigned grid = unsigned(nmb) + unsigned((px + kMbTPB - 1) / kMbTPB);  // + the strips' workgroups
    if (grid) {
        if (n == 4) hipLaunchKernelGGL(pf_macroblock_kernel<4>, dim3(grid), dim3(kMbTPB), 0, s, a);
        else hipLaunchKernelGGL(pf_macroblock_kernel<8>, dim3(grid), dim3(kMbTPB), 0, s, a);
    }
    if (n == 4 && nmb > 0) {
        const int ntiles = (nb + kPfTileBlocks - 1) / kPfTileBlocks;
        if (a.st) {  // one launch: the scan by look-back
            hipLaunchKernelGGL(pf_emit_chain_kernel, dim3(ntiles), dim3(kTPB), 0, s, a, nb, ntiles, head);
        } else {     // (ticket mode: tiles may not run in dispatch order) tile sums, scan, emission
            hipLaunchKernelGGL(pf_tile_sum_kernel, dim3(ntiles), dim3(kTPB), 0, s, a.bits, nb, tsum);
            hipLaunchKernelGGL(pf_tile_scan_kernel, dim3(1), dim3(kTPB), 0, s, tsum, ntiles, head, a.start, a.end);
            hipLaunchKernelGGL(pf_emit_kernel, dim3(ntiles), dim3(kTPB), 0, s, a, nb, tsum, head);
        }
    } else {
        hipLaunchKernelGGL(pf_end_kernel, dim3(1), dim3(64), 0, s, a.start, a.end, head);
    }
}

int pframe_tiles(int nb) { return (nb + kPfTileBlocks - 1) / kPfTileBlocks; }

}  // namespace ie
