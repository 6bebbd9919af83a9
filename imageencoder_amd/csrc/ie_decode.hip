// imageencoder_amd/csrc/ie_decode.hip -- the inverse path on gfx950 (ImageDecoder.cpp:55-122).
//
// The reference parses block records serially (Block::loadFromStream, Block.cpp:442-472) because
// a record's length is only known once its header is read.  Here the parse is made parallel:
//   walk_kernel   the stream is cut into fixed chunks of bits; one lane walks each chunk from an
//                 entry position, record by record (length = 4 + bl*(rle + Lw) or 4 + bl*N*N),
//                 and reports where it leaves the chunk.  The first walk starts every chunk at its
//                 first bit (speculative); a record header that cannot occur in a real stream
//                 (bl = 0, Lw > N*N) makes the walk slide one bit, so wrong walks quickly fall onto
//                 the true record boundaries.  Fix-up rounds re-walk every chunk whose entry differs
//                 from its predecessor's exit until nothing changes; then chunk 0's exact entry
//                 (start_bit) makes every chunk exact by induction.
//   index_kernel  the final walks write the start bit of every record (block index = exclusive scan
//                 of per-chunk record counts).
//   decode_kernel one lane per block: read bl / Lw / values, sign-extend (utils.hpp:265-269), place
//                 them in zig-zag order, dequantise (Block.cpp:163-169), inverse DCT in the
//                 reference's FP64 order (algo.cpp:343-363), +128, clamp and truncate to uint8
//                 (Block.cpp:100-107).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "ie_common.hpp"
#include "ie_device.h"
#include "ie_recbits.h"

namespace ie {

namespace {
constexpr int kZZ4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
constexpr int kZZ8[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                          12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                          35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                          58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
}  // namespace

// bits [p, p+l) of the stream, l <= 32
__device__ __forceinline__ uint32_t getbits(const uint32_t* W, uint64_t p, int l) {
    if (l == 0) return 0;
    const uint64_t w = p >> 5;
    const uint64_t v = (uint64_t(bswap32(W[w])) << 32) | bswap32(W[w + 1]);
    return uint32_t((v << (p & 31)) >> (64 - l));
}

// ---- Huffman decode (Huffman.cpp:354-402; the per-bit tree walk of :190-204) -------------------
// One lane per chunk of bits decodes symbols with a prefix table until it leaves the chunk; its
// entry comes from composed transfer tables (the exact parse at the end of this file); a scan of
// the per-chunk symbol counts places every chunk's output; a last walk writes the symbols.  The
// reference walks to the end of the buffer, padding bits of the last byte included (a code may run
// past it with zero bits), and so does this walk.
//   lut   [2^15]: sym | len << 8 for every 15-bit prefix, len 0 = no code (codes are <= 15 bits:
//         the dictionary stores lengths in 4 bits, Huffman.cpp:41-42)
//   LDS   the 2^kHufL1 first-level entries (codes of <= kHufL1 bits resolve there)
constexpr int kHufL1 = 11;
constexpr int kHufD = 15;   // entry offsets of a chunk: codes are at most 15 bits
#ifndef IE_HUF_G
#define IE_HUF_G 256
#endif
constexpr int kHufG = IE_HUF_G;  // tables per composition group
struct HufArgs {
    const uint32_t* words;
    uint64_t nbits, start_bit, chunk_bits;
    int nchunks;
    const uint16_t* lut;
    uint64_t* entry;
    uint32_t* count;
    uint32_t* wgsum;    // [walk workgroups] their chunks' symbol totals
    unsigned* changed;  // [1] invalid code on the emitting walk; [0] output past out_cap (not written)
    uint64_t* base;     // symbols before each chunk within its walk workgroup
    uint8_t* out;
    uint16_t* lvl[kRecMaxLevels];  // mode 2: the composition's levels
    int levels;
    const uint32_t* E;
    uint64_t out_cap;   // bytes of out (the emit launched before the total is known checks it)
};

__device__ __forceinline__ void huf_l1(const uint16_t* lut, uint16_t* l1) {
    constexpr int B = 8;  // loads in flight per thread
    for (int q0 = 0; q0 < (1 << kHufL1); q0 += B * int(blockDim.x)) {
        uint16_t e[B];
#pragma unroll
        for (int u = 0; u < B; u++) {
            const int q = q0 + u * int(blockDim.x) + int(threadIdx.x);
            e[u] = q < (1 << kHufL1) ? lut[uint32_t(q) << (15 - kHufL1)] : uint16_t(0);
        }
#pragma unroll
        for (int u = 0; u < B; u++) {
            const int q = q0 + u * int(blockDim.x) + int(threadIdx.x);
            if (q < (1 << kHufL1)) l1[q] = ((e[u] >> 8) != 0 && (e[u] >> 8) <= kHufL1) ? e[u] : uint16_t(0);  // 0: look in lut
        }
    }
    __syncthreads();
}

// The symbols before workgroup g's chunks: the totals of the workgroups before it, summed by the
// whole workgroup (every thread receives it).
__device__ __forceinline__ uint64_t huf_wg_prefix(const uint32_t* wgsum, int g, uint32_t* scratch) {
    uint64_t part = 0;
    for (int i = threadIdx.x; i < g; i += kTPB) part += wgsum[i];
    const uint64_t w = wave_sum64(part);
    if ((threadIdx.x & 63) == 0) reinterpret_cast<uint64_t*>(scratch)[threadIdx.x >> 6] = w;
    __syncthreads();
    const uint64_t* s64 = reinterpret_cast<const uint64_t*>(scratch);
    return s64[0] + s64[1] + s64[2] + s64[3];
}

// total receives the symbol count (device, 1 word): the sum of the walk's workgroup totals.
__global__ __launch_bounds__(kTPB) void huf_total_kernel(const uint32_t* wgsum, int nwg, uint64_t* total) {
    __shared__ alignas(8) uint32_t scratch[8];
    const uint64_t t = huf_wg_prefix(wgsum, nwg, scratch);
    if (threadIdx.x == 0) *total = t;
}

// ---- exact record parse: transfer tables, composed -------------------------------------------
// A record's length depends on its own header, so the stream is a serial chain.  Cut it into
// chunks of C bits.  The first record starting at or after a chunk's first bit sits at an offset
// d < D (D = the longest record, 4 + 15*(N*N+1) bits: the record straddling the boundary ends
// within D bits).  So a chunk is a FUNCTION of d: walking from offset d gives the offset at which
// the walk enters the next chunk -- its transfer table T_k[d] over all D entries.  Tables compose
// (T_{k+1} o T_k), and the true entry of every chunk follows from the stream's start by composing
// tables: exact for any content, with no speculation to converge (periodic streams, which lock
// speculative walks into a wrong phase, cost nothing extra).
//   rec_table2_kernel  the D walks of a chunk share their work through claims in LDS -- the first
//                      walk to reach a position owns it, a later walk that lands there stops and
//                      takes the owner's exit -- so about one walk per chunk survives.
//   rec_compose_kernel one workgroup per group of G tables: the group's tables in LDS, every entry
//                      chased through them; the chase writes the group-relative prefix map P_j
//                      over each table (group entry -> entry of table j) and the group's
//                      composite.  Levels repeat on the composites until at most G remain; the
//                      last workgroup of that level chases the stream's start through them.
//   rec_count_kernel   one wave per chunk: entry = the prefix maps applied to its top-level entry;
//                      the chunk's true records are walked from it: their positions, their count,
//                      and the count added to a sum per 256 chunks.
//   rec_decode_kernel  one wave per chunk: first block index = the sums before the chunk's 256,
//                      plus the counts before it among them (one load per lane, a wave sum); the
//                      lanes decode the records: dequantise (Block.cpp:163-169), FP64 IDCT in the
//                      reference's order (algo.cpp:343-363), +128, clamp, truncate
//                      (Block.cpp:100-107).

constexpr uint32_t kRoot = 0x8000u;  // table pass: a walk result that is an exit, not an owner

// bits [p, p+l) of the LDS stream copy L (MSB-first words), l <= 32, p relative to the copy
__device__ __forceinline__ uint32_t lbits(const uint32_t* L, uint32_t p, int l) {
    const uint32_t w = p >> 5, s = p & 31u;
    const uint64_t v = (uint64_t(L[w]) << 32) | L[w + 1];
    return l ? uint32_t((v << s) >> (64 - l)) : 0u;
}

// length of the record whose 20 header bits (bl:4, then the RLE length's bl bits) are `head`; 1
// if no record can start there (a walk slides one bit; never on the true path of a well-formed
// stream)
template <int N>
__device__ __forceinline__ uint32_t rec_len_head(uint32_t head, int rle) {
    constexpr int NN = N * N;
    const uint32_t bl = head >> 16;
    if (!bl) return 1u;
    if (!rle) return 4u + bl * NN;
    const uint32_t lw = (head & 0xFFFFu) >> (16 - bl);
    return lw <= uint32_t(NN) ? 4u + bl * (lw + 1u) : 1u;
}
// rec_len_head without branches (the walk loops: every lane runs it every step)
template <int N>
__device__ __forceinline__ uint32_t rec_len_sel(uint32_t head, int rle) {
    constexpr uint32_t NN = N * N;
    const uint32_t bl = head >> 16;
    const uint32_t lw = rle ? ((head & 0xFFFFu) >> (16u - bl)) : NN - 1u;  // (bl = 0: shifted out)
    return (bl != 0u && lw <= NN) ? 4u + bl * (lw + 1u) : 1u;
}
// length of the record at p, 0 if no record can start there
template <int N>
__device__ __forceinline__ uint32_t rec_len(const uint32_t* L, uint32_t p, int rle) {
    const uint32_t l = rec_len_head<N>(lbits(L, p, 20), rle);
    return l > 1u ? l : 0u;
}

__host__ __device__ constexpr int rec_table_stream_words(uint32_t C) { return int((C + 95) >> 5) + 3; }
// (a multiple of 4 words, with room for stage_words16's alignment offset)
__host__ __device__ constexpr int rec_decode_stream_words(uint32_t C, int D) { return (int((C + D + 95) >> 5) + 3 + 3 + 3) & ~3; }
// a count wave's LDS words: seg chunks' bits + 64 + alignment slack, a multiple of 4 (16-byte rows)
__host__ __device__ constexpr int rec_count_wave_words(uint32_t C, int seg) {
    return (int((uint64_t(seg) * C + 95) >> 5) + 3 + 3 + 3) & ~3;
}
int rec_count_seg(uint32_t C) {  // chunks per count wave: <= 16, a wave's bits within 10 KB
    return int(std::max<uint64_t>(1, std::min<uint64_t>(16, (uint64_t(10 * 1024) * 8 - 256) / C)));
}


// The stream word w (byte-swapped to MSB-first) with its bits at or past nbits cleared: the last
// word may be read in place from a caller's buffer, whose bytes past the stream are not zero.
__device__ __forceinline__ uint32_t tail_word(uint32_t raw, uint64_t w, uint64_t nbits) {
    const uint32_t b = bswap32(raw);
    const uint64_t vb = nbits - (w << 5);  // valid bits of this word (>= 1)
    return vb >= 32 ? b : (b & ~(0xFFFFFFFFu >> uint32_t(vb)));
}

// Words [w0, w0 + nw) of the stream, byte-swapped to MSB-first, zeros past the stream's nbits,
// with one pad word after every 32 (word i at i + i / 32): lanes walking chunks of
// 1 024 bits side by side read words 32 apart -- one bank -- without it (lbits_pad reads it)
__device__ __forceinline__ void stage_words_pad(uint32_t* L, const uint32_t* W, uint64_t w0, int nw, uint64_t nbits,
                                                int tid, int nthreads) {
    const uint64_t nwords = (nbits + 31) >> 5;
    constexpr int B = 8;
    for (int i0 = 0; i0 < nw; i0 += B * nthreads) {
        uint32_t v[B];
#pragma unroll
        for (int u = 0; u < B; u++) {
            const int i = i0 + u * nthreads + tid;
            const uint64_t w = w0 + i;
            if (i < nw && (w + 1) * 32 <= nbits) {
                v[u] = __builtin_nontemporal_load(W + w);
            } else if (i < nw && w < nwords) {  // the stream's last, partial word: its bytes only (the
                                                // caller's buffer may end there)
                const uint8_t* b = reinterpret_cast<const uint8_t*>(W + w);
                uint32_t x = 0;
                for (uint32_t e = 0; e < 4u && 32 * w + 8 * e < nbits; e++) x |= uint32_t(b[e]) << (8 * e);
                v[u] = x;
            } else {
                v[u] = 0u;
            }
        }
#pragma unroll
        for (int u = 0; u < B; u++) {
            const int i = i0 + u * nthreads + tid;
            if (i < nw) L[i + (i >> 5)] = (w0 + i < nwords) ? tail_word(v[u], w0 + i, nbits) : 0u;
        }
    }
}
__host__ __device__ constexpr int pad_words(int nw) { return nw + (nw >> 5) + 1; }
__device__ __forceinline__ uint32_t lbits_pad(const uint32_t* L, uint32_t p, int l) {
    const uint32_t w = p >> 5, w1 = w + 1u, s = p & 31u;
    const uint64_t v = (uint64_t(L[w + (w >> 5)]) << 32) | L[w1 + (w1 >> 5)];
    return l ? uint32_t((v << s) >> (64 - l)) : 0u;
}

// zig-zag rank of every coefficient position (the inverse of kZZ4 / kZZ8)
template <int N> struct InvZZ {
    int r[N * N];
    constexpr InvZZ() : r() {
        for (int k = 0; k < N * N; k++) r[(N == 4) ? kZZ4[k] : kZZ8[k]] = k;
    }
};

// decode the record at p (relative to L) as block g; returns the bit after it.  Coefficient uv
// (row-major) is value number izz[uv] of the record, read straight from its bit position, so the
// IDCT runs in the reference's uv-ascending order without a zig-zag array.
// sR / sq: the FP64 cos products R[uv][ij] and the quantiser through the constant address space:
// the loads are uniform, so they become scalar loads and the FP64 multiplies take their operands
// from SGPRs
using const_f64 = const __attribute__((address_space(4))) double*;
template <int N>
__device__ __forceinline__ uint32_t decode_record(const uint32_t* L, uint32_t p, uint64_t g, const DecArgs& a,
                                                  const_f64 sR, const_f64 sq) {
    constexpr int NN = N * N;
    constexpr InvZZ<N> izz;
    const int bl = int(lbits(L, p, 4));
    p += 4;
    int length = NN;
    if (a.rle) {
        length = int(lbits(L, p, bl));
        p += bl;
    }
    if (length > NN) length = NN;
    const int sh = 16 - bl;
    double t[NN];
#pragma unroll
    for (int k = 0; k < NN; k++) t[k] = 0.0;
    // Block::processIDCTMulQ: Y *= q, then temp[ij] += R[uv][ij] * Y[uv] over uv ascending.  A
    // zero Y term adds +-0: it leaves every partial sum unchanged but possibly the sign of a zero,
    // which +128 and the clamp erase, so a term is skipped when it is zero in every lane (the
    // branch stays uniform and the R rows come through the scalar cache).
#pragma unroll
    for (int uv = 0; uv < NN; uv++) {
        const int kz = izz.r[uv];
        double y = 0.0;
        if (kz < length) {
            const uint32_t raw = lbits(L, p + uint32_t(kz * bl), bl);
            y = double(int16_t(int16_t(uint16_t(raw << sh)) >> sh)) * sq[uv];  // utils.hpp:265-269
        }
        if (__ballot(y != 0.0)) {
            const_f64 R = sR + uv * NN;
#pragma unroll
            for (int ij = 0; ij < NN; ij++) t[ij] = t[ij] + R[ij] * y;
        }
    }
    const uint64_t bpf = uint64_t(a.bx) * a.by;
    const uint64_t f = g / bpf, r = g - f * bpf;
    const int byi = int(r / a.bx), bxi = int(r - uint64_t(byi) * a.bx);
    uint8_t* o = a.out + f * a.frame_pitch + uint64_t(byi) * N * a.stride + uint64_t(bxi) * N;
#pragma unroll
    for (int i = 0; i < N; i++) {
        uint32_t wv[N / 4];
#pragma unroll
        for (int j = 0; j < N; j++) {
            double x = t[i * N + j] + 128.0;
            if (a.add_base) x = double(o[uint64_t(i) * a.stride + j]) + x;  // expandDifferences
            x = x < 0.0 ? 0.0 : (x > 255.0 ? 255.0 : x);
            const uint32_t b = uint32_t(uint8_t(x));
            if (j % 4 == 0) wv[j / 4] = b;
            else wv[j / 4] |= b << (8 * (j % 4));
        }
        uint8_t* row = o + uint64_t(i) * a.stride;
        if ((reinterpret_cast<uintptr_t>(row) & 3u) == 0) {
#pragma unroll
            for (int m = 0; m < N / 4; m++) reinterpret_cast<uint32_t*>(row)[m] = wv[m];
        } else {
#pragma unroll
            for (int j = 0; j < N; j++) row[j] = uint8_t(wv[j / 4] >> (8 * (j % 4)));
        }
    }
    return p + uint32_t(length * bl);
}

// One composition level over n tables ([n][D], 16-bit exits): prefix maps written over the
// tables, composites into comp ([ceil(n/G)][D]).  Shared by the record parse (D = the longest
// record) and the Huffman decode (D = the longest code).
// n 16-bit entries from global memory into LDS, 16 bytes per load where both sides allow it
// (eight 16-byte loads per thread in flight before their LDS stores: one load-to-store round trip
// per 32 KiB instead of one per 4 KiB)
__device__ __forceinline__ void stage_u16(uint16_t* S, const uint16_t* T, int n, int tid) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    int head = 0;
    if (((reinterpret_cast<uintptr_t>(T) | reinterpret_cast<uintptr_t>(S)) & 15u) == 0) {
        head = n & ~7;
        const int nv = head / 8;
        const u4* src = reinterpret_cast<const u4*>(T);
        u4* dst = reinterpret_cast<u4*>(S);
        for (int i0 = 0; i0 < nv; i0 += 8 * kTPB) {
            u4 v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int i = i0 + u * kTPB + tid;
                if (i < nv) v[u] = src[i];
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int i = i0 + u * kTPB + tid;
                if (i < nv) dst[i] = v[u];
            }
        }
    }
    for (int i = head + tid; i < n; i += kTPB) S[i] = T[i];
}

template <int D, int G>
__global__ __launch_bounds__(kTPB) void compose_kernel(uint16_t* tab, int n, uint16_t* comp) {
    __shared__ __attribute__((aligned(16))) uint16_t S[G * D];
    const int tid = threadIdx.x, g = blockIdx.x;
    const int k0 = g * G, nk = min(G, n - k0);
    uint16_t* T = tab + size_t(k0) * D;
    stage_u16(S, T, nk * D, tid);
    __syncthreads();
    // every entry chased through the group's tables; a thread's entries (tid, tid + kTPB, ...) are
    // chased side by side, so their dependent LDS reads overlap
    constexpr int CH = (D + kTPB - 1) / kTPB;
    uint32_t x[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = uint32_t(tid + c * kTPB);
    for (int j = 0; j < nk; j++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            const int d = tid + c * kTPB;
            if (d < D) {
                T[j * D + d] = uint16_t(x[c]);  // P_j: group entry d -> entry of table j
                x[c] = S[j * D + x[c]];
            }
        }
    }
#pragma unroll
    for (int c = 0; c < CH; c++) {
        const int d = tid + c * kTPB;
        if (d < D) comp[size_t(g) * D + d] = uint16_t(x[c]);
    }
}

// The top chase: the stream's start (entry 0) through the ng <= G top-level composites, E[q] = the
// entry of composite q (one workgroup; a launch of its own, so the composites are visible without
// a device-wide fence in every composing workgroup).  (A segmented chase -- every entry through
// each of 8 segments, then entry 0 through the segment maps -- measured slower here and in
// compose_kernel: 9.2 -> 11.6 and 15.2 -> 18.1 us.)
template <int D, int G>
__global__ __launch_bounds__(kTPB) void compose_top_kernel(const uint16_t* comp, int ng, uint32_t* E) {
    __shared__ __attribute__((aligned(16))) uint16_t S[G * D];
    stage_u16(S, comp, ng * D, threadIdx.x);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t x = 0;
        for (int q = 0; q < ng; q++) {
            E[q] = x;
            x = S[q * D + x];
        }
    }
}

// The composition levels over n tables: level l+1's tables are level l's composites, until at
// most G remain (the top chase).  lvl[l] receives level l's table array; returns the number of
// levels, or -1 past kRecMaxLevels.
template <int D, int G>
int launch_compose(uint16_t* tab, int n, uint32_t* E, unsigned* ticket, uint16_t** lvl, hipStream_t s) {
    int cur = n, levels = 0;
    uint16_t* arr = tab;
    for (;;) {
        const int ng = (cur + G - 1) / G;
        const int top = ng <= G ? 1 : 0;
        if (levels >= kRecMaxLevels) return -1;
        lvl[levels] = arr;
        uint16_t* comp = arr + size_t(cur) * D;
        hipLaunchKernelGGL((compose_kernel<D, G>), dim3(ng), dim3(kTPB), 0, s, arr, cur, comp);
        levels++;
        if (top) {
            hipLaunchKernelGGL((compose_top_kernel<D, G>), dim3(1), dim3(kTPB), 0, s, comp, ng, E);
            (void)ticket;
            return levels;
        }
        arr = comp;
        cur = ng;
    }
}

// Table rows a composition over n tables needs (the tables and every level's composites).
template <int D, int G>
size_t compose_rows(int n) {
    size_t rows = 0;
    for (int cur = n;; cur = (cur + G - 1) / G) {
        rows += size_t(cur);
        if ((cur + G - 1) / G <= G) return rows + size_t((cur + G - 1) / G);
    }
}

// the entry offset of table k: its top-level entry, then the prefix maps of every level down
template <int D, int G>
__device__ __forceinline__ uint32_t table_entry(const uint32_t* E, uint16_t* const* lvl, int levels, int k) {
    int u = k;
    for (int l = 0; l < levels; l++) u /= G;
    uint32_t x = E[u];
    for (int l = levels - 1; l >= 0; l--) {
        int ul = k;
        for (int m = 0; m < l; m++) ul /= G;
        x = lvl[l][size_t(ul) * D + x];
    }
    return x;
}

// the chunk's entry offset (record parse): composed tables, or the predecessor's speculative exit
template <int N>
__device__ __forceinline__ uint32_t rec_chunk_entry(const RecParseArgs& a, int k) {
    if (a.spec) return k ? a.spec[k - 1] : 0u;
    return table_entry<RecGeom<N>::D, RecGeom<N>::G>(a.E, a.lvl, a.levels, k);
}

// The record span of a launch: [start, nbits) -- the host's, or, device-chained (a.dstart), from
// an earlier launch's end bit (clamped to the stream; ~0 = that launch found no end) for at most
// a.span bits.  Chunks past the span's end see no stream bits and hold no record.
struct RecSpan {
    uint64_t start, nbits;
};
__device__ __forceinline__ RecSpan rec_span(const RecParseArgs& a) {
    if (!a.dstart) return {a.start_bit, a.nbits};
    const uint64_t st = min(min(*a.dstart, a.nbits) + a.start_add, a.nbits);
    return {st, min(a.nbits, st + a.span)};
}
__device__ __forceinline__ uint64_t sat_sub(uint64_t x, uint64_t y) { return x > y ? x - y : 0ull; }

// L[i] = bswap(W[w0 + i]) for i < nw (zeros past nwords) by one wave with 16-byte loads, four
// per lane in flight; L must be 16-byte aligned.  The copy starts at the aligned word w0 & ~3:
// returns the offset of word w0 in L (0..3).
__device__ __forceinline__ int stage_words16(uint32_t* L, const uint32_t* W, uint64_t w0, int nw, uint64_t nbits,
                                             int lane) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const uint64_t wa = w0 & ~3ull;
    const int off = int(w0 - wa);
    const int nq = (nw + off + 3) >> 2;  // 16-byte groups
    const uint64_t nwords = (nbits + 31) >> 5;
    const uint64_t nfull = (nbits >> 5) >> 2;  // groups of whole words wholly inside the stream
    for (int q0 = 0; q0 < nq; q0 += 64 * 4) {
        u4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int q = q0 + u * 64 + lane;
            const uint64_t g = (wa >> 2) + uint64_t(q);
            if (q < nq && g < nfull) {
                v[u] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(W) + g);
            } else {
                u4 z = {0u, 0u, 0u, 0u};  // (kept byte-swapped back: the store below swaps again)
                if (q < nq)
                    for (int e = 0; e < 4; e++)
                        if (4 * g + e < nwords) z[e] = bswap32(tail_word(W[4 * g + e], 4 * g + e, nbits));
                v[u] = z;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int q = q0 + u * 64 + lane;
            if (q < nq) {
                u4 b = {bswap32(v[u].x), bswap32(v[u].y), bswap32(v[u].z), bswap32(v[u].w)};
                reinterpret_cast<u4*>(L)[q] = b;
            }
        }
    }
    return off;
}

// Table pass, round 3: one wave tabulates tm consecutive chunks (runtime, rec_table_geometry) and
// walks only from positions where a record can start.  Entry d of a chunk first slides to the next
// valid position nv(d) -- every entry between two valid positions shares one walk -- so the walks
// start at the valid positions of [0, min(D, C)) plus, for the entries past the last of them, the
// first valid position after (v*, entry slot D of the chunk).  The walk list is compacted from the
// bitmap and lanes take walks from it as theirs end, across all tm chunks, so a wave's 64 lanes
// carry several chunks' surviving walks side by side.  Claims: one open-addressing table per wave,
// keyed by the wave-relative position (walks of different chunks never meet: a walk stops at its
// chunk's end).  Results: a walk that merged takes its owner's exit (owner chains are read-only
// chases; only non-roots are written).  The valid-header bitmap comes 32 positions at a time from
// bitwise operations on shifted windows (valid_mask32, ie_recbits.h).
// The first valid position at or after p before ce (ce: a chunk end, a multiple of 32), else ce.
// NZ[i]: the first bitmap word at or after word i holding a valid position (a sentinel past the
// last), so a run of positions where no record can start costs one read, not one per word.
template <int N>
__device__ __forceinline__ uint32_t next_valid(const uint32_t* VB, const uint16_t* NZ, uint32_t p, uint32_t ce) {
    if (p >= ce) return p;
    uint32_t wi = p >> 5, msk = VB[wi] & (0xFFFFFFFFu << (p & 31u));
    if (!msk) {
        wi = NZ[wi + 1];
        if (wi >= (ce >> 5)) return ce;
        msk = VB[wi];
    }
    return (wi << 5) + uint32_t(__builtin_ctz(msk));
}

// next_valid without branches, for the loops every lane runs: the bitmap word, the next non-empty
// word and that word's bits are all read (the last only matters past an empty word); word
// indices are clamped to the chunk's last bitmap word, so every read stays inside the chunk.
__device__ __forceinline__ uint32_t next_valid_sel(const uint32_t* VB, const uint16_t* NZ, uint32_t p, uint32_t ce) {
    const uint32_t cw = (ce >> 5) - 1u;  // the chunk's last bitmap word
    const uint32_t wi = min(p >> 5, cw), nz = NZ[wi + 1];
    const uint32_t mk = VB[wi] & (0xFFFFFFFFu << (p & 31u));
    const uint32_t m2 = VB[min(uint32_t(nz), cw)];
    const uint32_t q = mk ? (wi << 5) + uint32_t(__builtin_ctz(mk))
                          : (nz <= cw ? (uint32_t(nz) << 5) + uint32_t(__builtin_ctz(m2)) : ce);
    return p >= ce ? p : q;
}

__host__ __device__ constexpr int rec_table2_words(uint32_t C, int D, int tm, int hbits) {
    // L (stream words, 16-byte aligned staging: +4), VB, claims, then the u16 walk results (an
    // exit with kRoot set, or the owner a merged walk joined), the u16 walk list (walk ids: the
    // start position follows from the id, except a chunk's v*), the chunks' v* positions and the
    // u16 next-valid-word table (tm CW + 1 entries)
    return (rec_table_stream_words(uint32_t(tm) * C) + 4 + 3) / 4 * 4 + tm * int(C >> 5) + (1 << hbits) +
           2 * ((tm * (D + 1) + 1) / 2) + tm + (tm * int(C >> 5) + 2) / 2;
}

template <int N>
__global__ __launch_bounds__(64) void rec_table2_kernel(RecParseArgs a) {
    constexpr int D = RecGeom<N>::D, D1 = D + 1;
    extern __shared__ __attribute__((aligned(16))) uint32_t Ls[];
    const int lane = threadIdx.x, tm = a.tm;
    const int k0 = blockIdx.x * tm;
    const int m = min(tm, a.nchunks - k0);
    const uint32_t C = a.C, CW = C >> 5;
#if IE_PROFILE
    unsigned long long* ws = a.wstamp ? a.wstamp + size_t(blockIdx.x) * 8 : nullptr;
    auto wstamp = [&](int i) {
        if (ws && lane == 0) ws[i] = __builtin_amdgcn_s_memrealtime();
    };
    wstamp(0);
#else
    auto wstamp = [](int) {};
#endif
    const int SW = (rec_table_stream_words(uint32_t(tm) * C) + 4 + 3) / 4 * 4;
    uint32_t* L = Ls;
    uint32_t* VB = Ls + SW;
    uint32_t* H = VB + tm * int(CW);
    const uint32_t HM = (1u << a.hbits) - 1u;
    // res[id]: kRoot | the exit of a walk that left its chunk, or the id of the walk it merged into
    // (ids < D1 * tm < kRoot; one u16 per walk keeps a wave in 4.8 KB of LDS: 32 waves per CU)
    uint16_t* res = reinterpret_cast<uint16_t*>(H + HM + 1);
    const int RW = (tm * D1 + 1) / 2;                                  // words of res, and of wl
    uint16_t* wl = reinterpret_cast<uint16_t*>(H + HM + 1 + RW);
    uint32_t* vst = H + HM + 1 + 2 * RW;                               // [tm] every chunk's v* position
    uint16_t* NZ = reinterpret_cast<uint16_t*>(vst + tm);
    const RecSpan sp = rec_span(a);
    const uint64_t c0 = sp.start + uint64_t(k0) * C;
    const uint64_t base = c0 & ~31ull;
    const int off = stage_words16(L, a.words, base >> 5, int(((c0 - base) + uint64_t(m) * C + 64) >> 5) + 2,
                                  sp.nbits, lane);
    const uint32_t s0 = uint32_t(c0 - base) + 32u * uint32_t(off);  // the wave's first bit in L
    // positions below are relative to s0; no record starts at or past the stream's end
    const uint32_t lim = uint32_t(min<uint64_t>(sat_sub(sp.nbits, c0), uint64_t(m) * C));
    for (uint32_t i = lane; i <= HM; i += 64) H[i] = 0xFFFFFFFFu;
    __syncthreads();
    wstamp(1);
    // 1. valid-header bitmap, 32 positions per word
    for (uint32_t i = lane; i < uint32_t(m) * CW; i += 64) {
        const uint32_t p0 = i << 5;
        uint32_t msk = 0;
        if (p0 < lim) {
            const uint32_t q = s0 + p0, w0 = q >> 5, sb = q & 31u;
            const uint64_t v = (((uint64_t(L[w0]) << 32) | L[w0 + 1]) << sb) |
                               (sb ? (uint64_t(L[w0 + 2]) >> (32 - sb)) : 0ull);
            msk = valid_mask32<N>(v, a.rle);
            const uint32_t cut = lim - p0;
            if (cut < 32u) msk &= (1u << cut) - 1u;
        }
        VB[i] = msk;
    }
    __syncthreads();
    {  // NZ: a suffix minimum over the bitmap words, 64 at a time from the end (lane l takes
       // word b0 + 63 - l, so the suffix is a DPP prefix over the lanes)
        const uint32_t nwd = uint32_t(m) * CW;
        uint32_t carry = nwd;
        for (int b0 = int((nwd - 1) & ~63u); b0 >= 0; b0 -= 64) {
            const uint32_t i = uint32_t(b0 + 63 - lane);
            const uint32_t v = min(wave_incl_min_dpp((i < nwd && VB[i]) ? i : nwd), carry);
            if (i < nwd) NZ[i] = uint16_t(v);
            carry = __builtin_amdgcn_readlane(v, 63);
        }
        if (lane == 0) NZ[nwd] = uint16_t(nwd);
    }
    __syncthreads();
    wstamp(2);
    // 2. the walk list: valid positions of [0, min(D, C)) of every chunk, then every chunk's v*
    const uint32_t De = min(uint32_t(D), C), DW = (De + 31) >> 5;
    uint32_t nw = 0;  // (wave-uniform)
    for (uint32_t i0 = 0; i0 < uint32_t(m) * DW; i0 += 64) {
        const uint32_t i = i0 + lane;
        uint32_t bits = 0, j = 0, w = 0;
        if (i < uint32_t(m) * DW) {
            j = i / DW;
            w = i - j * DW;
            bits = VB[j * CW + w];
            const uint32_t rem = De - (w << 5);
            if (rem < 32u) bits &= (1u << rem) - 1u;
        }
        const uint32_t cnt = __popc(bits);
        uint32_t incl = cnt;  // inclusive scan over the wave
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(incl, d, 64);
            if (lane >= d) incl += o;
        }
        uint32_t at = nw + incl - cnt;
        while (bits) {
            const uint32_t b = __builtin_ctz(bits);
            bits &= bits - 1u;
            wl[at++] = uint16_t(j * D1 + (w << 5) + b);  // (starts at j C + (w << 5) + b)
        }
        nw += __shfl(incl, 63, 64);
    }
    {
        uint32_t vs = 0xFFFFFFFFu;
        if (lane < m && De < C) {
            const uint32_t cs = uint32_t(lane) * C, ce = cs + C;
            const uint32_t v = next_valid<N>(VB, NZ, cs + De, ce);
            if (v < ce) vs = v;
        }
        const uint64_t bm = __ballot(vs != 0xFFFFFFFFu);
        if (vs != 0xFFFFFFFFu) {
            const uint32_t r = __builtin_amdgcn_mbcnt_hi(uint32_t(bm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(bm), 0u));
            wl[nw + r] = uint16_t(uint32_t(lane) * D1 + D);
            vst[lane] = vs;
        }
        nw += uint32_t(__popcll(bm));
    }
    __syncthreads();
    wstamp(3);
    // 3. the walks: lanes take the next walk of the list as theirs ends
    {
        uint32_t nxt = 0, p = 0, id = 0, ce = 0, nsteps = 0, wsteps = 0, rsteps = 0;
        bool act = false;
        // One step of an active walk at p (< ce, a valid position): the record's header, the claim
        // and the next position.  The claim's result is read last, so the atomic's round trip
        // overlaps the header read and the bitmap reads of the next position.  The claim table is
        // direct-mapped and lossy: a slot another position holds is not probed on -- the walk goes
        // on unclaimed there and meets its owner's claims further on.
        auto walk_step = [&]() {
            nsteps++;
            wsteps++;
            const uint32_t head = lbits(L, s0 + p, 20);
            const uint32_t o = atomicCAS(&H[(p * 2654435761u) >> 16 & HM], 0xFFFFFFFFu, (p << 16) | id);
            const uint32_t np = next_valid_sel(VB, NZ, p + rec_len_sel<N>(head, a.rle), ce);
            if (o != 0xFFFFFFFFu && (o >> 16) == p) {  // an earlier walk was here: take its exit
                res[id] = uint16_t(o & 0xFFFFu);
                act = false;
                wsteps = 0;
            } else if (np >= ce) {  // left the chunk
                res[id] = uint16_t(kRoot | (np - ce));
                act = false;
                rsteps += wsteps;  // (profiling: steps of walks that reached the chunk's end)
                wsteps = 0;
            } else {
                p = np;
            }
        };
        // (a) while the list lasts: idle lanes take the next walks, every step claims its position
        // (claiming 4-16 steps longer measured equal or slower)
        while (nxt < nw) {  // (wave-uniform)
            const uint64_t need = __ballot(!act);
            if (!act) {
                const uint32_t r = nxt + __builtin_amdgcn_mbcnt_hi(uint32_t(need >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(need), 0u));
                if (r < nw) {
                    id = wl[r];
                    const uint32_t j = id / D1, d = id - j * D1;
                    p = (d < uint32_t(D)) ? j * C + d : vst[j];  // (< the chunk's end: d < min(D, C))
                    ce = (j + 1u) * C;
                    act = true;
                }
            }
            nxt += uint32_t(__popcll(need));
            if (act) walk_step();
        }
        // (b) the list is empty.  The walks still going are many (a lane per walk when the list ran
        // out, most of them on the same few paths).  8x8: they keep claiming until every lane's walk
        // has left its chunk or merged -- they merge into each other.  4x4: they run to the chunk's
        // end unclaimed, a third cheaper per step.  Measured on one 4K noise frame (tools/ab.py --op
        // decode, same process): claims to the end take the 4x4 walk from 575 to 222 lane-steps per
        // chunk and 47.6 to 32.7 steps of the longest lane (tools/dec_stamps.py), yet the decode
        // 132.0 -> 135.4 us; 8x8 210.3 -> 206.6 us.
        constexpr bool kClaimToEnd = N == 8;
        if (kClaimToEnd) {
            while (__ballot(act)) {
                if (act) walk_step();
            }
        } else if (act) {
            while (p < ce) {
                nsteps++;
                wsteps++;
                p = next_valid_sel(VB, NZ, p + rec_len_sel<N>(lbits(L, s0 + p, 20), a.rle), ce);
            }
            res[id] = uint16_t(kRoot | (p - ce));
            rsteps += wsteps;
        }
#if IE_PROFILE
        if (ws) {
            const uint32_t mx = __reduce_max_sync(~0ull, nsteps);
            const uint32_t sm = __reduce_add_sync(~0ull, nsteps);
            const uint32_t rs = __reduce_add_sync(~0ull, rsteps);
            if (lane == 0) {
                ws[6] = (uint64_t(mx) << 32) | sm;
                ws[7] = (uint64_t(nw) << 32) | rs;  // walks, steps of the walks that left the chunk
            }
        }
#endif
        (void)nsteps;
        (void)rsteps;
    }
    __syncthreads();
    wstamp(4);
    // 4. merged walks take their root's exit.  A lane may overwrite an entry another lane's chase
    // passes through: it writes the root's own value (kRoot | exit), so that chase ends there with
    // the same answer.
    for (uint32_t r = lane; r < nw; r += 64) {
        const uint32_t id = wl[r];
        uint32_t x = res[id];
        if (x & kRoot) continue;
        while (!(x & kRoot)) x = res[x];
        res[id] = uint16_t(x);
    }
    __syncthreads();
    // 5. every entry: its walk's exit
    uint16_t* T = a.tab + size_t(k0) * D;
    for (uint32_t e = lane; e < uint32_t(m) * D; e += 64) {
        const uint32_t j = e / D, d = e - j * D;
        uint32_t out;
        if (d >= C) {
            out = d - C;
        } else {
            const uint32_t cs = j * C, ce = cs + C;
            const uint32_t nv = next_valid_sel(VB, NZ, cs + d, ce);
            if (nv >= ce) {
                out = nv - ce;
            } else {
                out = res[j * D1 + min(nv - cs, uint32_t(D))] & ~kRoot;
            }
        }
        T[e] = uint16_t(out);
    }
    wstamp(5);
}

// Speculative pass: one lane per chunk k walks from the first bit of chunk k - W (W = a.warm
// chunks of warm-up; from the stream's first record, an exact entry, when k - W <= 0) through chunk
// k, sliding one bit past positions where no record can start, and stores where it leaves chunk k.
// A walk from an arbitrary bit meets the true record boundaries after a few records on typical
// content, long before the warm-up ends; the count pass proves it did (or flags the stream).
template <int N>
__global__ __launch_bounds__(kTPB) void rec_spec_kernel(RecParseArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t Lall[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int seg = a.seg, W = a.warm;
    const int k0 = (blockIdx.x * 4 + wv) * seg;
    const int m = max(0, min(seg, a.nchunks - k0));
    if (blockIdx.x == 0 && tid == 0) *a.fail = 0u;  // (the count pass runs after this launch)
    if (m == 0) return;
    const int kw = max(k0 - W, 0);  // the wave's first staged chunk
    uint32_t* L = Lall + size_t(wv) * rec_count_wave_words(a.C, seg + W);
    const RecSpan sp = rec_span(a);
    const uint64_t c0 = sp.start + uint64_t(kw) * a.C;
    const uint64_t base = c0 & ~31ull;
    const int off = stage_words16(L, a.words, base >> 5,
                                  int(((c0 - base) + uint64_t(k0 + m - kw) * a.C + 64) >> 5) + 2, sp.nbits, lane);
    const uint32_t s0 = uint32_t(c0 - base) + 32u * uint32_t(off);  // chunk kw's first bit in L
    wave_sync();
    const int k = k0 + lane;
    if (lane < m && k < a.nchunks - 1) {  // (the last chunk's exit enters nothing)
        const uint32_t ce = s0 + uint32_t(k + 1 - kw) * a.C;
        uint32_t p = s0 + uint32_t(max(k - W, 0) - kw) * a.C;
        while (p < ce) p += rec_len_head<N>(lbits(L, p, 20), a.rle);
        a.spec[k] = p - ce;
    }
}

// Count pass: each wave stages `seg` consecutive chunks' bits in LDS and one lane per chunk walks
// its true records from its entry (the prefix maps applied to its top-level entry), storing up to
// kRecPosCap record positions (relative to the chunk's first word) and the count; the workgroup
// then scans its 4 * seg chunks' counts (records before each chunk among them, and their total).
template <int N>
__global__ __launch_bounds__(kTPB) void rec_count_kernel(RecParseArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t Lall[];
    __shared__ alignas(8) uint32_t scratch[8];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int seg = a.seg;
    const int k0 = (blockIdx.x * 4 + wv) * seg;  // this wave's first chunk
    const int m = max(0, min(seg, a.nchunks - k0));
    uint32_t* L = Lall + size_t(wv) * rec_count_wave_words(a.C, seg);
    uint32_t s0 = 0;
    const RecSpan sp = rec_span(a);
    if (m > 0) {
        const uint64_t c0 = sp.start + uint64_t(k0) * a.C;
        const uint64_t base = c0 & ~31ull;
        const int off = stage_words16(L, a.words, base >> 5, int(((c0 - base) + uint64_t(m) * a.C + 64) >> 5) + 2,
                                      sp.nbits, lane);
        s0 = uint32_t(c0 - base) + 32u * uint32_t(off);  // the wave's first bit, relative to L
    }
    const int k = k0 + lane;
    const bool mine = lane < m;
    const uint32_t x = mine ? rec_chunk_entry<N>(a, k) : 0u;
    wave_sync();
    uint32_t R = 0;
    if (mine) {
        const uint64_t c0 = sp.start + uint64_t(k0) * a.C;  // = bit s0 of L
        const uint32_t lim = uint32_t(min<uint64_t>(sat_sub(sp.nbits, c0) + s0, uint64_t(s0) + uint64_t(m) * a.C));
        const uint32_t cs = s0 + uint32_t(lane) * a.C;
        const uint32_t cb = cs & ~31u;  // the chunk's first word
        const uint32_t ce = min(cs + a.C, lim);  // no record starts at or past the stream's end
        uint16_t* pos = a.pos + size_t(k) * kRecPosCap;
        uint32_t p = cs + x;
        while (p < ce) {
            const uint32_t l = rec_len_sel<N>(lbits(L, p, 20), a.rle);
            if (l > 1u) {
                if (R < uint32_t(kRecPosCap)) pos[R] = uint16_t(p - cb);
                R++;
            }
            p += l;
        }
        // speculative entries: this walk started at the true entry if every earlier one did; its
        // exit must be the entry the next chunk's walk took
        if (a.spec && k < a.nchunks - 1 && p - (cs + a.C) != a.spec[k]) *a.fail = 1u;
    }
    // records before each chunk within the workgroup (thread order = chunk order; idle lanes add 0)
    uint32_t tot;
    const uint32_t ex = block_excl_scan(R, scratch, &tot);
    if (mine) {
        a.cnt[k] = R;
        a.lbase[k] = ex;
    }
    if (tid == 0) a.wgsum[blockIdx.x] = tot;
}

// Decode pass: a wave decodes the records of kDecChunks consecutive chunks (about 64 records: a
// chunk holds about 32), one record per lane, so the FP64 IDCT -- the pass's cost -- runs on full
// waves.  Record positions come from the count pass (relative to each chunk's first word; chunk j
// of the wave starts j * C bits after chunk 0, C a multiple of 32).
template <int N>
__global__ __launch_bounds__(64 * kRecWPB) void rec_decode_kernel(RecParseArgs a, DecArgs d) {
    constexpr int D = RecGeom<N>::D;
    constexpr int P = kDecChunks;
    extern __shared__ __attribute__((aligned(16))) uint32_t dyn_all[];  // per wave: the P chunks' bits + D + 64
    const const_f64 sR = (const_f64)(d.tab->R);
    const const_f64 sq = (const_f64)(d.tab->qd);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int k0 = (blockIdx.x * kRecWPB + wv) * P;
    if (k0 >= a.nchunks) return;
    if (a.spec && *a.fail) {  // a speculative entry was wrong: nothing is written, the host re-runs
        if (k0 == 0 && lane == 0) *a.total = ~0ull;
        return;
    }
    const int m = min(P, a.nchunks - k0);
    uint32_t* L = dyn_all + size_t(wv) * rec_decode_stream_words(uint32_t(P) * a.C, D);
    const RecSpan sp = rec_span(a);
    const uint64_t c0 = sp.start + uint64_t(k0) * a.C;
    const uint64_t base = c0 & ~31ull;
    // the chunks' bits first (16-byte loads in flight while the indices below are read); bit
    // positions in L are relative to word `off` of L, which holds the first chunk's first word
    const int off = stage_words16(L, a.words, base >> 5, int((uint32_t(c0 - base) + uint32_t(m) * a.C + D + 64) >> 5) + 2,
                                  sp.nbits, lane);
    const uint32_t ob = 32u * uint32_t(off);
    const uint32_t s0 = uint32_t(c0 - base) + ob;
    const uint64_t lbase0 = base - ob;  // stream bit of L's bit 0
    // first block index: the totals of the count pass's workgroups before chunk k0's, plus the
    // records before it in its own (no separate scan launch); the next chunks follow on
    uint64_t part = 0;
    for (int g = lane; g < k0 / (4 * a.seg); g += 64) part += a.wgsum[g];
    const uint64_t first = wave_sum64(part) + a.lbase[k0];
    uint32_t R[P], Rall = 0;
    bool listed = true;
#pragma unroll
    for (int j = 0; j < P; j++) {
        R[j] = j < m ? a.cnt[k0 + j] : 0u;
        Rall += R[j];
        listed = listed && R[j] <= uint32_t(kRecPosCap);
    }
    if (k0 + m == a.nchunks && lane == 0) *a.total = first + Rall;
    wave_sync();
    const uint64_t nblocks = uint64_t(d.nframes) * d.bx * d.by;
    if (listed) {
        for (uint32_t i = lane; i < Rall; i += 64) {
            const uint64_t b = first + i;
            if (b >= nblocks) break;
            uint32_t j = 0, r = i;
#pragma unroll
            for (int jj = 0; jj < P - 1; jj++)
                if (j == uint32_t(jj) && r >= R[jj]) {
                    r -= R[jj];
                    j++;
                }
            const uint32_t q = decode_record<N>(L, ob + j * a.C + a.pos[size_t(k0 + j) * kRecPosCap + r], b, d, sR, sq);
            if (b == nblocks - 1) *a.end_out = lbase0 + q;
        }
        return;
    }
    // a chunk with more records than its position list holds: walk the chunks again, 64 records
    // at a time
    uint64_t gi = first;
    for (int j = 0; j < m; j++) {
        uint32_t p = s0 + uint32_t(j) * a.C + rec_chunk_entry<N>(a, k0 + j);
        const uint32_t wend = uint32_t(min<uint64_t>(s0 + uint64_t(j + 1) * a.C, sat_sub(sp.nbits, lbase0)));
        while (p < wend && gi < nblocks) {
            uint32_t mine = 0, n = 0;
            while (n < 64u && p < wend) {
                const uint32_t len = rec_len<N>(L, p, d.rle);
                if (!len) {
                    p++;
                    continue;
                }
                if (n == uint32_t(lane)) mine = p;
                n++;
                p += len;
            }
            const uint64_t b = gi + lane;
            if (uint32_t(lane) < n && b < nblocks) {
                const uint32_t q = decode_record<N>(L, mine, b, d, sR, sq);
                if (b == nblocks - 1) *a.end_out = lbase0 + q;
            }
            gi += n;
        }
    }
}

int rec_group_chunks(int n) { return n == 4 ? RecGeom<4>::G : RecGeom<8>::G; }
int rec_entry_span(int n) { return n == 4 ? RecGeom<4>::D : RecGeom<8>::D; }
// chunks per table wave and claim slots: tm chunks' positions fit the 16-bit claim keys.  The
// claim table is small on purpose (lossy, direct-mapped): measured on 4K streams, the occupancy a
// small LDS footprint buys beats the merges a larger table finds (IE_REC_TM / IE_REC_HB override)
void rec_table_geometry(uint32_t C, int n, int* tm, int* hbits) {
    static const char* et = getenv("IE_REC_TM");
    static const char* eh = getenv("IE_REC_HB");
    int t = et ? atoi(et) : (n == 4 ? 2 : 1);
    while (t > 1 && uint64_t(t) * C > 65535u) t--;
    t = std::max(1, t);
    int hb = eh ? atoi(eh) : ((n == 4 ? 7 : 9) + (t >= 4 ? 2 : t >= 2 ? 1 : 0));
    *tm = t;
    *hbits = std::min(14, std::max(6, hb));
}
size_t rec_decode_lds(uint32_t C, int n) {
    return size_t(rec_decode_stream_words(uint32_t(kDecChunks) * C, rec_entry_span(n))) * 4 * kRecWPB;
}

int launch_rec_parse_decode(RecParseArgs a, const DecArgs& d, int n, hipStream_t s) {
    if (a.nchunks <= 0) return 0;
    const int nb = (a.nchunks + kRecWPB * kDecChunks - 1) / (kRecWPB * kDecChunks);  // decode blocks
    const int nt = (a.nchunks + RecGeom<4>::M - 1) / RecGeom<4>::M;  // table waves (M chunks each)
    (void)nt;
    rec_table_geometry(a.C, n, &a.tm, &a.hbits);
    const int nt2 = (a.nchunks + a.tm - 1) / a.tm;
    const size_t l2 = size_t(rec_table2_words(a.C, rec_entry_span(n), a.tm, a.hbits)) * 4;
    if (n == 4) hipLaunchKernelGGL((rec_table2_kernel<4>), dim3(nt2), dim3(64), l2, s, a);
    else hipLaunchKernelGGL((rec_table2_kernel<8>), dim3(nt2), dim3(64), l2, s, a);
    const int levels = (n == 4) ? launch_compose<RecGeom<4>::D, RecGeom<4>::G>(a.tab, a.nchunks, a.E, a.ticket + 1, a.lvl, s)
                                : launch_compose<RecGeom<8>::D, RecGeom<8>::G>(a.tab, a.nchunks, a.E, a.ticket + 1, a.lvl, s);
    if (levels < 0) return -1;
    a.levels = levels;
    const int nbc = (a.nchunks + 4 * a.seg - 1) / (4 * a.seg);
    const size_t lc = size_t(rec_count_wave_words(a.C, a.seg)) * 4 * 4;
    if (n == 4) hipLaunchKernelGGL((rec_count_kernel<4>), dim3(nbc), dim3(kTPB), lc, s, a);
    else hipLaunchKernelGGL((rec_count_kernel<8>), dim3(nbc), dim3(kTPB), lc, s, a);
    if (n == 4) hipLaunchKernelGGL((rec_decode_kernel<4>), dim3(nb), dim3(64 * kRecWPB), rec_decode_lds(a.C, 4), s, a, d);
    else hipLaunchKernelGGL((rec_decode_kernel<8>), dim3(nb), dim3(64 * kRecWPB), rec_decode_lds(a.C, 8), s, a, d);
    return levels;
}

__global__ void gop_init_kernel(uint64_t* pos, uint64_t* tot, int n, uint64_t start) {
    for (int i = threadIdx.x; i <= n; i += blockDim.x) {
        pos[i] = i ? ~0ull : start;
        if (i < n) tot[i] = 0;
    }
}
void launch_gop_init(uint64_t* pos, uint64_t* tot, int n, uint64_t start, hipStream_t s) {
    hipLaunchKernelGGL(gop_init_kernel, dim3(1), dim3(256), 0, s, pos, tot, n, start);
}

void launch_rec_spec_decode(const RecParseArgs& a, const DecArgs& d, int n, hipStream_t s) {
    if (a.nchunks <= 0) return;
    const int nb = (a.nchunks + kRecWPB * kDecChunks - 1) / (kRecWPB * kDecChunks);
    const int nbc = (a.nchunks + 4 * a.seg - 1) / (4 * a.seg);
    const size_t lc = size_t(rec_count_wave_words(a.C, a.seg)) * 4 * 4;
    const size_t lw = size_t(rec_count_wave_words(a.C, a.seg + a.warm)) * 4 * 4;
    if (n == 4) {
        hipLaunchKernelGGL((rec_spec_kernel<4>), dim3(nbc), dim3(kTPB), lw, s, a);
        hipLaunchKernelGGL((rec_count_kernel<4>), dim3(nbc), dim3(kTPB), lc, s, a);
        hipLaunchKernelGGL((rec_decode_kernel<4>), dim3(nb), dim3(64 * kRecWPB), rec_decode_lds(a.C, 4), s, a, d);
    } else {
        hipLaunchKernelGGL((rec_spec_kernel<8>), dim3(nbc), dim3(kTPB), lw, s, a);
        hipLaunchKernelGGL((rec_count_kernel<8>), dim3(nbc), dim3(kTPB), lc, s, a);
        hipLaunchKernelGGL((rec_decode_kernel<8>), dim3(nb), dim3(64 * kRecWPB), rec_decode_lds(a.C, 8), s, a, d);
    }
}

// ---- exact Huffman parse: the same transfer tables --------------------------------------------
// A code is at most 15 bits long, so the first code that starts at or after a chunk's first bit
// sits at an offset d < 15: a chunk of the Huffman stream is a function of d exactly like a chunk
// of the record stream, with 15 entries instead of D.  huf_table_kernel walks all 15 entries of
// kHufTC chunks per workgroup (the chunks' bits staged in LDS; a position where no code
// starts slides one bit -- never on the true path of a valid stream); compose_kernel composes the
// tables; huf_count_kernel reads each chunk's symbol count at its true entry, and huf_emit_kernel
// writes the symbols.  Exact for any content: a periodic stream (e.g. a
// flat image's records, Huffman-coded) no longer leaves speculative walks locked in a wrong phase.
// Walks from different entries of a chunk fall onto the same code boundaries after a few codes
// (prefix codes resynchronise), so only the first kHufSync bits are walked from all 15 entries: the
// walks that stand on the same first boundary at or past cs + kHufSync have merged; one walk per
// distinct boundary (almost always one per chunk) goes on to the chunk's end, the workgroup's
// survivors side by side.  Every entry also gets its symbol count to the exit (cnt), so the true
// path's counts follow from the composed entries without another walk (huf_count_kernel).
#ifndef IE_HUF_SYNC
#define IE_HUF_SYNC 64
#endif
constexpr uint32_t kHufSync = IE_HUF_SYNC;
#ifndef IE_HUF_TC
#define IE_HUF_TC 64
#endif
constexpr int kHufTC = IE_HUF_TC;  // chunks per table workgroup: its survivors fill a wave
__global__ __launch_bounds__(kTPB) void huf_table_kernel(HufArgs a, uint16_t* tab, uint16_t* cnt, uint16_t* mo,
                                                          uint16_t* mc) {
    constexpr int S = kHufTC * 16, U = S / kTPB;  // walk slots (chunk, entry); slots per thread
    static_assert(S % kTPB == 0, "whole slots per thread");
    __shared__ uint16_t l1[1 << kHufL1];
    __shared__ uint32_t P[S], X[S], R[S + 1];  // boundary after the sync walk; exit; survivors
    __shared__ uint16_t K2[S];                 // a survivor's codes from P to its exit
    __shared__ uint32_t M[S];                  // its first boundary at or past the chunk's middle
    __shared__ uint16_t KM[S];                 // its codes from P to that boundary
    extern __shared__ uint32_t L[];            // the workgroup's chunks' bits (+ 64 past the last)
    const int tid = threadIdx.x;
    if (tid == 0) R[S] = 0u;
    const int k0 = blockIdx.x * kHufTC;
    const uint32_t C = uint32_t(a.chunk_bits);
    const int m = min(kHufTC, a.nchunks - k0);
    const uint64_t c0 = a.start_bit + uint64_t(k0) * C;
    const uint64_t base = c0 & ~31ull;
    const uint32_t s0 = uint32_t(c0 - base);
    stage_words_pad(L, a.words, base >> 5, int((s0 + uint32_t(m) * C + 64) >> 5) + 2, a.nbits, tid, kTPB);
    huf_l1(a.lut, l1);  // (ends with a barrier: L staged too)
    const uint32_t lim = uint32_t(min<uint64_t>(a.nbits - base, uint64_t(s0) + uint64_t(m) * C));
    // one step from p: the next position (a code at p: counted in *n); past the stream: the
    // chunk's end e (the last chunk's exit is never used)
    auto step = [&](uint32_t p, uint32_t e, uint32_t* n) -> uint32_t {
        if (p >= lim) return e;
        const uint32_t p15 = lbits_pad(L, p, 15);
        uint32_t v = l1[p15 >> (15 - kHufL1)];
        if (!v) v = a.lut[p15];
        const uint32_t len = v >> 8;
        *n += len ? 1u : 0u;
        return p + (len ? len : 1u);
    };
    // slot u of this thread: s = u kTPB + tid, chunk s / 16, entry s % 16 (15: none)
    auto kc_of = [&](int u) { return (u * kTPB + tid) >> 4; };
    const int d = tid & 15;
    uint32_t p[U], n1[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        p[u] = s0 + uint32_t(kc_of(u)) * C + uint32_t(d);
        n1[u] = 0;
    }
    // the sync walks, the thread's U slots interleaved (independent chains: their LDS reads overlap)
    for (;;) {
        bool any = false;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int kc = kc_of(u);
            const uint32_t cs = s0 + uint32_t(kc) * C, ce = cs + C;
            if (d < kHufD && kc < m && p[u] < min(cs + kHufSync, ce)) {
                p[u] = step(p[u], ce, &n1[u]);
                any = true;
            }
        }
        if (!any) break;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int kc = kc_of(u);
        const bool act = d < kHufD && kc < m;
        p[u] = min(p[u], s0 + uint32_t(kc + 1) * C);
        P[u * kTPB + tid] = act ? p[u] : 0xFFFFFFFFu;
    }
    __syncthreads();
    // the first entry of the chunk standing on the same boundary leads; leaders still inside the
    // chunk are the survivors
    int lead[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int kc = kc_of(u), sl = u * kTPB + tid;
        const uint32_t ce = s0 + uint32_t(kc + 1) * C;
        lead[u] = d;
        if (d < kHufD && kc < m) {
            for (int j = 0; j < d; j++)
                if (P[(kc << 4) + j] == p[u]) {
                    lead[u] = j;
                    break;
                }
            if (lead[u] == d) {
                if (p[u] < ce) {
                    R[atomicAdd(&R[S], 1u)] = uint32_t(sl);
                } else {
                    X[sl] = p[u];
                    K2[sl] = 0;
                    M[sl] = p[u];
                    KM[sl] = 0;
                }
            }
        }
    }
    __syncthreads();
    const uint32_t nr = R[S];
    for (uint32_t r = tid; r < nr; r += kTPB) {
        const uint32_t t = R[r], e = s0 + ((t >> 4) + 1u) * C, mid = e - C / 2u;
        uint32_t q = P[t], n2 = 0;
        while (q < mid) q = step(q, e, &n2);  // (the sync walk ends well before the middle)
        M[t] = q;
        KM[t] = uint16_t(n2);
        while (q < e) q = step(q, e, &n2);
        X[t] = q;
        K2[t] = uint16_t(n2);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int kc = kc_of(u);
        if (d >= kHufD || kc >= m) continue;
        const uint32_t ce = s0 + uint32_t(kc + 1) * C;
        const int lt = (kc << 4) + lead[u], k = k0 + kc;
        tab[size_t(k) * kHufD + d] = uint16_t(X[lt] - ce);
        cnt[size_t(k) * kHufD + d] = uint16_t(n1[u] + K2[lt]);
        mo[size_t(k) * kHufD + d] = uint16_t(M[lt] - (ce - C));  // (from the chunk's first bit)
        mc[size_t(k) * kHufD + d] = uint16_t(n1[u] + KM[lt]);
    }
}

// The true entry of every chunk through the composed tables, its symbol count from the table pass,
// and the workgroup scan of the counts (base[k], wgsum[g]) -- no walk.
__global__ __launch_bounds__(kTPB) void huf_count_kernel(HufArgs a, const uint16_t* cnt) {
    __shared__ alignas(8) uint32_t scratch[8];
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t c = 0;
    if (k < a.nchunks) {
        const uint64_t cstart = a.start_bit + uint64_t(k) * a.chunk_bits;
        int u = k;
        for (int l = 0; l < a.levels; l++) u /= kHufG;
        uint32_t x = a.E[u];
        for (int l = a.levels - 1; l >= 0; l--) {
            int ul = k;
            for (int m = 0; m < l; m++) ul /= kHufG;
            x = a.lvl[l][size_t(ul) * kHufD + x];
        }
        a.entry[k] = cstart + x;
        c = cnt[size_t(k) * kHufD + x];
        a.count[k] = c;
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan(c, scratch, &tot);
    if (k < a.nchunks) a.base[k] = ex;
    if (threadIdx.x == 0) a.wgsum[blockIdx.x] = tot;
}

// The emitting walk: every chunk again from its entry, over the workgroup's chunks' bits staged
// in LDS (a step reads LDS, not the stream in memory: the walk is one dependent chain per lane,
// and the ~800 waves of a 4K payload are too few to hide a memory round trip per code), its
// symbols into LDS at the chunk's place in the workgroup's output, then the workgroup's output
// copied out whole (consecutive lanes, consecutive bytes) -- a lane writing its own chunk's bytes
// straight to memory touches 64 lines per store instruction.  A workgroup whose output exceeds the
// buffer writes from the walk.  A position no code prefixes flags the stream (changed[1]).
#ifndef IE_HUF_EMIT_LDS
#define IE_HUF_EMIT_LDS 40960
#endif
constexpr int kHufEmitT = 2 * kTPB;  // emit threads: two per chunk (its halves, split at the
                                     // middle boundary the table pass recorded)
__global__ __launch_bounds__(kHufEmitT) void huf_emit_kernel(HufArgs a, const uint16_t* mo, const uint16_t* mc) {
    __shared__ uint16_t l1[1 << kHufL1];
    __shared__ alignas(8) uint64_t scratch[kHufEmitT / 64];
    __shared__ uint8_t sym[IE_HUF_EMIT_LDS > 0 ? IE_HUF_EMIT_LDS : 1];
    extern __shared__ uint32_t L[];  // the workgroup's chunks' bits (+ 64 past the last)
    const int tid = threadIdx.x, j = tid % kTPB, half = tid / kTPB;
    const uint32_t C = uint32_t(a.chunk_bits);
    const int k0 = blockIdx.x * kTPB, m = min(kTPB, a.nchunks - k0);
    const uint64_t c0 = a.start_bit + uint64_t(k0) * C;
    const uint64_t base = c0 & ~31ull;
    const uint32_t s0 = uint32_t(c0 - base);
    stage_words_pad(L, a.words, base >> 5, int((s0 + uint32_t(m) * C + 64) >> 5) + 2, a.nbits, tid, kHufEmitT);
    huf_l1(a.lut, l1);  // (ends with a barrier: L staged too)
    // the symbols before this workgroup's chunks: the totals of the workgroups before it
    uint64_t part = 0;
    for (int i = tid; i < int(blockIdx.x); i += kHufEmitT) part += a.wgsum[i];
    const uint64_t ws = wave_sum64(part);
    if ((tid & 63) == 0) scratch[tid >> 6] = ws;
    __syncthreads();
    uint64_t pre = 0;
#pragma unroll
    for (int w = 0; w < kHufEmitT / 64; w++) pre += scratch[w];
    const uint32_t tot = a.wgsum[blockIdx.x];
    const bool staged = IE_HUF_EMIT_LDS > 0 && tot <= uint32_t(IE_HUF_EMIT_LDS);
    const int k = k0 + j;
    if (j < m) {
        const uint32_t lim = uint32_t(min<uint64_t>(a.nbits - base, uint64_t(s0) + uint64_t(m) * C));
        const uint32_t cs = s0 + uint32_t(j) * C, e = cs + C;
        const uint32_t x = uint32_t(a.entry[k] - (a.start_bit + uint64_t(k) * C));  // the true entry offset
        const uint32_t mid = cs + mo[size_t(k) * kHufD + x];
        uint32_t p = half ? mid : cs + x, c = 0;
        const uint32_t end = half ? e : mid;
        const uint64_t at = a.base[k] + (half ? mc[size_t(k) * kHufD + x] : 0u);
        uint8_t* o = staged ? sym + at : a.out + pre + at;
        const uint64_t room = staged ? ~0ull : (a.out_cap > pre + at ? a.out_cap - pre - at : 0ull);
        while (p < end && p < lim) {
            const uint32_t p15 = lbits_pad(L, p, 15);
            uint32_t v = l1[p15 >> (15 - kHufL1)];
            if (!v) v = a.lut[p15];
            const uint32_t len = v >> 8;
            if (!len) {
                atomicOr(&a.changed[1], 1u);
                break;
            }
            if (c >= room) {
                atomicOr(&a.changed[0], 1u);
                break;
            }
            o[c++] = uint8_t(v);
            p += len;
        }
    }
    if (!staged) return;
    __syncthreads();
    if (pre + tot > a.out_cap && tid == 0) atomicOr(&a.changed[0], 1u);
    for (uint32_t i = tid; i < tot && pre + i < a.out_cap; i += kHufEmitT) a.out[pre + i] = sym[i];
}

int huffman_decode_device(const uint32_t* W, uint64_t nbits, uint64_t start_bit, const uint16_t* lut,
                          uint64_t chunk_bits, uint64_t* entry, uint16_t* tab, uint32_t* E, unsigned* ticket,
                          uint32_t* count, uint64_t* base, unsigned* changed, uint64_t* total, uint8_t* out,
                          bool write, hipStream_t s, uint64_t out_cap) {
    const uint64_t span = nbits > start_bit ? nbits - start_bit : 0;
    const int nchunks = int((span + chunk_bits - 1) / chunk_bits);
    if (nchunks == 0) return 0;
    HufArgs a{};
    a.words = W;
    a.nbits = nbits;
    a.start_bit = start_bit;
    a.chunk_bits = chunk_bits;
    a.nchunks = nchunks;
    a.lut = lut;
    a.entry = entry;
    a.count = count;
    a.wgsum = count + nchunks;  // [ceil(nchunks / kTPB)] after the counts (huffman_count_words)
    a.changed = changed;
    a.base = base;
    a.out = out;
    a.out_cap = out_cap;
    const dim3 g((nchunks + kTPB - 1) / kTPB), blk(kTPB);
    if (write) {
        const uint16_t* cnt = tab + compose_rows<kHufD, kHufG>(nchunks) * kHufD;
        const uint16_t* mo = cnt + size_t(nchunks) * kHufD;
        hipLaunchKernelGGL(huf_emit_kernel, g, dim3(kHufEmitT), size_t(pad_words(int(((uint64_t(kTPB) * chunk_bits + 95) >> 5) + 3))) * 4, s,
                           a, mo, mo + size_t(nchunks) * kHufD);
        return 0;
    }
    const size_t lds = size_t(pad_words(int(((uint64_t(kHufTC) * chunk_bits + 95) >> 5) + 3))) * 4;
    // the symbol counts after the composition's rows (compose_kernel rewrites the exit tables)
    uint16_t* cnt = tab + compose_rows<kHufD, kHufG>(nchunks) * kHufD;
    uint16_t* mo = cnt + size_t(nchunks) * kHufD;  // then the middle boundaries and their counts
    hipLaunchKernelGGL(huf_table_kernel, dim3((nchunks + kHufTC - 1) / kHufTC), blk, lds, s, a, tab, cnt, mo,
                       mo + size_t(nchunks) * kHufD);
    const int levels = launch_compose<kHufD, kHufG>(tab, nchunks, E, ticket, a.lvl, s);
    if (levels < 0) return -1;
    a.levels = levels;
    a.E = E;
    hipLaunchKernelGGL(huf_count_kernel, g, blk, 0, s, a, cnt);
    hipLaunchKernelGGL(huf_total_kernel, dim3(1), blk, 0, s, a.wgsum, int(g.x), total);
    return levels;
}

size_t huffman_table_rows(uint64_t nbits, uint64_t start_bit, uint64_t chunk_bits) {
    const uint64_t span = nbits > start_bit ? nbits - start_bit : 0;
    const int nchunks = int((span + chunk_bits - 1) / chunk_bits);
    return nchunks ? (compose_rows<kHufD, kHufG>(nchunks) + 3 * size_t(nchunks)) * kHufD : 0;  // (+ counts, middles)
}

}  // namespace ie
