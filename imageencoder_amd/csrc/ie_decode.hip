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

#include "ie_common.hpp"
#include "ie_device.h"

namespace ie {

namespace {
constexpr int kZZ4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
constexpr int kZZ8[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                          12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                          35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                          58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
}  // namespace

struct WalkArgs {
    const uint32_t* words;  // stream as stored (big-endian bytes), zero-padded by >= 2 words
    uint64_t nbits;         // stream length in bits
    uint64_t start_bit;
    uint64_t chunk_bits;
    int nchunks;
    int nn;                 // N*N
    int rle;
    uint64_t* entry;        // [nchunks]
    const uint64_t* exit_in;
    uint64_t* exit_out;
    uint32_t* count;
    unsigned* changed;
    int first;              // speculative first pass
};

// bits [p, p+l) of the stream, l <= 32
__device__ __forceinline__ uint32_t getbits(const uint32_t* W, uint64_t p, int l) {
    if (l == 0) return 0;
    const uint64_t w = p >> 5;
    const uint64_t v = (uint64_t(bswap32(W[w])) << 32) | bswap32(W[w + 1]);
    return uint32_t((v << (p & 31)) >> (64 - l));
}

__device__ __forceinline__ void walk(const WalkArgs& a, uint64_t pos, uint64_t end, uint64_t* exit_pos,
                                     uint32_t* cnt, uint64_t* out_idx_base, uint64_t* block_bit, uint64_t nblocks) {
    uint32_t c = 0;
    while (pos < end && pos < a.nbits) {
        const uint32_t head = getbits(a.words, pos, 20);
        const int bl = int(head >> 16);
        int lw;
        bool ok;
        if (a.rle) {
            lw = bl ? int((head << 16 >> 16) >> (16 - bl)) : 0;
            ok = bl >= 1 && lw <= a.nn;
        } else {
            lw = a.nn;
            ok = bl >= 1;
        }
        if (!ok) {  // cannot be a record start: slide (never happens on the true path)
            pos += 1;
            continue;
        }
        if (block_bit) {
            const uint64_t idx = *out_idx_base + c;
            if (idx < nblocks) block_bit[idx] = pos;
        }
        c++;
        pos += 4 + uint64_t(bl) * uint64_t(lw + a.rle);
    }
    *exit_pos = pos;
    *cnt = c;
}

__global__ void walk_kernel(WalkArgs a) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.nchunks) return;
    const uint64_t cstart = a.start_bit + uint64_t(k) * a.chunk_bits;
    const uint64_t cend = cstart + a.chunk_bits;
    uint64_t e;
    if (a.first) {
        e = cstart;
    } else {
        if (k == 0) {
            a.exit_out[0] = a.exit_in[0];
            return;
        }
        e = a.exit_in[k - 1];
        if (e == a.entry[k]) {
            a.exit_out[k] = a.exit_in[k];
            return;
        }
        atomicOr(a.changed, 1u);
    }
    a.entry[k] = e;
    uint64_t x;
    uint32_t c;
    uint64_t dummy = 0;
    walk(a, e, cend, &x, &c, &dummy, nullptr, 0);
    a.exit_out[k] = x;
    a.count[k] = c;
}

__global__ void index_kernel(WalkArgs a, const uint64_t* base, uint64_t* block_bit, uint64_t nblocks) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.nchunks) return;
    const uint64_t cstart = a.start_bit + uint64_t(k) * a.chunk_bits;
    uint64_t x, b = base[k];
    uint32_t c;
    walk(a, a.entry[k], cstart + a.chunk_bits, &x, &c, &b, block_bit, nblocks);
}

// exclusive scan of per-chunk counts: one workgroup, each thread owns kScanRun consecutive counts
// (one block scan per kTPB * kScanRun counts instead of one per kTPB)
constexpr int kScanRun = 32;
__global__ __launch_bounds__(kTPB) void scan_counts_kernel(const uint32_t* count, uint64_t* base, int n) {
    __shared__ uint32_t scratch[8];
    uint64_t carry = 0;  // the same in every thread
    for (int s = 0; s < n; s += kTPB * kScanRun) {
        const int i0 = s + int(threadIdx.x) * kScanRun;
        uint32_t v[kScanRun];
        uint32_t sum = 0;
#pragma unroll
        for (int j = 0; j < kScanRun; j++) {
            v[j] = (i0 + j < n) ? count[i0 + j] : 0u;
            sum += v[j];
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan(sum, scratch, &tot);
        uint64_t run = carry + ex;
#pragma unroll
        for (int j = 0; j < kScanRun; j++) {
            if (i0 + j < n) base[i0 + j] = run;
            run += v[j];
        }
        carry += tot;
        __syncthreads();  // scratch is reused by the next strip's scan
    }
}

// Inverse of one block: parse, dequantise, IDCT in the reference order, clamp/truncate.
template <int N>
__global__ __launch_bounds__(kTPB) void decode_kernel(DecArgs a, const uint32_t* W, uint64_t* end_out) {
    constexpr int NN = N * N;
    const uint64_t nblocks = uint64_t(a.nframes) * a.bx * a.by;
    const uint64_t b = uint64_t(blockIdx.x) * kTPB + threadIdx.x;
    if (b >= nblocks) return;
    const EncTables* __restrict__ tab = a.tab;
    uint64_t pos = a.block_bit[b];
    const int bl = int(getbits(W, pos, 4));
    pos += 4;
    int length = NN;
    if (a.rle) {
        length = int(getbits(W, pos, bl));
        pos += bl;
    }
    if (length > NN) length = NN;  // cannot happen for a well-formed stream
    double Y[NN];
#pragma unroll
    for (int k = 0; k < NN; k++) Y[k] = 0.0;
    const int* zz = (N == 4) ? kZZ4 : kZZ8;
    for (int k = 0; k < length; k++) {
        const uint32_t raw = getbits(W, pos, bl);
        pos += bl;
        const int sh = 16 - bl;
        const int16_t v = int16_t(int16_t(uint16_t(raw << sh)) >> sh);
        Y[zz[k]] = double(v);
    }
    if (b == nblocks - 1 && end_out) *end_out = pos;
    // Block::processIDCTMulQ: Y *= q, then temp[ij] += R[uv][ij] * Y[uv] over uv ascending.
    // Zero Y terms add +-0 and leave every partial sum unchanged, so they are skipped.
    double t[NN];
#pragma unroll
    for (int k = 0; k < NN; k++) t[k] = 0.0;
#pragma unroll
    for (int uv = 0; uv < NN; uv++) {
        const double y = Y[uv] * tab->qd[uv];
        if (y != 0.0) {
            const double* R = &tab->R[uv * NN];
#pragma unroll
            for (int ij = 0; ij < NN; ij++) t[ij] = t[ij] + R[ij] * y;
        }
    }
    const uint64_t bpf = uint64_t(a.bx) * a.by;
    const uint64_t f = b / bpf, r = b - f * bpf;
    const int byi = int(r / a.bx), bxi = int(r - uint64_t(byi) * a.bx);
    uint8_t* o = a.out + f * a.frame_pitch + uint64_t(byi) * N * a.stride + uint64_t(bxi) * N;
#pragma unroll
    for (int i = 0; i < N; i++) {
#pragma unroll
        for (int j = 0; j < N; j++) {
            double x = t[i * N + j] + 128.0;
            x = x < 0.0 ? 0.0 : (x > 255.0 ? 255.0 : x);
            o[uint64_t(i) * a.stride + j] = uint8_t(x);
        }
    }
}

// ---- Huffman decode (Huffman.cpp:354-402; the per-bit tree walk of :190-204) -------------------
// Same chunked speculation as the record walk: one lane per chunk of bits decodes symbols with a
// prefix table until it leaves the chunk; fix-up rounds re-walk chunks whose entry differs from the
// predecessor's exit (prefix codes resynchronise within a few symbols); a scan of the per-chunk
// symbol counts places every chunk's output; a last walk writes the symbols.  The reference walks
// to the end of the buffer, padding bits of the last byte included (a code may run past it with
// zero bits), and so does this walk.
//   lut   [2^15]: sym | len << 8 for every 15-bit prefix, len 0 = no code (codes are <= 15 bits:
//         the dictionary stores lengths in 4 bits, Huffman.cpp:41-42)
//   LDS   the 2^kHufL1 first-level entries (codes of <= kHufL1 bits resolve there)
constexpr int kHufL1 = 11;
struct HufArgs {
    const uint32_t* words;
    uint64_t nbits, start_bit, chunk_bits;
    int nchunks;
    const uint16_t* lut;
    uint64_t* entry;
    const uint64_t* exit_in;
    uint64_t* exit_out;
    uint32_t* count;
    unsigned* changed;  // [0] a round changed an entry, [1] invalid code on the exact walk
    int first;
    const uint64_t* base;
    uint8_t* out;
};

__device__ __forceinline__ void huf_l1(const uint16_t* lut, uint16_t* l1) {
    for (int q = threadIdx.x; q < (1 << kHufL1); q += blockDim.x) {
        const uint16_t e = lut[uint32_t(q) << (15 - kHufL1)];
        l1[q] = ((e >> 8) != 0 && (e >> 8) <= kHufL1) ? e : uint16_t(0);  // 0: look in lut
    }
    __syncthreads();
}

// Walk [pos, end): returns the exit position; *cnt symbols; out (optional) receives them.
__device__ __forceinline__ uint64_t huf_walk(const HufArgs& a, const uint16_t* l1, uint64_t pos, uint64_t end,
                                             uint32_t* cnt, uint8_t* out, bool exact) {
    uint32_t c = 0;
    while (pos < end && pos < a.nbits) {
        const uint32_t p15 = getbits(a.words, pos, 15);
        uint32_t e = l1[p15 >> (15 - kHufL1)];
        if (!e) e = a.lut[p15];
        const uint32_t len = e >> 8;
        if (!len) {  // no code starts here: a speculative walk slides; the exact walk reports
            if (exact) {
                atomicOr(&a.changed[1], 1u);
                break;
            }
            pos += 1;
            continue;
        }
        if (out) out[c] = uint8_t(e);
        c++;
        pos += len;
    }
    *cnt = c;
    return pos;
}

__global__ __launch_bounds__(kTPB) void huf_walk_kernel(HufArgs a) {
    __shared__ uint16_t l1[1 << kHufL1];
    huf_l1(a.lut, l1);
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.nchunks) return;
    const uint64_t cstart = a.start_bit + uint64_t(k) * a.chunk_bits;
    uint64_t e;
    if (a.first) {
        e = cstart;
    } else {
        if (k == 0) {
            a.exit_out[0] = a.exit_in[0];
            return;
        }
        e = a.exit_in[k - 1];
        if (e == a.entry[k]) {
            a.exit_out[k] = a.exit_in[k];
            return;
        }
        atomicOr(a.changed, 1u);
    }
    a.entry[k] = e;
    uint32_t c;
    a.exit_out[k] = huf_walk(a, l1, e, cstart + a.chunk_bits, &c, nullptr, false);
    a.count[k] = c;
}

__global__ __launch_bounds__(kTPB) void huf_emit_kernel(HufArgs a) {
    __shared__ uint16_t l1[1 << kHufL1];
    huf_l1(a.lut, l1);
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.nchunks) return;
    const uint64_t cstart = a.start_bit + uint64_t(k) * a.chunk_bits;
    uint32_t c;
    huf_walk(a, l1, a.entry[k], cstart + a.chunk_bits, &c, a.out + a.base[k], true);
}

// Returns the number of fix-up rounds (>= 0), -1 on a HIP error, -2 if the rounds did not settle.
// total receives the symbol count (device, 1 word) = base[last] + count[last].
__global__ void huf_total_kernel(const uint64_t* base, const uint32_t* count, int n, uint64_t* total) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *total = base[n - 1] + count[n - 1];
}

int huffman_decode_device(const uint32_t* W, uint64_t nbits, uint64_t start_bit, const uint16_t* lut,
                          uint64_t chunk_bits, uint64_t* entry, uint64_t* exA, uint64_t* exB, uint32_t* count,
                          uint64_t* base, unsigned* changed, uint64_t* total, uint8_t* out, bool write,
                          hipStream_t s, int max_rounds) {
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
    a.changed = changed;
    a.base = base;
    a.out = out;
    const dim3 g((nchunks + kTPB - 1) / kTPB), blk(kTPB);
    if (!write) {
        a.first = 1;
        a.exit_in = exA;
        a.exit_out = exA;
        hipLaunchKernelGGL(huf_walk_kernel, g, blk, 0, s, a);
        uint64_t* cur = exA;
        uint64_t* nxt = exB;
        // fix-up rounds in growing groups (1, 2, 4, 8, 8, ...) between host checks of the
        // "changed" flag (a round after convergence is a near-empty launch; a host round trip per
        // round costs more)
        int rounds = 0, group = 1;
        bool done = false;
        while (!done && rounds < max_rounds + 8) {
            unsigned h = 0;
            if (hipMemsetAsync(changed, 0, sizeof(unsigned), s) != hipSuccess) return -1;
            for (int r = 0; r < group; r++) {
                a.first = 0;
                a.exit_in = cur;
                a.exit_out = nxt;
                hipLaunchKernelGGL(huf_walk_kernel, g, blk, 0, s, a);
                uint64_t* t = cur;
                cur = nxt;
                nxt = t;
            }
            rounds += group;
            group = group < 8 ? 2 * group : 8;
            if (hipMemcpyAsync(&h, changed, sizeof(unsigned), hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
            if (hipStreamSynchronize(s) != hipSuccess) return -1;
            done = (h == 0);
        }
        if (!done) return -2;
        hipLaunchKernelGGL(scan_counts_kernel, dim3(1), blk, 0, s, count, base, nchunks);
        hipLaunchKernelGGL(huf_total_kernel, dim3(1), dim3(1), 0, s, base, count, nchunks, total);
        return rounds;
    }
    hipLaunchKernelGGL(huf_emit_kernel, g, blk, 0, s, a);
    return 0;
}

// ---- fused record parse + decode (one launch) ---------------------------------------------------
// The stream is cut into SEGMENTS of kDecTPB * C bits, one workgroup each, staged in LDS with
// coalesced loads (plus a margin covering the longest record).  Inside a segment every lane walks
// C bits from a speculative entry, from LDS; local fix-up rounds (entry := the left neighbour's
// exit) make the segment's path consistent from its first bit; that path's record starts are
// marked in an LDS bitmap.  A record stream resynchronises within a few records, so the path
// from the segment's TRUE entry (the predecessor's exit) merges with the marked path after a few
// records and the segment's exit does not depend on its entry: every segment publishes its exit
// at once, and its successor walks from it only up to the merge.  The true record count then
// feeds a decoupled look-back (ie_common.hpp) for the global block index, and the lanes decode
// their records straight from LDS: dequantise (Block.cpp:163-169), FP64 IDCT in the reference's
// order (algo.cpp:343-363), +128, clamp, truncate (Block.cpp:100-107).  Should a walk from the
// true entry not merge inside its segment (or a spin time out), the launch reports it in err[1]
// and the host re-runs the multi-kernel path above.
constexpr int kDecTPB = 256;
template <int N> struct DecSeg {
    static constexpr int C = (N == 4) ? 256 : 512;    // bits per lane
    static constexpr int S = kDecTPB * C;              // bits per segment
    static constexpr int MARGIN = 1024 + 64;           // > longest record (4 + 15 * 65) + 64-bit reads
    static constexpr int WORDS = (S + MARGIN) / 32 + 2;
    static constexpr int MAXPRE = 64;                  // records walked from the true entry before merging
};

struct FusedArgs {
    const uint32_t* words;  // stream as stored (big-endian bytes), zero-padded
    uint64_t nbits, start_bit;
    int nseg;
    int rle;
    uint64_t* st;           // chain state (kGran words per segment): 0 count aggregate, 1 inclusive, 3 exit
    uint32_t tag;
    unsigned* err;          // [0] spin timeouts, [1] fallback needed (no merge / malformed)
    uint64_t* end_out;      // end bit of the last block's record
    DecArgs d;
};

// bits [p, p+l) of the LDS stream copy L (MSB-first words), l <= 32, p relative to the copy
__device__ __forceinline__ uint32_t lbits(const uint32_t* L, uint32_t p, int l) {
    const uint32_t w = p >> 5, s = p & 31u;
    const uint64_t v = (uint64_t(L[w]) << 32) | L[w + 1];
    return l ? uint32_t((v << s) >> (64 - l)) : 0u;
}

// length of the record whose header is at p, 0 if no record can start there
template <int N>
__device__ __forceinline__ uint32_t rec_len(const uint32_t* L, uint32_t p, int rle) {
    constexpr int NN = N * N;
    const uint32_t head = lbits(L, p, 20);
    const uint32_t bl = head >> 16;
    if (!bl) return 0;
    if (!rle) return 4u + bl * NN;
    const uint32_t lw = (head & 0xFFFFu) >> (16 - bl);
    return lw <= uint32_t(NN) ? 4u + bl * (lw + 1u) : 0u;
}

// speculative walk of [e, end): exit position and record count (invalid headers slide one bit)
template <int N>
__device__ __forceinline__ uint32_t spec_walk(const uint32_t* L, uint32_t e, uint32_t end, uint32_t lim, int rle,
                                              uint32_t* cnt, uint32_t* bitmap) {
    uint32_t c = 0;
    while (e < end && e < lim) {
        const uint32_t len = rec_len<N>(L, e, rle);
        if (!len) {
            e++;
            continue;
        }
        if (bitmap) atomicOr(&bitmap[e >> 5], 1u << (e & 31u));
        c++;
        e += len;
    }
    *cnt = c;
    return e;
}

// decode the record at p (relative to L) as block g; returns the bit after it
template <int N>
__device__ __forceinline__ uint32_t decode_record(const uint32_t* L, uint32_t p, uint64_t g, const DecArgs& a) {
    constexpr int NN = N * N;
    const EncTables* __restrict__ tab = a.tab;
    const int bl = int(lbits(L, p, 4));
    p += 4;
    int length = NN;
    if (a.rle) {
        length = int(lbits(L, p, bl));
        p += bl;
    }
    if (length > NN) length = NN;
    double Y[NN];
#pragma unroll
    for (int k = 0; k < NN; k++) Y[k] = 0.0;
    const int* zz = (N == 4) ? kZZ4 : kZZ8;
    for (int k = 0; k < length; k++) {
        const uint32_t raw = lbits(L, p, bl);
        p += bl;
        const int sh = 16 - bl;
        Y[zz[k]] = double(int16_t(int16_t(uint16_t(raw << sh)) >> sh));
    }
    double t[NN];
#pragma unroll
    for (int k = 0; k < NN; k++) t[k] = 0.0;
#pragma unroll
    for (int uv = 0; uv < NN; uv++) {
        const double y = Y[uv] * tab->qd[uv];
        if (y != 0.0) {
            const double* R = &tab->R[uv * NN];
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
    return p;
}

template <int N>
__global__ __launch_bounds__(kDecTPB) void parse_decode_kernel(FusedArgs a) {
    using G = DecSeg<N>;
    __shared__ uint32_t L[G::WORDS];
    __shared__ uint32_t mark[G::S / 32 + 1];
    __shared__ uint32_t X[kDecTPB];
    __shared__ uint32_t pre[G::MAXPRE];
    __shared__ uint32_t misc[24];  // [0..3] scan scratch, [4] any, [5] merge, [6] c_pre, [8..9] excl, [10] fail
    const int tid = threadIdx.x, k = blockIdx.x;
    const uint64_t seg0 = a.start_bit + uint64_t(k) * G::S;  // the segment's first bit
    const uint64_t base = seg0 & ~31ull;                       // bit 0 of L
    const uint32_t s0 = uint32_t(seg0 - base);                 // segment start, relative
    const uint32_t s1 = s0 + G::S;                             // segment end (exclusive), relative
    const uint32_t lim = uint32_t(min<uint64_t>(a.nbits - base, uint64_t(G::WORDS - 2) * 32));  // readable bits
    // 1. stage the segment's bits (MSB-first words), zeros past the stream
    const uint64_t w0 = base >> 5, nw = (a.nbits + 31) >> 5;
    for (int i = tid; i < G::WORDS; i += kDecTPB)
        L[i] = (w0 + i < nw) ? bswap32(__builtin_nontemporal_load(a.words + w0 + i)) : 0u;
    for (int i = tid; i < G::S / 32 + 1; i += kDecTPB) mark[i] = 0u;
    __syncthreads();
    // 2. speculative lane walks, then local rounds until every lane continues its neighbour's path
    const uint32_t lane_end = s0 + uint32_t(tid + 1) * G::C;
    uint32_t entry = s0 + uint32_t(tid) * G::C, cnt;
    uint32_t ex = spec_walk<N>(L, entry, lane_end, lim, a.rle, &cnt, nullptr);
    for (int round = 0; round <= kDecTPB; round++) {
        X[tid] = ex;
        __syncthreads();
        const uint32_t ne = tid ? X[tid - 1] : s0;
        const bool ch = ne != entry;
        if (ch) {
            entry = ne;
            ex = spec_walk<N>(L, entry, lane_end, lim, a.rle, &cnt, nullptr);
        }
        if (!__syncthreads_or(ch)) break;
    }
    // 3. mark the segment's path; its exit is published at once (entry-independent, see above)
    spec_walk<N>(L, entry, lane_end, lim, a.rle, &cnt, mark);
    __syncthreads();  // marks visible
    if (tid == kDecTPB - 1) st_state(&a.st[kGran * k + 3], (uint64_t(a.tag) << 56) | ((base + ex) & kMask56));
    // 4. the true entry (predecessor's exit) and the walk from it to the merge with the marked path
    if (tid == 0) {
        uint64_t e = a.start_bit;
        bool ok = true;
        if (k > 0) {
            unsigned sp = 0;
            for (;;) {
                const uint64_t g = ld_state(&a.st[kGran * (k - 1) + 3]);
                if (uint32_t(g >> 56) == a.tag) {
                    e = g & kMask56;
                    break;
                }
                if (++sp > kSpinLimit) {
                    atomicAdd(&a.err[0], 1u);
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        uint32_t p = uint32_t(e - base), c = 0;
        // walk until a marked record start (the merge), the segment's end or the stream's end
        while (ok && p < s1 && p < lim && !((mark[p >> 5] >> (p & 31u)) & 1u)) {
            const uint32_t len = rec_len<N>(L, p, a.rle);
            if (!len || c == G::MAXPRE) {  // malformed, or no merge within reach: fall back
                ok = false;
                break;
            }
            pre[c++] = p;
            p += len;
        }
        // no merge inside the segment: its true exit must be the published one, else fall back
        if (ok && p >= s1 && k != a.nseg - 1 && p != X[kDecTPB - 1]) ok = false;
        misc[10] = ok ? 0u : 1u;
        misc[5] = p;
        misc[6] = c;
    }
    __syncthreads();
    // (a fallback still publishes a count below, so successors' look-backs terminate; the host
    // discards this launch's output)
    if (misc[10] && tid == 0) atomicOr(&a.err[1], 1u);
    const uint32_t m = misc[5], c_pre = misc[6];
    // 5. true count = records before the merge + marked records from the merge on
    uint32_t mine = 0;  // this lane's path records at or after m (the true records among them)
    for (uint32_t e2 = entry; e2 < lane_end && e2 < lim;) {
        const uint32_t len = rec_len<N>(L, e2, a.rle);
        if (!len) {
            e2++;
            continue;
        }
        mine += (e2 >= m) ? 1u : 0u;
        e2 += len;
    }
    uint32_t tot2;
    const uint32_t off = block_excl_scan<kDecTPB>(mine, misc, &tot2);
    const uint32_t A = c_pre + tot2;
    // 6. global index of the segment's first block: decoupled look-back over the counts
    if (tid == 0) chain_publish_count(a.st, k, k, a.tag, A);
    if (tid < 64 && k > 0) {
        const Probe pr = probe_issue(a.st, k, k, 1, 0, kProbe0);
        const uint64_t excl = lookback_wave(pr, a.st, k, k, 1, a.tag, a.err);
        if (tid == 0) {
            publish(a.st, k, 1, a.tag, excl + A);
            misc[8] = uint32_t(excl);
            misc[9] = uint32_t(excl >> 32);
        }
    } else if (tid == 0) {
        misc[8] = 0u;
        misc[9] = 0u;
    }
    __syncthreads();
    const uint64_t excl = uint64_t(misc[8]) | (uint64_t(misc[9]) << 32);
    // 7. decode: the pre-merge records (thread 0), then every lane's records from the merge on
    const uint64_t nblocks = uint64_t(a.d.nframes) * a.d.bx * a.d.by;
    if (tid == 0) {
        for (uint32_t i = 0; i < c_pre; i++) {
            const uint64_t g = excl + i;
            if (g < nblocks) {
                const uint32_t q = decode_record<N>(L, pre[i], g, a.d);
                if (g == nblocks - 1) *a.end_out = base + q;
            }
        }
    }
    uint64_t g = excl + c_pre + off;
    uint32_t e3 = entry;
    while (e3 < lane_end && e3 < lim && g < nblocks) {
        const uint32_t len = rec_len<N>(L, e3, a.rle);
        if (!len) {
            e3++;
            continue;
        }
        if (e3 >= m) {
            const uint32_t q = decode_record<N>(L, e3, g, a.d);
            if (g == nblocks - 1) *a.end_out = base + q;
            g++;
        }
        e3 += len;
    }
}

uint64_t parse_decode_segment_bits(int n) { return (n == 4) ? DecSeg<4>::S : DecSeg<8>::S; }

// One launch: returns the number of segments (the host checks err[1] afterwards).
int launch_parse_decode(const uint32_t* W, uint64_t nbits, uint64_t start_bit, const DecArgs& d, int n,
                        uint64_t* st, uint32_t tag, unsigned* err, uint64_t* end_out, hipStream_t s) {
    const uint64_t S = (n == 4) ? DecSeg<4>::S : DecSeg<8>::S;
    const uint64_t span = nbits > start_bit ? nbits - start_bit : 0;
    const int nseg = int((span + S - 1) / S);
    if (nseg == 0) return 0;
    FusedArgs a{};
    a.words = W;
    a.nbits = nbits;
    a.start_bit = start_bit;
    a.nseg = nseg;
    a.rle = d.rle;
    a.st = st;
    a.tag = tag;
    a.err = err;
    a.end_out = end_out;
    a.d = d;
    if (n == 4) hipLaunchKernelGGL((parse_decode_kernel<4>), dim3(nseg), dim3(kDecTPB), 0, s, a);
    else hipLaunchKernelGGL((parse_decode_kernel<8>), dim3(nseg), dim3(kDecTPB), 0, s, a);
    return nseg;
}

// Host-driven decode sequence (ie_capi.cpp::decode calls this).
int decode_frames_device(const uint32_t* W, uint64_t nbits, uint64_t start_bit, const DecArgs& da, int n,
                         uint64_t chunk_bits, uint64_t* entry, uint64_t* exA, uint64_t* exB, uint32_t* count,
                         uint64_t* base, uint64_t* block_bit, unsigned* changed, uint64_t* end_out, hipStream_t s,
                         int max_rounds) {
    const uint64_t span = nbits > start_bit ? nbits - start_bit : 0;
    const int nchunks = int(span / chunk_bits + 1);
    WalkArgs wa{};
    wa.words = W;
    wa.nbits = nbits;
    wa.start_bit = start_bit;
    wa.chunk_bits = chunk_bits;
    wa.nchunks = nchunks;
    wa.nn = n * n;
    wa.rle = da.rle;
    wa.entry = entry;
    wa.count = count;
    wa.changed = changed;
    const dim3 g((nchunks + kTPB - 1) / kTPB), blk(kTPB);
    wa.first = 1;
    wa.exit_in = exA;
    wa.exit_out = exA;
    hipLaunchKernelGGL(walk_kernel, g, blk, 0, s, wa);
    uint64_t* cur = exA;
    uint64_t* nxt = exB;
    // fix-up rounds in growing groups (1, 2, 4, 8, 8, ...) between host checks: most 4x4 streams
    // settle after one round, 8x8 ones take ~20; a round after convergence is a near-empty launch
    // (~15 us), a host round trip per round costs more
    int rounds = 0, group = 1;
    bool done = false;
    // (convergence takes at most max_rounds rounds; a group after it confirms it)
    while (!done && rounds < max_rounds + 8) {
        unsigned h = 0;
        if (hipMemsetAsync(changed, 0, sizeof(unsigned), s) != hipSuccess) return -1;
        for (int r = 0; r < group; r++) {
            wa.first = 0;
            wa.exit_in = cur;
            wa.exit_out = nxt;
            hipLaunchKernelGGL(walk_kernel, g, blk, 0, s, wa);
            uint64_t* t = cur;
            cur = nxt;
            nxt = t;
        }
        rounds += group;
        group = group < 8 ? 2 * group : 8;
        if (hipMemcpyAsync(&h, changed, sizeof(unsigned), hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
        if (hipStreamSynchronize(s) != hipSuccess) return -1;
        done = (h == 0);
    }
    if (!done) return -2;
    hipLaunchKernelGGL(scan_counts_kernel, dim3(1), blk, 0, s, count, base, nchunks);
    hipLaunchKernelGGL(index_kernel, g, blk, 0, s, wa, base, block_bit, uint64_t(da.nframes) * da.bx * da.by);
    DecArgs d = da;
    d.block_bit = block_bit;
    const uint64_t nblocks = uint64_t(da.nframes) * da.bx * da.by;
    const dim3 gd(unsigned((nblocks + kTPB - 1) / kTPB));
    if (n == 4) hipLaunchKernelGGL((decode_kernel<4>), gd, blk, 0, s, d, W, end_out);
    else hipLaunchKernelGGL((decode_kernel<8>), gd, blk, 0, s, d, W, end_out);
    return rounds;
}

}  // namespace ie
