// imageencoder_amd/csrc/ie_huffman.hip -- device side of the Huffman post-pass (config 5).
//
// algo::Huffman<uint8_t>::encode (Huffman.cpp:233-344) is split three ways:
//   hist_kernel   byte histogram + first occurrence of every value (the insertion order of the
//                 reference's std::unordered_map, Huffman.cpp:237-243);
//   (host)        tree / dictionary build, replayed with the reference's own libstdc++
//                 containers (imageencoder_amd/csrc/host/Huffman.cpp);
//   pack_kernel   re-encode every byte with its code, MSB-first (Huffman.cpp:314-319): the same
//                 tile scan + LDS image + decoupled look-back + funnel store as the block encoder.
// bitshift_kernel: the shifted byte copy (ie_bitcopy: the "no gain" path '0' + input,
// Huffman.cpp:329-341, and the multi-GPU segment re-shift) -- every output word's source bits are
// known from its index, so it needs no scan and no look-back: it can run beside any other kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "ie_common.hpp"
#include "ie_device.h"

namespace ie {

#ifndef IE_PACK_WAVES  // pack_kernel's minimum waves per SIMD (launch bound; 1: the compiler's choice)
#define IE_PACK_WAVES 1
#endif

constexpr int kHistTile = kTPB * 16;  // bytes per workgroup pass
constexpr int kHistLoads = 4;          // hist_body: 16-byte loads per thread in flight

// Byte histogram of [0, n) of `in`, grid-strided over workgroups blockIdx.x of gridDim.x: one
// non-returning LDS add per byte into the wave's own sub-histogram, merged with global atomics.
// The first occurrences (the reference's unordered_map insertion order) come from first_scan /
// first_full below, which only touch the bytes up to each value's first appearance.
__device__ __forceinline__ void hist_body(const uint8_t* __restrict__ in, uint64_t n, uint32_t* hist) {
    __shared__ uint32_t h[4][256];
    const int tid = threadIdx.x, wv = tid >> 6;
#pragma unroll
    for (int q = 0; q < 4; q++) h[q][tid] = 0;
    __syncthreads();
    const bool al = (reinterpret_cast<uintptr_t>(in) & 15) == 0;
    // kHistLoads 16-byte loads per thread in flight per step (a workgroup step covers
    // kHistLoads * kHistTile bytes; load q of thread tid at q * kHistTile + 16 * tid: coalesced)
    constexpr uint64_t kStep = uint64_t(kHistLoads) * kHistTile;
    for (uint64_t base = uint64_t(blockIdx.x) * kStep; base < n; base += uint64_t(gridDim.x) * kStep) {
        if (base + kStep <= n && al) {
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            v4u v[kHistLoads];
#pragma unroll
            for (int q = 0; q < kHistLoads; q++)
                v[q] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(in + base + q * kHistTile) + tid);
#pragma unroll
            for (int q = 0; q < kHistLoads; q++) {
                const uint32_t w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
                for (int e = 0; e < 16; e++) atomicAdd(&h[wv][(w[e >> 2] >> (8 * (e & 3))) & 0xFFu], 1u);
            }
        } else {
            for (int q = 0; q < kHistLoads; q++) {
                const uint64_t p = base + uint64_t(q) * kHistTile + uint64_t(tid) * 16;
                if (p + 16 <= n && al) {
                    const uint4 v = *reinterpret_cast<const uint4*>(in + p);
                    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int e = 0; e < 16; e++) atomicAdd(&h[wv][(w[e >> 2] >> (8 * (e & 3))) & 0xFFu], 1u);
                } else {
                    for (int e = 0; e < 16; e++)
                        if (p + e < n) atomicAdd(&h[wv][in[p + e]], 1u);
                }
            }
        }
    }
    __syncthreads();
    const uint32_t c = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
    if (c) atomicAdd(&hist[tid], c);
}

// First occurrence of every byte value that occurs (hist > 0), scanning from the start of the
// string in kHistTile chunks and stopping as soon as all of them are found: for encoder output
// (every value appears within a few KiB) one or two chunks.  At most kFirstScanChunks chunks;
// values still missing after that are left to first_full (unresolved[k] = 1).
constexpr int kFirstScanChunks = 64;
#ifndef IE_FIRST_Q
#define IE_FIRST_Q 4
#endif
constexpr int kFirstScanQ = IE_FIRST_Q;  // chunks per round of first_scan
// (hv: this thread's value's count; returns its first position, *unres = 1 if the scan stopped short)
__device__ __forceinline__ unsigned long long first_scan_core(const uint8_t* __restrict__ in, uint64_t n, uint32_t hv,
                                                              unsigned* unres) {
    __shared__ unsigned long long f[256];
    const int tid = threadIdx.x;
    f[tid] = ~0ull;
    const int need = __syncthreads_count(hv != 0u);
    int have = 0;
    // kFirstScanQ chunks per round, one 16-byte load each per thread, all in flight together (a
    // round per chunk made the scan a chain of load round trips)
    constexpr int Q = kFirstScanQ;
    static_assert(kFirstScanChunks % Q == 0, "whole rounds");
    const bool al = (reinterpret_cast<uintptr_t>(in) & 15) == 0;
    for (int ch = 0; ch < kFirstScanChunks && have < need; ch += Q) {
        uint4 v[Q];
#pragma unroll
        for (int q = 0; q < Q; q++) {
            const uint64_t p = uint64_t(ch + q) * kHistTile + uint64_t(tid) * 16;
            if (al && p + 16 <= n) {
                v[q] = *reinterpret_cast<const uint4*>(in + p);
            } else {
                uint32_t w[4] = {0u, 0u, 0u, 0u};
                for (int e = 0; e < 16; e++)
                    if (p + e < n) w[e >> 2] |= uint32_t(in[p + e]) << (8 * (e & 3));
                v[q] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
#pragma unroll
        for (int q = 0; q < Q; q++) {
            const uint64_t p = uint64_t(ch + q) * kHistTile + uint64_t(tid) * 16;
            const uint32_t w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
            for (int e = 0; e < 16; e++)
                if (p + e < n) {
                    const uint32_t b = (w[e >> 2] >> (8 * (e & 3))) & 0xFFu;
                    // (> and not "unset": another thread of this round may have set a later position)
                    if (f[b] > p + e) atomicMin(&f[b], (unsigned long long)(p + e));
                }
        }
        have = __syncthreads_count(f[tid] != ~0ull);
        if (uint64_t(ch + Q) * kHistTile >= n) break;
    }
    *unres = (have < need) ? 1u : 0u;
    return f[tid];
}
__device__ __forceinline__ void first_scan_body(const uint8_t* __restrict__ in, uint64_t n, const uint32_t* hist,
                                                unsigned long long* first, unsigned* unresolved) {
    unsigned u;
    first[threadIdx.x] = first_scan_core(in, n, hist[threadIdx.x], &u);
    if (threadIdx.x == 0) *unresolved = u;
}

// The values first_scan did not find: every byte of the string (past the scanned prefix) checks a
// per-value "missing" flag; atomicMin where set.  Workgroups of resolved strings exit at once.
__device__ __forceinline__ void first_full_body(const uint8_t* __restrict__ in, uint64_t n, const uint32_t* hist,
                                                unsigned long long* first, const unsigned* unresolved) {
    if (*unresolved == 0u) return;
    __shared__ unsigned long long f[256];
    __shared__ uint8_t miss[256];
    const int tid = threadIdx.x;
    const uint64_t from = uint64_t(kFirstScanChunks) * kHistTile;
    f[tid] = ~0ull;
    // Missing = not within the scanned prefix [0, from): the scan's positions are final, and this
    // pass writes only positions >= from.  (Round 5 tested first == ~0: a workgroup of a later
    // range that finished first had already lowered first[v], so a workgroup of an earlier range
    // starting after it skipped v and the later position stood -- intermittently wrong
    // dictionaries in the counted pipeline's late-values case.)
    miss[tid] = (hist[tid] != 0u && first[tid] >= from) ? 1 : 0;
    __syncthreads();
    for (uint64_t base = from + uint64_t(blockIdx.x) * kHistTile; base < n; base += uint64_t(gridDim.x) * kHistTile) {
        const uint64_t p = base + uint64_t(tid) * 16;
        for (int e = 0; e < 16; e++)
            if (p + e < n) {
                const uint32_t b = in[p + e];
                if (miss[b] && f[b] > p + e) atomicMin(&f[b], (unsigned long long)(p + e));
            }
    }
    __syncthreads();
    if (miss[tid] && f[tid] != ~0ull) atomicMin(&first[tid], f[tid]);
}

__global__ __launch_bounds__(kTPB) void hist_kernel(const uint8_t* __restrict__ in, uint64_t n, uint32_t* hist) {
    hist_body(in, n, hist);
}
__global__ __launch_bounds__(kTPB) void first_scan_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                          const uint32_t* hist, unsigned long long* first,
                                                          unsigned* unresolved) {
    first_scan_body(in, n, hist, first, unresolved);
}
__global__ __launch_bounds__(kTPB) void first_full_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                          const uint32_t* hist, unsigned long long* first,
                                                          const unsigned* unresolved) {
    first_full_body(in, n, hist, first, unresolved);
}

// string blockIdx.y of a batch
__global__ __launch_bounds__(kTPB) void hist_batch_kernel(const uint8_t* __restrict__ in, uint64_t pitch,
                                                           const uint64_t* __restrict__ n, uint32_t* hist) {
    const int k = blockIdx.y;
    hist_body(in + uint64_t(k) * pitch, n[k], hist + 256 * k);
}
__global__ __launch_bounds__(kTPB) void first_scan_batch_kernel(const uint8_t* __restrict__ in, uint64_t pitch,
                                                                const uint64_t* __restrict__ n, const uint32_t* hist,
                                                                unsigned long long* first, unsigned* unresolved) {
    const int k = blockIdx.x;
    first_scan_body(in + uint64_t(k) * pitch, n[k], hist + 256 * k, first + 256 * k, unresolved + k);
}
__global__ __launch_bounds__(kTPB) void first_full_batch_kernel(const uint8_t* __restrict__ in, uint64_t pitch,
                                                                const uint64_t* __restrict__ n, const uint32_t* hist,
                                                                unsigned long long* first, const unsigned* unresolved) {
    const int k = blockIdx.y;
    first_full_body(in + uint64_t(k) * pitch, n[k], hist + 256 * k, first + 256 * k, unresolved + k);
}

// The first-occurrence pass of the counted pipeline (ie_encode_images_counted, then
// ie_huffman_hist_batch_ends_async): string blockIdx.x's length from its end bit, its counts from
// the encoder's histogram -- CLEARED here for the next counted encode (no memset launch) -- and the
// counts, first positions and unresolved flag written straight into the caller's pinned read-back
// slot h_* (no copy launch).  n / first / unresolved (device) keep what first_full needs for the
// rare string whose scan stopped short (run by the host's wait, ie_huffman_hist_batch_wait).
__global__ __launch_bounds__(kTPB) void first_scan_counted_kernel(const uint8_t* __restrict__ in, uint64_t pitch,
                                                                  const uint64_t* __restrict__ ends, uint64_t cap,
                                                                  uint32_t* hist, uint64_t* n_out,
                                                                  unsigned long long* first, unsigned* unresolved,
                                                                  uint32_t* h_hist, unsigned long long* h_first,
                                                                  unsigned* h_unres) {
    const int k = blockIdx.x, tid = threadIdx.x;
    const uint64_t n = min<uint64_t>((ends[k] + 7) / 8, cap);
    const uint32_t hv = hist[256 * k + tid];
    hist[256 * k + tid] = 0u;
    h_hist[256 * k + tid] = hv;
    unsigned u;
    const unsigned long long f = first_scan_core(in + uint64_t(k) * pitch, n, hv, &u);
    first[256 * k + tid] = f;
    h_first[256 * k + tid] = f;
    if (tid == 0) {
        n_out[k] = n;
        unresolved[k] = u;
        h_unres[k] = u;
    }
}
void launch_first_counted(const uint8_t* in, uint64_t pitch, const uint64_t* ends, uint64_t cap, int count,
                          uint32_t* hist, uint64_t* n, unsigned long long* first, unsigned* unresolved, uint32_t* h_hist,
                          unsigned long long* h_first, unsigned* h_unres, hipStream_t s) {
    hipLaunchKernelGGL(first_scan_counted_kernel, dim3(count), dim3(kTPB), 0, s, in, pitch, ends, cap, hist, n, first,
                       unresolved, h_hist, h_first, h_unres);
}
// first_full over a batch whose first_scan left strings unresolved (hist: any device-readable copy)
void launch_first_full_batch(const uint8_t* in, uint64_t pitch, const uint64_t* n, uint64_t maxn, int count,
                             const uint32_t* hist, unsigned long long* first, const unsigned* unresolved, hipStream_t s) {
    const uint64_t tiles = (maxn + kHistTile - 1) / kHistTile;
    const uint64_t per = (4096 + count - 1) / count;
    const int gx = int(tiles < per ? (tiles ? tiles : 1) : per);
    hipLaunchKernelGGL(first_full_batch_kernel, dim3(gx, count), dim3(kTPB), 0, s, in, pitch, n, hist, first,
                       unresolved);
}

// n[k] = the byte length of a stream ending at bit ends[k] (capped at cap): the batched Huffman
// pass reads the encoder's own end bits, with no host round trip in between.
// Also clears the histograms (hist = 0) and first positions (~0) of the count strings when given:
// no separate memset launches in the pipeline.
__global__ void ends_to_bytes_kernel(const uint64_t* ends, uint64_t cap, int count, uint64_t* n, uint32_t* hist,
                                     unsigned long long* first) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < count) n[k] = min<uint64_t>((ends[k] + 7) / 8, cap);
    if (k < 256 * count) {
        if (hist) hist[k] = 0u;
        if (first) first[k] = ~0ull;
    }
}
void launch_ends_to_bytes(const uint64_t* ends, uint64_t cap, int count, uint64_t* n, hipStream_t s, uint32_t* hist,
                          unsigned long long* first) {
    const int threads = (hist || first) ? 256 * count : count;
    hipLaunchKernelGGL(ends_to_bytes_kernel, dim3((threads + kTPB - 1) / kTPB), dim3(kTPB), 0, s, ends, cap, count, n,
                       hist, first);
}

// unresolved: one word per string (device scratch)
void launch_hist(const uint8_t* in, uint64_t n, uint32_t* hist, unsigned long long* first, unsigned* unresolved,
                 hipStream_t s) {
    const uint64_t tiles = (n + kHistTile - 1) / kHistTile;
    const int grid = int(tiles < 2048 ? (tiles ? tiles : 1) : 2048);
    hipLaunchKernelGGL(hist_kernel, dim3(grid), dim3(kTPB), 0, s, in, n, hist);
    hipLaunchKernelGGL(first_scan_kernel, dim3(1), dim3(kTPB), 0, s, in, n, hist, first, unresolved);
    hipLaunchKernelGGL(first_full_kernel, dim3(grid), dim3(kTPB), 0, s, in, n, hist, first, unresolved);
}

void launch_hist_batch(const uint8_t* in, uint64_t pitch, const uint64_t* n, uint64_t maxn, int count, uint32_t* hist,
                       unsigned long long* first, unsigned* unresolved, hipStream_t s, bool counts) {
    const uint64_t tiles = (maxn + kHistTile - 1) / kHistTile;
    const uint64_t per = (4096 + count - 1) / count;  // ~4096 workgroups over the batch
    const int gx = int(tiles < per ? (tiles ? tiles : 1) : per);
    if (counts) hipLaunchKernelGGL(hist_batch_kernel, dim3(gx, count), dim3(kTPB), 0, s, in, pitch, n, hist);
    hipLaunchKernelGGL(first_scan_batch_kernel, dim3(count), dim3(kTPB), 0, s, in, pitch, n, hist, first, unresolved);
    hipLaunchKernelGGL(first_full_batch_kernel, dim3(gx, count), dim3(kTPB), 0, s, in, pitch, n, hist, first,
                       unresolved);
}

// One tile = kTPB threads x BPT input bytes, codes of up to MAXLEN bits: <16, 32> for any code,
// <64, 16> for Huffman codes (<= 15 bits) and the identity copy -- 4x the bytes per tile, so a
// quarter of the tiles (and look-backs) for the same LDS image size.
// The tile image is sized per launch for the table's longest code (pack_image_words: dynamic LDS),
// so short-code tables leave room for more resident tiles.
__host__ __device__ constexpr int pack_image_words(int bpt, int maxlen) { return kTPB * bpt * maxlen / 32 + 4; }
template <int BPT, int MAXLEN>
__global__ __launch_bounds__(kTPB, IE_PACK_WAVES) void pack_kernel(PackArgs a) {
    extern __shared__ uint32_t smem[];  // [pack_image_words(BPT, a.maxlen)] image, [32] misc
    __shared__ uint32_t s_code[256];
    __shared__ uint8_t s_len[256];
    uint32_t* img = smem;
    uint32_t* misc = smem + pack_image_words(BPT, min(max(a.maxlen, 1), MAXLEN));
    const int tid = threadIdx.x;
    // tile order = dispatch order (see encode_kernel); the atomic ticket is the fallback
    if (a.ticket && tid == 0) misc[4] = uint32_t(atomicAdd(a.ticket, 1ull) - a.ticket_base);
    if (a.ticket) __syncthreads();
    const int t = a.ticket ? int(misc[4]) : int(blockIdx.x);
    if (t >= a.ntiles) return;
    // the tile's string: its chain, bytes, code table and output.  A batch interleaves its strings'
    // tiles (tile t -> string t % count, position t / count; past a string's last tile a slot is
    // idle), so every chain advances together and each has only ~1/count of the resident tiles in
    // flight: the look-back finds an inclusive prefix within its first window.
    int k = 0, chain_pos = t, step = 1;
    const uint8_t* in = a.in;
    uint64_t n = a.n, start = a.start_bit;
    uint32_t* out = a.out;
    const uint32_t* hdr = a.out;  // words holding the bits before `start`
    bool last = (t == a.ntiles - 1);
    if (a.count) {
        k = t % a.count;
        chain_pos = t / a.count;
        step = a.count;
        const uint64_t tiles_k = a.tiles[k];
        if (uint64_t(chain_pos) >= tiles_k) return;  // idle slot: no chain state, no output
        last = uint64_t(chain_pos) + 1 == tiles_k;
        in = a.in + uint64_t(k) * a.in_pitch;
        n = a.bn[k];
        start = a.bstart[k];
        out = a.out + uint64_t(k) * a.out_pitch_words;
        hdr = a.prefix + uint64_t(k) * a.prefix_pitch_words;
        if (chain_pos == 0)  // the prefix words (the chain's bits before `start` live in hdr)
            for (uint32_t w = tid; w < uint32_t(start >> 5); w += kTPB) out[w] = hdr[w];
    }
    if constexpr (MAXLEN <= 16) {  // {code, len << 16}
        s_code[tid] = (a.code[256 * k + tid] & 0xFFFFu) | (uint32_t(a.len[256 * k + tid]) << 16);
    } else {
        s_code[tid] = a.code[256 * k + tid];
        s_len[tid] = a.len[256 * k + tid];
    }
    __syncthreads();

    const uint64_t p = uint64_t(chain_pos) * (kTPB * BPT) + uint64_t(tid) * BPT;
    uint32_t w[BPT / 4];  // the thread's bytes, four per word
    int nb = 0;
    if (p < n) nb = int(min<uint64_t>(BPT, n - p));
    if (nb == BPT && ((reinterpret_cast<uintptr_t>(in) & 15) == 0)) {
#pragma unroll
        for (int q = 0; q < BPT / 16; q++) {
            const uint4 v = *reinterpret_cast<const uint4*>(in + p + 16 * q);
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < BPT / 4; q++) {
            uint32_t v = 0;
#pragma unroll
            for (int e = 0; e < 4; e++) v |= (4 * q + e < nb) ? uint32_t(in[p + 4 * q + e]) << (8 * e) : 0u;
            w[q] = v;
        }
    }
    auto byte = [&](int e) -> uint32_t { return (w[e >> 2] >> (8 * (e & 3))) & 0xFFu; };
    uint32_t mybits = 0;
    // codes of <= 16 bits: one LDS read per byte ({code, len << 16}); the emission's units, pairs
    // of codes (<= 32 bits), stay in registers: cp[i] the pair's bits, lp the lengths, 4 per word
    constexpr int NPAIR = MAXLEN <= 16 ? BPT / 2 : 1;
    uint32_t cp[NPAIR], lp[(NPAIR + 3) / 4];
    if constexpr (MAXLEN <= 16) {
#pragma unroll
        for (int i = 0; i < NPAIR; i++) {
            const uint32_t e1 = (2 * i < nb) ? s_code[byte(2 * i)] : 0u;
            const uint32_t e2 = (2 * i + 1 < nb) ? s_code[byte(2 * i + 1)] : 0u;
            const uint32_t l2 = e2 >> 16, l = (e1 >> 16) + l2;
            cp[i] = ((e1 & 0xFFFFu) << l2) | (e2 & 0xFFFFu);
            if (i % 4 == 0) lp[i / 4] = l;
            else lp[i / 4] |= l << (8 * (i % 4));
            mybits += l;
        }
    } else {
#pragma unroll
        for (int e = 0; e < BPT; e++) mybits += (e < nb) ? s_len[byte(e)] : 0u;
    }

    uint32_t A;
    const uint32_t off = block_excl_scan(mybits, misc, &A);
    if (tid == 0) chain_publish_count(a.st, t, chain_pos, a.tag, A);
    Probe pr{0, 0, 0};
    if (tid < 64 && chain_pos != 0) pr = probe_issue(a.st, t, chain_pos, step, 0, kProbe0);
    const uint32_t nw = (A + 31) >> 5;
    if constexpr (MAXLEN <= 16) {
        // only the words two threads share need zeros first: every thread's first and end word
        // (and the word past the image, the store's look-ahead); the words strictly inside a
        // thread's bits are written whole, without an OR
        if (mybits) {
            img[off >> 5] = 0u;
            img[(off + mybits) >> 5] = 0u;
        }
        if (tid == 0) img[nw] = 0u;
    } else {
        for (uint32_t w = tid; w < nw + 1; w += kTPB) img[w] = 0u;
    }
    __syncthreads();
    if (mybits) {
        if constexpr (MAXLEN <= 16) {
            // two codes at a time (<= 32 bits), so at most one completed word per step; bits of
            // acc above the pending ones are stale and never reach a word (32-bit truncation).
            // The first completed word may hold the previous thread's bits (OR); later ones are
            // this thread's alone (plain store); the partial end word is shared with the next.
            uint64_t acc = 0;
            uint32_t n = off & 31u, wi = off >> 5;
            const uint32_t w0 = wi;
#pragma unroll
            for (int i = 0; i < NPAIR; i++) {
                const uint32_t l = (lp[i / 4] >> (8 * (i % 4))) & 0xFFu;
                acc = (acc << l) | cp[i];
                n += l;
                if (n >= 32u) {
                    n -= 32u;
                    if (wi == w0) atomicOr(&img[wi], uint32_t(acc >> n));
                    else img[wi] = uint32_t(acc >> n);
                    wi++;
                }
            }
            if (n) atomicOr(&img[wi], uint32_t(acc << (32u - n)));
        } else {
            BitSink sink(img, off);
#pragma unroll
            for (int e = 0; e < BPT; e++)
                if (e < nb) sink.put(s_len[byte(e)], s_code[byte(e)]);
            sink.finish();
        }
    }
    __syncthreads();

    // one chain per string in tile order -- the same protocol as encode_kernel
    const uint64_t excl = chain_resolve(a.st, t, chain_pos, step, a.tag, img, A, hdr, start, a.err, misc, pr);
    if (tid == 0 && last) a.chain_end[k] = start + excl + A;
    store_image(out, img, A, start + excl, misc[7], last);
}

// Output words [w0, w1) of `out` (32-bit stream words stored as bytes, MSB-first) receive the n
// input bytes' bits from stream bit A on: word W holds stream bits [32W, 32W + 32) = input bits
// [32W - A, 32W - A + 32).  Bits before A (first word only) keep out's own bits -- the one thread
// that writes word w0 reads it first; bits past the input's end are zero.  Thread t writes words
// w0 + 4t .. +3.
__global__ __launch_bounds__(256) void bitshift_kernel(const uint8_t* __restrict__ in, uint64_t n, uint32_t* out,
                                                       uint64_t A, uint64_t w0, uint64_t w1) {
    const uint64_t W0 = w0 + 4ull * (uint64_t(blockIdx.x) * 256u + threadIdx.x);
    if (W0 >= w1) return;
    const uint64_t nw_in = (n + 3) / 4;
    // big-endian input word q (q < 0 or past the end: 0; the last word's bytes past n: 0)
    auto inw = [&](int64_t q) -> uint32_t {
        if (q < 0 || uint64_t(q) >= nw_in) return 0u;
        const uint64_t b = uint64_t(q) * 4;
        if (b + 4 <= n && !(reinterpret_cast<uintptr_t>(in + b) & 3))
            return bswap32(*reinterpret_cast<const uint32_t*>(in + b));
        uint32_t v = 0;
        for (int e = 0; e < 4; e++) v |= (b + e < n ? uint32_t(in[b + e]) : 0u) << (24 - 8 * e);
        return v;
    };
    // input bit offset of word W0: d = 32*W0 - A = 32*q + r, 0 <= r < 32 (the same r for every word)
    const int64_t d = int64_t(32 * W0) - int64_t(A);
    const int64_t q = (d >= 0) ? (d >> 5) : -((-d + 31) >> 5);
    const uint32_t r = uint32_t(d - 32 * q);
    uint32_t wq[5];
#pragma unroll
    for (int k = 0; k < 5; k++) wq[k] = inw(q + k);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t W = W0 + k;
        if (W >= w1) break;
        uint32_t v = __builtin_amdgcn_alignbit(wq[k], wq[k + 1], 32u - r);  // bits [r, r+32) of wq[k]:wq[k+1]
        if (r == 0) v = wq[k];
        if (W == w0 && (A & 31)) {  // the caller's bits before A
            const uint32_t keep = ~(0xFFFFFFFFu >> (A & 31));
            v = (bswap32(out[W]) & keep) | (v & ~keep);
        }
        out[W] = bswap32(v);
    }
}

void launch_bitshift(const uint8_t* in, uint64_t n, uint32_t* out, uint64_t start_bit, hipStream_t s) {
    const uint64_t w0 = start_bit / 32, w1 = (start_bit + 8 * n + 31) / 32;
    if (w1 <= w0) return;
    const uint64_t threads = (w1 - w0 + 3) / 4;
    hipLaunchKernelGGL(bitshift_kernel, dim3(unsigned((threads + 255) / 256)), dim3(256), 0, s, in, n, out, start_bit,
                       w0, w1);
}

#ifndef IE_PACK_BPT
#define IE_PACK_BPT 64  // input bytes per thread of a pack tile for codes of <= 16 bits (32: 138 against 88 us)
#endif
int pack_tile_bytes(int maxlen) { return maxlen <= 16 ? kTPB * IE_PACK_BPT : kTPB * 16; }

void launch_pack(const PackArgs& a, hipStream_t s) {
    const int ml = std::max(1, a.maxlen);
    if (ml <= 16)
        hipLaunchKernelGGL((pack_kernel<IE_PACK_BPT, 16>), dim3(a.ntiles), dim3(kTPB),
                           size_t(pack_image_words(IE_PACK_BPT, ml) + 32) * 4, s, a);
    else
        hipLaunchKernelGGL((pack_kernel<16, 32>), dim3(a.ntiles), dim3(kTPB),
                           size_t(pack_image_words(16, std::min(ml, 32)) + 32) * 4, s, a);  // (ml <= 32: checked by the callers)
}

}  // namespace ie
