// imageencoder_amd/csrc/ie_common.cuh -- device building blocks shared by the gfx950 kernels:
// wave/workgroup scans, the LDS bit sink, the decoupled look-back over tile states and the
// funnel-shift store of a tile's bit image.  Wavefront = 64 lanes, workgroup = kTPB = 256.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ie_device.h"

namespace ie {

constexpr uint64_t kMask56 = (1ull << 56) - 1;
constexpr unsigned kSpinLimit = 1u << 22;  // bounded spins: a protocol bug reports, never hangs

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Inclusive wave scan of a 32-bit value (64 lanes).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(v, d, 64);
        if (l >= d) v += o;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t lo = __shfl_xor(uint32_t(v), d, 64);
        const uint32_t hi = __shfl_xor(uint32_t(v >> 32), d, 64);
        v += (uint64_t(hi) << 32) | lo;
    }
    return v;
}

// Exclusive workgroup scan of per-thread bit counts.  scratch: >= 4 words of LDS.
// Returns the thread's exclusive offset; *total receives the workgroup sum.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t* total) {
    const int tid = threadIdx.x, wid = tid >> 6;
    const uint32_t incl = wave_incl_scan(v);
    if ((tid & 63) == 63) scratch[wid] = incl;
    __syncthreads();
    uint32_t before = 0, sum = 0;
#pragma unroll
    for (int w = 0; w < kTPB / 64; w++) {
        const uint32_t s = scratch[w];
        before += (w < wid) ? s : 0u;
        sum += s;
    }
    *total = sum;
    return before + incl - v;
}

// MSB-first bit sink into the tile's LDS word image (word 0 bit 31 = tile bit 0).  A thread's
// first and last words may be shared with neighbouring threads and are ORed (the image is
// zeroed first); words strictly inside its span are plain stores.
struct BitSink {
    uint32_t* lds;
    uint64_t acc;
    int n;       // valid bits in acc
    int wi;      // next word index
    bool first;
    __device__ __forceinline__ BitSink(uint32_t* l, uint32_t bitoff)
        : lds(l), acc(0), n(int(bitoff & 31)), wi(int(bitoff >> 5)), first(true) {}
    __device__ __forceinline__ void flush_word(uint32_t w) {
        if (first) {
            atomicOr(&lds[wi], w);
            first = false;
        } else {
            lds[wi] = w;
        }
        wi++;
    }
    // append the low `len` (0..32) bits of v
    __device__ __forceinline__ void put(int len, uint32_t v) {
        const uint64_t m = (len >= 32) ? 0xFFFFFFFFull : ((1ull << len) - 1);
        acc = (acc << len) | (uint64_t(v) & m);
        n += len;
        if (n >= 32) {
            n -= 32;
            flush_word(uint32_t(acc >> n));
            acc &= (n ? ((1ull << n) - 1) : 0ull);
        }
    }
    __device__ __forceinline__ void finish() {
        if (n > 0) atomicOr(&lds[wi], uint32_t(acc << (32 - n)));
    }
};

// The last min(bits, 32) bits of a tile image of `bits` bits, right-aligned.
__device__ __forceinline__ uint32_t image_tail32(const uint32_t* L, uint32_t bits) {
    if (bits >= 32) {
        const uint32_t p = bits - 32, w = p >> 5, s = p & 31;
        return s ? ((L[w] << s) | (L[w + 1] >> (32 - s))) : L[w];
    }
    return bits ? (L[0] >> (32 - bits)) : 0u;
}

__device__ __forceinline__ uint64_t ld_state(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_state(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Decoupled look-back executed by the WHOLE workgroup (all kTPB threads must call it).
// Tile t sits at position chain_pos of its chain; its d-th predecessor (d = 0, 1, ...) is tile
// t - step*(d+1).  Every tile publishes two 8-byte granules st[2t] = {tag:8, aggregate:24,
// tail32:32} and st[2t+1] = {tag:8, inclusive:56}, each with ONE agent-scope store, so the
// payload travels inside the atomic word and no fence is needed.  One round trip reads 4*kTPB
// predecessor states; the exclusive prefix is the sum of aggregates up to the nearest
// inclusive value.  Returns the exclusive prefix (chain-relative bits); *pred_tail receives the
// last 32 bits of the chain before t (the immediate predecessor's tail granule).
// sh: >= 8 words of LDS scratch.
__device__ uint64_t lookback_wg(uint64_t* st, int t, int chain_pos, int step, uint32_t tag, uint32_t* pred_tail,
                                unsigned* err, uint32_t* sh) {
    constexpr int Q = 4;                  // predecessors per thread per round
    constexpr int WIN = kTPB * Q;
    constexpr int NONE = 0x7FFFFFFF;
    const int tid = threadIdx.x, wid = tid >> 6;
    int* s_min = reinterpret_cast<int*>(sh);      // [0] nearest inclusive distance
    int* s_x = reinterpret_cast<int*>(sh + 1);    // [1] a not-ready state before it
    uint64_t* s_sum = reinterpret_cast<uint64_t*>(sh + 2);  // [2..9] per-wave sums
    uint64_t excl = 0;
    int d0 = 0;
    unsigned spins = 0;
    if (tid == 0) {
        *s_min = NONE;
        *s_x = 0;
    }
    __syncthreads();
    for (;;) {
        int status[Q];
        uint64_t agg[Q], inc[Q];
        int myP = NONE;
#pragma unroll
        for (int q = 0; q < Q; q++) {
            const int d = d0 + tid * Q + q;
            agg[q] = inc[q] = 0;
            if (chain_pos - 1 - d < 0) {
                status[q] = 2;  // before the chain start: a virtual inclusive prefix of 0
            } else {
                const int idx = t - step * (d + 1);
                const uint64_t gi = ld_state(&st[2 * idx + 1]);
                if (uint32_t(gi >> 56) == tag) {
                    status[q] = 2;
                    inc[q] = gi & kMask56;
                } else {
                    const uint64_t ga = ld_state(&st[2 * idx]);
                    if (uint32_t(ga >> 56) == tag) {
                        status[q] = 1;
                        agg[q] = (ga >> 32) & 0xFFFFFFull;
                    } else {
                        status[q] = 0;
                    }
                }
            }
            if (status[q] == 2 && myP == NONE) myP = d;
        }
        if (myP != NONE) atomicMin(s_min, myP);
        __syncthreads();
        const int dP = *s_min;
        uint64_t contrib = 0;
        bool x = false;
#pragma unroll
        for (int q = 0; q < Q; q++) {
            const int d = d0 + tid * Q + q;
            if (d < dP) {
                x |= (status[q] == 0);
                contrib += agg[q];
            } else if (d == dP) {
                contrib += inc[q];
            }
        }
        if (x) atomicOr(s_x, 1);
        contrib = wave_sum64(contrib);
        if ((tid & 63) == 0) s_sum[wid] = contrib;
        __syncthreads();
        const bool retry = *s_x != 0;
        uint64_t tot = 0;
#pragma unroll
        for (int w = 0; w < kTPB / 64; w++) tot += s_sum[w];
        __syncthreads();
        if (tid == 0) {
            *s_min = NONE;
            *s_x = 0;
        }
        if (retry) {
            if (++spins > kSpinLimit) {
                if (tid == 0) atomicAdd(&err[0], 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
            __syncthreads();
            continue;
        }
        excl += tot;
        __syncthreads();
        if (dP != NONE) break;
        d0 += WIN;
    }
    // the immediate predecessor's tail (published with or before its inclusive value)
    uint32_t tail = 0;
    if (tid == 0) {
        const int idx = t - step;
        unsigned sp = 0;
        for (;;) {
            const uint64_t ga = ld_state(&st[2 * idx]);
            if (uint32_t(ga >> 56) == tag) {
                tail = uint32_t(ga);
                break;
            }
            if (++sp > kSpinLimit) {
                atomicAdd(&err[0], 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    *pred_tail = tail;  // meaningful in thread 0 (the only reader)
    return excl;
}

// Store a tile's bit image L (bits bits, tile bit 0 at absolute stream bit P) into the word
// array out.  Word floor(P/32) is completed with `prev` (the 32 bits that precede bit P,
// right-aligned).  The last partial word is left to the successor unless `last`.
__device__ __forceinline__ void store_image(uint32_t* out, const uint32_t* L, uint32_t bits, uint64_t P,
                                            uint32_t prev, bool last) {
    const uint64_t w0 = P >> 5;
    const uint32_t s = uint32_t(P & 31);
    const uint64_t end = P + bits;
    const uint64_t w1 = last ? ((end + 31) >> 5) : (end >> 5);
    const uint32_t nL = (bits + 31) >> 5;
    const uint32_t nw = uint32_t(w1 - w0);
    for (uint32_t r = threadIdx.x; r < nw; r += kTPB) {
        const uint32_t cur = (r < nL) ? L[r] : 0u;
        uint32_t v;
        if (s == 0) {
            v = cur;
        } else {
            const uint32_t pw = (r == 0) ? prev : L[r - 1];
            v = (pw << (32 - s)) | (cur >> s);
        }
        out[w0 + r] = bswap32(v);
    }
}

}  // namespace ie
