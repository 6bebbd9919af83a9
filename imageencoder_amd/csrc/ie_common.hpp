// imageencoder_amd/csrc/ie_common.hpp -- device building blocks shared by the gfx950 kernels:
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

// The lane id computed afresh (two VALU): an opaque value the compiler cannot CSE with earlier
// copies, so a kernel that re-derives it per phase holds no lane-derived VGPR across its phases
// (values live across a whole tile otherwise end up spilled at higher occupancy).
__device__ __forceinline__ int fresh_lane() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations but not for its
// global loads, so a prefetch of the next tile's pixels stays in flight across it (a
// __syncthreads() would drain it).  Global memory is never handed between the threads of a
// workgroup through these barriers.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Make a wave's LDS writes visible to its other lanes (LDS operations of one wave execute in
// order; this only stops the compiler from moving accesses across).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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

// Inclusive minimum over lanes 0..l of a wave by DPP row shifts and row broadcasts (six VALU, no
// LDS): lanes a shift reads from outside the wave keep their own value.
__device__ __forceinline__ uint32_t wave_incl_min_dpp(uint32_t v) {
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(int(~0u), int(v), 0x111, 0xF, 0xF, false)));  // row_shr:1
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(int(~0u), int(v), 0x112, 0xF, 0xF, false)));  // row_shr:2
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(int(~0u), int(v), 0x114, 0xF, 0xF, false)));  // row_shr:4
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(int(~0u), int(v), 0x118, 0xF, 0xF, false)));  // row_shr:8
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(int(~0u), int(v), 0x142, 0xA, 0xF, false)));  // row_bcast:15
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(int(~0u), int(v), 0x143, 0xC, 0xF, false)));  // row_bcast:31
    return v;
}

// Exclusive workgroup scan of per-thread bit counts (TPB threads).  scratch: >= TPB/64 words of
// LDS.  Returns the thread's exclusive offset; *total receives the workgroup sum.
template <int TPB = kTPB>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t* total) {
    const int tid = threadIdx.x, wid = tid >> 6;
    const uint32_t incl = wave_incl_scan(v);
    if constexpr (TPB == 64) {
        *total = __shfl(incl, 63, 64);
        return incl - v;
    }
    if ((tid & 63) == 63) scratch[wid] = incl;
    lds_barrier();
    uint32_t before = 0, sum = 0;
#pragma unroll
    for (int w = 0; w < TPB / 64; w++) {
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

// ---- tile chain protocol ------------------------------------------------------------------
// A chain is a sequence of tiles whose bit images are concatenated; tile t sits at position
// chain_pos of its chain and its d-th predecessor (d = 0, 1, ...) is tile t - step*(d+1).
// Every tile publishes its state with agent-scope stores of single 8-byte words, so the payload
// travels inside the atomic word and no fence is needed:
//   st[kGran t + 0] = {tag:8 | 0:1 | aggregate:55}  as soon as the tile's bit count is known
//                   = {tag:8 | 1:1 | inclusive:55}  once the look-back has resolved the prefix
//   st[kGran t + 2] = {tag:8 | tail:32}            the last 32 bits of the chain up to and
//                                                  including t
// The early aggregate lets successors resolve their offsets while this tile is still emitting.
// The inclusive value overwrites the aggregate in the same word (both stores come from the one
// thread that publishes the tile, in that order), so a probe reads ONE word per predecessor:
// whichever it sees is a correct term of the look-back sum.  (Round 5 kept them in two words and
// read both: every probed predecessor cost two uncached loads -- C4's single chain reads 1.7 KB of
// other XCDs' state lines per tile.)
// granules per tile in the state array: 3 packed (24 B per tile) or IE_GRAN_STRIDE words apart
// (16: each tile's state in a 128-B line of its own, no false sharing between tiles)
#ifndef IE_GRAN_STRIDE
#define IE_GRAN_STRIDE 16
#endif
constexpr int kGran = IE_GRAN_STRIDE;
static_assert(kGran >= 3 && kGran <= kStateWordsPerTile, "three granules per tile within the allocation");

#ifndef IE_STATE_1W
#define IE_STATE_1W 1  // 0: aggregate and inclusive in two words (round 5; A/B builds)
#endif
constexpr uint64_t kIncl = 1ull << 55, kMask55 = kIncl - 1;
// g = 0: the aggregate, 1: the inclusive prefix, 2: the tail
__device__ __forceinline__ void publish(uint64_t* st, int t, int g, uint32_t tag, uint64_t v) {
    if (IE_STATE_1W && g < 2)
        st_state(&st[kGran * t], (uint64_t(tag) << 56) | (g == 1 ? kIncl : 0ull) | (v & kMask55));
    else
        st_state(&st[kGran * t + g], (uint64_t(tag) << 56) | (v & kMask56));
}

// A look-back probe: the states of the 64 chain predecessors d0 .. d0+63 of tile t (both
// granules at once) and, for d0 = 0, the immediate predecessor's tail, loaded by one wave.  The
// first probe is issued right after the tile publishes its own count, so its loads are in flight
// while the tile emits its records; it is evaluated afterwards.
struct Probe {
    uint64_t gi, ga, gt;
};

// First probe window: most tiles find an inclusive prefix among their nearest predecessors, and
// every probed state is an uncached agent-scope load, so the first round reads only a few.
#ifndef IE_PROBE0
#define IE_PROBE0 16
#endif
constexpr int kProbe0 = IE_PROBE0;

// One probed predecessor: *status 2 (inclusive prefix), 1 (aggregate) or 0 (nothing published in
// this launch), *val its value.
__device__ __forceinline__ void probe_status(const Probe& p, uint32_t tag, int* status, uint64_t* val) {
    if (IE_STATE_1W) {
        const bool mine = uint32_t(p.ga >> 56) == tag;
        *status = mine ? ((p.ga & kIncl) ? 2 : 1) : 0;
        *val = p.ga & kMask55;
    } else if (uint32_t(p.gi >> 56) == tag) {
        *val = p.gi & kMask56;
    } else {
        *status = (uint32_t(p.ga >> 56) == tag) ? 1 : 0;
        *val = p.ga & kMask56;
    }
}

__device__ __forceinline__ Probe probe_issue(const uint64_t* st, int t, int chain_pos, int step, int d0,
                                             int width) {
    Probe p;
    p.gi = p.ga = p.gt = 0;
    const int lane = lane_id();
    const int d = d0 + lane;
    if (lane < width && chain_pos - 1 - d >= 0) {
        const int idx = t - step * (d + 1);
        p.ga = ld_state(&st[kGran * idx]);
        p.gi = IE_STATE_1W ? 0ull : ld_state(&st[kGran * idx + 1]);
    }
    if (d0 == 0 && lane == 0 && chain_pos > 0) p.gt = ld_state(&st[kGran * (t - step) + 2]);
    return p;
}

// Later look-back windows are issued kLbAhead at a time (64 predecessors each, all loads in
// flight together): a tile far from the nearest resolved predecessor -- a launch whose tiles all
// reach their look-back at once, e.g. one frame -- walks back 64 * kLbAhead tiles per round trip.
#ifndef IE_LB_AHEAD
#define IE_LB_AHEAD 8
#endif
constexpr int kLbAhead = IE_LB_AHEAD;

// Exclusive prefix of tile t, executed by ONE wave from a first probe (width kProbe0): the sum of
// aggregates up to the nearest inclusive value (predecessors publish their aggregate as soon as
// their bit count is known).  Later windows read 64 predecessors.  Returns the prefix in every
// lane.
// deep: the launch's tiles all reach their look-back at about the same time (a launch too small to
// fill the chip), so a tile's nearest inclusive predecessor is far away: the windows after the
// first probe are issued at once, before it is evaluated.
template <int kLbAhead = ie::kLbAhead, int kLbW = 64>
__device__ uint64_t lookback_wave(Probe p, const uint64_t* st, int t, int chain_pos, int step, uint32_t tag,
                                  unsigned* err, unsigned* rounds = nullptr, bool deep = false,
                                  int width0 = kProbe0) {
    const int lane = lane_id();
    uint64_t excl = 0;
    int d0 = 0, width = width0;  // (the first probe's width)
    const int wl = deep ? 64 : kLbW;  // the later windows' width
    unsigned spins = 0;
    Probe ahead[kLbAhead];  // windows d0 + 64, d0 + 128, ... already in flight
    int nahead = 0;
    if (rounds) *rounds = 0;
    if (deep && chain_pos > kProbe0) {
#pragma unroll
        for (int k = kLbAhead - 1; k >= 0; k--) ahead[k] = probe_issue(st, t, chain_pos, step, kProbe0 + 64 * (kLbAhead - 1 - k), 64);
        nahead = kLbAhead;
    }
    for (;;) {
        const int d = d0 + lane;
        int status = 2;  // before the chain start: a virtual inclusive prefix of 0
        uint64_t val = 0;
        if (lane >= width) {
            status = 3;  // outside the window
        } else if (chain_pos - 1 - d >= 0) {
            probe_status(p, tag, &status, &val);
        }
        const uint64_t incl = __ballot(status == 2);
        const int dP = incl ? (__ffsll((unsigned long long)incl) - 1) : width;
        const uint64_t before = (dP < 64) ? ((1ull << dP) - 1ull) : ~0ull;
        if (__ballot(status == 0) & before) {
            if (++spins > kSpinLimit) {
                if (lane == 0) atomicAdd(&err[0], 1u);
                return excl;
            }
            __builtin_amdgcn_s_sleep(1);
            p = probe_issue(st, t, chain_pos, step, d0, width);
            if (rounds) *rounds += 1;
            continue;
        }
        excl += wave_sum64((lane <= dP && lane < width) ? val : 0ull);
        if (dP < width) return excl;
        d0 += width;
        width = wl;
        if (nahead == 0) {  // the next kLbAhead windows in one round trip
#pragma unroll
            for (int k = kLbAhead - 1; k >= 0; k--) ahead[k] = probe_issue(st, t, chain_pos, step, d0 + wl * (kLbAhead - 1 - k), wl);
            nahead = kLbAhead;
            if (rounds) *rounds += 0x10000;
        }
        // (ahead[nahead - 1] is window d0; a window read ahead may be re-probed by the spin above)
        p = ahead[0];
#pragma unroll
        for (int k = 1; k < kLbAhead; k++)
            if (k == nahead - 1) p = ahead[k];
        nahead--;
    }
}

// One probe window's share of a look-back (predecessors d0 .. d0 + width - 1 of the tile, as probe
// p read them): found -- the nearest inclusive prefix (or the chain start) lies in the window;
// sum -- the values up to and including it (the whole window's aggregates when not found);
// ready -- every value summed was published.  Every lane gets the result.
struct WinSum {
    uint64_t sum;
    bool found, ready;
};
__device__ __forceinline__ WinSum window_sum(const Probe& p, int chain_pos, int d0, int width, uint32_t tag) {
    const int lane = lane_id(), d = d0 + lane;
    int status = 2;  // before the chain start: a virtual inclusive prefix of 0
    uint64_t val = 0;
    if (lane >= width) {
        status = 3;
    } else if (chain_pos - 1 - d >= 0) {
        probe_status(p, tag, &status, &val);
    }
    const uint64_t incl = __ballot(status == 2);
    const int dP = incl ? (__ffsll((unsigned long long)incl) - 1) : width;
    const uint64_t upto = (dP < 64) ? ((2ull << dP) - 1ull) : ~0ull;  // lanes 0 .. dP
    WinSum r;
    r.ready = !(__ballot(status == 0) & upto);
    r.sum = wave_sum64((lane <= dP && lane < width) ? val : 0ull);
    r.found = dP < width;
    return r;
}

// The tail granule of tile idx (one thread).
__device__ __forceinline__ uint32_t wait_tail(const uint64_t* st, int idx, uint32_t tag, unsigned* err,
                                              unsigned* polls = nullptr) {
    unsigned sp = 0;
    for (;;) {
        const uint64_t g = ld_state(&st[kGran * idx + 2]);
        if (polls) *polls += 1;
        if (uint32_t(g >> 56) == tag) return uint32_t(g);
        if (++sp > kSpinLimit) {
            atomicAdd(&err[0], 1u);
            return 0u;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// Phase A, right after the tile's bit count A is known: publish the aggregate (and, for a
// chain's first tile, the inclusive prefix).  Thread 0 only.
__device__ __forceinline__ void chain_publish_count(uint64_t* st, int t, int chain_pos, uint32_t tag, uint32_t A) {
    publish(st, t, 0, tag, A);
    if (chain_pos == 0) publish(st, t, 1, tag, A);
}

// chain_resolve's look-back windows after the first probe (encode_kernel, pack_kernel)
#ifndef IE_CR_AHEAD
#define IE_CR_AHEAD 1
#endif
#ifndef IE_CR_LBW
#define IE_CR_LBW 32
#endif

// Phase B, after the LDS image is complete (all threads): tail publication, look-back from the
// probe `pr` wave 0 issued after phase A, and the
// values the store needs (wave 0 resolves; the others wait at the closing barrier).  out: the
// chain's output words; start: the chain's first bit.  Returns the exclusive prefix; misc[7]
// receives the 32 bits preceding the tile (its store's `prev`).
__device__ __forceinline__ uint64_t chain_resolve(uint64_t* st, int t, int chain_pos, int step, uint32_t tag,
                                                  const uint32_t* img, uint32_t A, const uint32_t* out,
                                                  uint64_t start, unsigned* err, uint32_t* misc, const Probe& pr,
                                                  uint64_t* dbg = nullptr, bool defer_tail = false, bool deep = false) {
    const int tid = threadIdx.x;
    if (tid == 0) {
        const uint32_t my_tail = image_tail32(img, A);
        if (chain_pos == 0) {
            // chain start: the bits before `start` belong to the caller (header); keep them
            const uint32_t s = uint32_t(start & 31);
            const uint32_t ptail = s ? (bswap32(out[start >> 5]) >> (32 - s)) : 0u;
            const uint32_t tl = (A >= 32) ? my_tail : ((A ? (ptail << A) : ptail) | my_tail);
            publish(st, t, 2, tag, tl);
            misc[5] = 0;
            misc[6] = 0;
            misc[7] = ptail;
            misc[8] = 0;
        } else if (A >= 32) {
            publish(st, t, 2, tag, my_tail);
        }
    }
    if (chain_pos != 0 && tid < 64) {
        unsigned rounds = 0, polls = 0;
        const uint64_t excl = lookback_wave<IE_CR_AHEAD, IE_CR_LBW>(pr, st, t, chain_pos, step, tag, err,
                                                                    dbg ? &rounds : nullptr, deep);
        if (tid == 0) {
            publish(st, t, 1, tag, excl + A);
            const bool have = uint32_t(pr.gt >> 56) == tag;
            // deferred: only the tile's first output word needs the predecessor's tail, and only
            // when the tile starts inside a word; store_tile() fetches it after the bulk store
            const bool later = defer_tail && !have && A >= 32 && ((start + excl) & 31) != 0;
            const uint32_t ptail = have ? uint32_t(pr.gt) : later ? 0u : wait_tail(st, t - step, tag, err, &polls);
            misc[8] = later ? 1u : 0u;
            if (dbg) *dbg = (uint64_t(rounds) << 32) | polls;
            if (A < 32) {
                // a short tile's tail carries predecessor bits
                publish(st, t, 2, tag, (A ? (ptail << A) : ptail) | image_tail32(img, A));
            }
            misc[5] = uint32_t(excl);
            misc[6] = uint32_t(excl >> 32);
            misc[7] = ptail;
        }
    }
    lds_barrier();
    return uint64_t(misc[5]) | (uint64_t(misc[6]) << 32);
}

// Store a tile's bit image L (bits bits, tile bit 0 at absolute stream bit P) into the word
// array out.  Word floor(P/32) is completed with `prev` (the 32 bits that precede bit P,
// right-aligned).  The last partial word is left to the successor unless `last`.  Aligned runs of
// four words go out as one 16-byte store per thread (TPB threads).
#ifndef IE_NT_STORE
#define IE_NT_STORE 1
#endif
// An optional observer of every stored word: cnt(word index, value as stored).
struct NoCount {
    __device__ __forceinline__ void operator()(uint64_t, uint32_t) const {}
};
template <int TPB = kTPB, class Cnt = NoCount>
__device__ __forceinline__ void store_image(uint32_t* out, const uint32_t* L, uint32_t bits, uint64_t P,
                                            uint32_t prev, bool last, bool skip0 = false, const Cnt& cnt = Cnt()) {
    // Output word r (r = 0 at word floor(P/32)) is the funnel shift of image words r-1 and r:
    // alignbit(L[r-1], L[r], s), with L[-1] = prev and s = 0 giving L[r] itself.  The caller's
    // image is zero through word ceil(bits/32), so L[r] needs no bound check.
    const uint64_t w0 = P >> 5;
    const uint32_t s = uint32_t(P & 31);
    const uint64_t end = P + bits;
    const uint64_t w1 = last ? ((end + 31) >> 5) : (end >> 5);
    const uint32_t nw = uint32_t(w1 - w0);
    const uint32_t tid = threadIdx.x;
    auto word = [&](uint32_t r) -> uint32_t {
        const uint32_t pw = (r == 0) ? prev : L[r - 1];
        return bswap32(__builtin_amdgcn_alignbit(pw, L[r], s));
    };
    // skip0: word 0 is written later by the caller (its predecessor bits are not known yet)
    const uint32_t head0 = min(nw, uint32_t((4u - uint32_t(w0 & 3u)) & 3u));
    const uint32_t head = (skip0 && head0 == 0) ? min(nw, 4u) : head0;
    if (tid < head && !(skip0 && tid == 0)) {
        const uint32_t v = word(tid);
        out[w0 + tid] = v;
        cnt(w0 + tid, v);
    }
    const uint32_t nq = (nw - head) >> 2;
#pragma unroll 2
    for (uint32_t q = tid; q < nq; q += TPB) {
        const uint32_t r = head + 4u * q;
        const uint32_t* l = L + r;
        const uint32_t am = L[max(r, 1u) - 1u];  // branch-free: read a valid word, then select
        const uint32_t a0 = (r == 0) ? prev : am;
        const uint32_t b0 = l[0], b1 = l[1], b2 = l[2], b3 = l[3];
        uint4 v;
        v.x = bswap32(__builtin_amdgcn_alignbit(a0, b0, s));
        v.y = bswap32(__builtin_amdgcn_alignbit(b0, b1, s));
        v.z = bswap32(__builtin_amdgcn_alignbit(b1, b2, s));
        v.w = bswap32(__builtin_amdgcn_alignbit(b2, b3, s));
#if IE_NT_STORE
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const v4u vv = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(vv, reinterpret_cast<v4u*>(out + w0 + r));
#else
        *reinterpret_cast<uint4*>(out + w0 + r) = v;
#endif
        cnt(w0 + r, v.x);
        cnt(w0 + r + 1, v.y);
        cnt(w0 + r + 2, v.z);
        cnt(w0 + r + 3, v.w);
    }
    const uint32_t t0 = head + 4u * nq;
    if (tid < nw - t0) {
        const uint32_t v = word(t0 + tid);
        out[w0 + t0 + tid] = v;
        cnt(w0 + t0 + tid, v);
    }
}

// The tile store after chain_resolve(..., defer_tail = true): the bulk of the words first, then
// (misc[8] set) thread 0 fetches the predecessor's tail and completes the first word.
template <int TPB = kTPB, class Cnt = NoCount>
__device__ __forceinline__ void store_tile(uint32_t* out, const uint32_t* L, uint32_t bits, uint64_t P,
                                           const uint32_t* misc, bool last, const uint64_t* st, int pred,
                                           uint32_t tag, unsigned* err, const Cnt& cnt = Cnt()) {
    const bool pend = misc[8] != 0u;
    store_image<TPB>(out, L, bits, P, misc[7], last, pend, cnt);
    if (pend && threadIdx.x == 0) {
        const uint32_t pt = wait_tail(st, pred, tag, err);
        const uint32_t s = uint32_t(P & 31);
        const uint32_t v = bswap32((pt << (32 - s)) | (L[0] >> s));
        out[P >> 5] = v;
        cnt(P >> 5, v);
    }
}

}  // namespace ie
