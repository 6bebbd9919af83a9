// imageencoder_amd/csrc/ie_device.h -- structures shared by the host context (ie_capi.cpp) and
// the gfx950 kernels (ie_encode.hip, ie_huffman.hip, ie_decode.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ie_dct.h"

namespace ie {

constexpr int kTPB = 256;  // threads per workgroup: 4 waves of 64

// Per-quant-matrix tables, built once on the host by ie_set_quant (ie_capi.cpp).
struct EncTables {
    // FP32 fast path (separable DCT, see encode_fast in ie_encode.hip)
    float cf[64];   // cf[u*N+i] = float(c[u][i])
    float g[64];    // float(S[uv] / q[uv])
    float thr[64];  // bound on |t32 - t_ref|; < 0: t32 exact (coefficient 0 only)
    float lim[64];  // 0.5 - thr: |t32 - rint(t32)| >= lim flags a possible rounding tie
    DctConsts dct;  // butterfly constants cos(k pi/16)
    Dct4Plan plan4; // 4x4 folded quotient transform (quot4)
    float lim_min;  // min of lim[k] over the non-structural coefficients: one compare per block
    int dc_exact;   // t[0] is exact in FP32 (q[0] a power of two): round it directly
    int rec_bits;   // largest record (bits) any block can produce with this matrix: sizes the tile image
    // 4x4 on the matrix pipe (encode4p_kernel, quot4j in ie_dct.h): the FP32 stage's constants, its
    // own tie limits (the tracked run of quot4j), and the i8 A fragment of every lane: lane l =
    // (r = l & 31, h = l >> 5) holds in byte 4i + j the weight of pixel (i, j) in J[rho], rho =
    // (r & 3) + 4 (r >> 3), when h == (r >> 2) & 1, else 0 -- so D register rho of a lane is J[rho]
    // of the lane's OWN block (C/D row = (reg & 3) + 8 (reg >> 2) + 4 h).
    Dct4JPlan plan4j;
    float lim4j[16];
    float lim_min4j;
    int dc_exact4j;
    // the same stage forming t + 1/2 (quot4j<true>): coefficient k is near a rounding tie when
    // fract(t + 1/2) <= dlo4h[k] or >= dhi4h[k] (2 x its tracked bound, rounded outward); the
    // non-structural coefficients share the loosest pair (dlo_max4h, dhi_min4h)
    float dlo4h[16], dhi4h[16];
    float dlo_max4h, dhi_min4h;
    int dc_exact4h;
    uint32_t mfma_w[64][4];
    // 4x4: P[16][16] then S, rq, qd of every coefficient, contiguous (the fix-up's LDS copy, staged
    // by DMA: 152 lanes x 16 bytes)
    double rows4[16 * 16 + 3 * 16];
    // the structural coefficients' rows P[k_s][*] (s = 0..2), then S, rq, qd of the three: the
    // fix-up's LDS copy, one contiguous block (3*NN + 9 doubles)
    double srow[3 * 64 + 9];
    // FP64 reference order (algo.cpp:309-331, Block.cpp:149-152)
    double S[64];   // C(u)*C(v)
    double qd[64];  // double(q[uv])
    double rq[64];  // 1/q when q is a power of two (exact), else 0 -> divide
    double c[64];   // c[u*N+i] (std::cos, algo.cpp:318-319)
    double P[64 * 64];  // P[uv*NN + ij] = c[u][i]*c[v][j]
    // inverse (algo.cpp:343-363): R[uv*NN + ij] = ((C(u)*C(v))*c[u][i])*c[v][j]
    double R[64 * 64];
};

// Division by a launch constant d (1 <= d < 2^31) for dividends n < 2^31, by a multiply-high:
// floor(n / d) = (mulhi(n, mul) + n) >> shr with shr = ceil(log2 d), mul = floor(2^32 (2^shr - d) / d) + 1
// (Granlund-Montgomery).  Built on the host (make_fastdiv), evaluated in scalar registers.
struct FastDiv {
    uint32_t d, mul, shr;
};
inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f{d, 0u, 0u};
    while ((1ull << f.shr) < d) f.shr++;
    f.mul = uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << f.shr) - d)) / d + 1);
    return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, uint32_t mul, uint32_t shr) {
    return (__umulhi(n, mul) + n) >> shr;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) { return fdiv(n, f.mul, f.shr); }

// One encode launch.  Tiles (workgroups) never straddle frames; a "chain" is the sequence of
// tiles whose bit offsets accumulate: the whole batch (concatenated stream) or one frame
// (independent images, segmented = 1).
struct EncArgs {
    const uint8_t* y;
    uint64_t stride, frame_pitch;
    int w, h, nframes;
    int bx, by;              // blocks per row / column
    int gpr;                 // thread groups per block row = ceil(bx / BPT)
    uint32_t gpr_magic;      // ceil(2^32 / gpr): exact floor(r / gpr) = mul_hi(r, magic) for r < gpr + 2^16
    int groups_per_frame;    // gpr * by
    int tiles_per_frame;     // ceil(groups_per_frame / encode_threads_per_tile())
    int ntiles;
    FastDiv div_frames, div_tpf, div_gpr;  // by nframes, tiles_per_frame, gpr
    int rle;
    int segmented;
    int vec_ok;              // rows may be read with 16-/8-byte loads
    uint32_t* out;           // 4-byte aligned, word w = stream bytes [4w, 4w+4)
    uint64_t out_pitch_words;
    uint64_t start_bit;
    const uint64_t* start_dev;  // non-null: the chain starts at *start_dev (device; overrides start_bit)
    uint64_t* st;            // [3*ntiles] tile chain granules (ie_common.hpp)
    unsigned long long* ticket;  // nullptr: tiles in blockIdx order; else an atomic ticket
    unsigned long long ticket_base;
    uint32_t tag;            // epoch tag 1..255
    uint64_t* frame_start;   // [nframes] absolute start bit of each frame's payload
    uint64_t* chain_end;     // [nchains] absolute end bit
    unsigned* err;           // [0] look-back timeouts (atomic, only ever on a timeout)
    uint32_t* wave_fix;      // [ntiles * kTPB/64] FP64 fix-up requests per wave (plain stores, statistics)
    const EncTables* tab;
    int16_t* coef;           // optional: quantised coefficients, natural order, [nframes*bx*by][N*N]
    int ablate;              // profiling only (IE_ABLATE): 1 no FP64, 2 no emission, 4 no look-back, 8 no store, 16 no DCT, 128 no pixel loads
    uint64_t* stamps;        // profiling only (IE_STAMPS): [tile][kStamps] s_memtime per phase, thread 0
    int deep_lb;             // the launch does not fill the chip: look-back windows issued at once
    int rec_bits;            // = tab->rec_bits (host copy): launch_encode sizes the LDS tile image from it
    int tri;                 // 4x4: every bl <= 11 (from rec_bits): records emitted three coefficients per field
    int img_words;           // set by launch_encode
    // optional (segmented launches): per-frame byte histograms [nframes][256] of the stream bytes
    // [0, ceil(end/8)) -- header included -- ADDED to by the launch (the Huffman pass's counts)
    uint32_t* hist;
};

constexpr int kStamps = 64;  // encode_kernel: [0, 16) by thread 0; encode4w_kernel: [4 waves][16] by each wave's lane 0
// chain-state words per tile (the host allocates; ie_common.hpp kGran must not exceed it)
constexpr int kStateWordsPerTile = 16;
// bpt: blocks per thread, encode_blocks_per_thread(n, ntiles at the default) for the launch
// returns the FP64-statistics words per tile the launched kernel writes (EncArgs::wave_fix)
int launch_encode(const EncArgs& a, int n, bool exact, hipStream_t s, int bpt);
int encode_blocks_per_thread(int n);  // the batch default (4x4: 4, 8x8: 1)
int encode_small_tiles();             // a launch of fewer tiles does not fill the chip (deep look-back)
void launch_word_scatter(const uint32_t* src, uint32_t* dst, uint64_t pitch_words, int n, hipStream_t s);  // horizontally adjacent blocks per lane (Geo<N>::BPT)
int encode_threads_per_tile();       // threads per encoder workgroup (= tile)

struct PackArgs {            // Huffman re-encode / bit copy: one variable-length code per byte
    const uint8_t* in;
    uint64_t n;              // input bytes
    const uint32_t* code;    // [256]
    const uint8_t* len;      // [256]
    int ntiles;
    uint32_t* out;
    uint64_t start_bit;
    uint64_t* st;
    unsigned long long* ticket;
    unsigned long long ticket_base;
    uint32_t tag;
    uint64_t* chain_end;
    unsigned* err;
    // batch mode (count > 0): string k owns the tiles t with t % count == k (position t / count,
    // tiles[k] of them), one chain each; its bytes at in + k*in_pitch (n[k] of them), its code
    // table at code/len + 256*k, its output at out + k*out_pitch_words from bit start[k], the words
    // before that from prefix + k*prefix_pitch_words (e.g. the Huffman dictionary), its end bit in
    // chain_end[k].  ntiles = count * max_k tiles[k].
    int count;
    const uint64_t* tiles;       // [count]
    const uint64_t* bn;          // [count]
    const uint64_t* bstart;      // [count]
    uint64_t in_pitch, out_pitch_words, prefix_pitch_words;
    const uint32_t* prefix;
    int maxlen;                  // longest code in the table(s): picks the tile shape
};
// input bytes per pack tile for codes of at most maxlen bits (ie_huffman.hip)
int pack_tile_bytes(int maxlen);
void launch_pack(const PackArgs& a, hipStream_t s);
// ie_bitcopy: n bytes to stream bit start_bit of out (no scan, no look-back; ie_huffman.hip)
void launch_bitshift(const uint8_t* in, uint64_t n, uint32_t* out, uint64_t start_bit, hipStream_t s);
// hist / first (each optional, count*256): cleared to 0 / ~0 by the same launch
void launch_ends_to_bytes(const uint64_t* ends, uint64_t cap, int count, uint64_t* n, hipStream_t s,
                          uint32_t* hist = nullptr, unsigned long long* first = nullptr);
// unresolved: device scratch, one word per string
void launch_hist(const uint8_t* in, uint64_t n, uint32_t* hist, unsigned long long* first, unsigned* unresolved,
                 hipStream_t s);
// count strings at in + k*pitch, n[k] (device array) bytes each, maxn >= every n[k]:
// hist/first + 256*k
// counts = false: hist already holds the counts (an encoder launch with EncArgs::hist); only the
// first occurrences are computed
// the counted pipeline's first-occurrence pass (ie_huffman.hip first_scan_counted_kernel)
void launch_first_counted(const uint8_t* in, uint64_t pitch, const uint64_t* ends, uint64_t cap, int count,
                          uint32_t* hist, uint64_t* n, unsigned long long* first, unsigned* unresolved, uint32_t* h_hist,
                          unsigned long long* h_first, unsigned* h_unres, hipStream_t s);
void launch_first_full_batch(const uint8_t* in, uint64_t pitch, const uint64_t* n, uint64_t maxn, int count,
                             const uint32_t* hist, unsigned long long* first, const unsigned* unresolved, hipStream_t s);
void launch_hist_batch(const uint8_t* in, uint64_t pitch, const uint64_t* n, uint64_t maxn, int count, uint32_t* hist,
                       unsigned long long* first, unsigned* unresolved, hipStream_t s, bool counts = true);

struct DecArgs {
    int nframes, bx, by, rle;
    int add_base;            // P-frames: pixel = clamp(pixel already in out + (IDCT + 128)) (Block.cpp:110-119)
    uint8_t* out;
    uint64_t stride, frame_pitch;
    const EncTables* tab;
};

// Exact record parse + decode (ie_decode.hip): per-chunk transfer tables over every entry offset
// [0, D), composed per group of G tables (levels until at most G remain), then the decode with a
// look-back over record counts; no host round trip.  D = the longest record (4 + 15*(N*N+1) bits).
#ifndef IE_REC_M
#define IE_REC_M 1  // measured on 4K streams: 1 beats 2, 4 and 8 (occupancy over lane packing)
#endif
// tables per composition group: measured on 4K frames and the reference's example images, 32
// beats 64 and 128 (more workgroups and 32-step chases instead of 128: 4K 4x4 noise 186 -> 175-180
// us, 400x400 88 -> 81 us per decode; 16 is no faster)
#ifndef IE_REC_G4
#define IE_REC_G4 32
#endif
#ifndef IE_REC_G8
#define IE_REC_G8 32
#endif
template <int N> struct RecGeom {
    static constexpr int D = 4 + 15 * (N * N + 1);
    static constexpr int G = (N == 4) ? IE_REC_G4 : IE_REC_G8;  // tables per group ([G][D] 16-bit exits in LDS)
    static constexpr int M = IE_REC_M;              // chunks per table wave
    static constexpr int HSB = (N == 4) ? 10 : 11;  // claim hash slots per chunk: 1 << HSB
    static constexpr int HS = 1 << HSB;
};
constexpr int kRecMaxLevels = 6;  // G^6 chunks per decode call
constexpr int kRecPosCap = 256;  // record positions kept per chunk (more: the decode walks again)
constexpr int kRecWPB = 4;       // chunk waves per block of the per-chunk passes
#ifndef IE_DEC_CHUNKS
#define IE_DEC_CHUNKS 2
#endif
constexpr int kDecChunks = IE_DEC_CHUNKS;  // chunks per decode wave (about 32 records each)
struct RecParseArgs {
    const uint32_t* words;  // stream as stored (big-endian bytes), zero-padded by >= 2 words
    uint64_t nbits, start_bit;
    uint32_t C;             // chunk bits (multiple of 32)
    int nchunks, rle;
    uint16_t* tab;          // [nchunks][D] transfer tables (then prefix maps), followed by the
                            // composites of every level
    uint16_t* lvl[kRecMaxLevels];  // set by the launcher: the table array of every level
    int levels;
    uint32_t* E;            // [<= G] entry offset of every top-level composite
    unsigned* ticket;       // [1]: the composition ticket, 0 before the launch (left 0)
    uint16_t* pos;          // [nchunks][kRecPosCap] record positions (relative to the chunk's word)
    uint32_t* cnt;          // [nchunks] records of every chunk
    uint32_t* lbase;        // [nchunks] records before every chunk within its count-pass workgroup
    uint32_t* wgsum;        // [count-pass workgroups] their record totals
    int seg;                // chunks per count-pass wave (rec_count_seg): a workgroup covers 4 * seg
    uint64_t* total;        // records on the true path
    uint64_t* end_out;      // end bit of the last block's record
    unsigned long long* stats;  // diagnostics (IE_DEC_STATS): walk steps; nullptr = off
    unsigned long long* wstamp; // diagnostics (IE_DEC_STAMPS): [table waves][8] phase times; nullptr = off
    int tm;                 // chunks per table wave (rec_table_geometry)
    int hbits;              // log2 of a table wave's claim slots
    // speculative parse (non-null): spec[k] = where the walk of chunk k from its first bit leaves
    // it (offset into chunk k+1) -- the entry of chunk k+1 in place of the composed tables; the
    // count pass, walking every chunk from its predecessor's spec exit, verifies each exit and sets
    // *fail on a mismatch (the decode pass then writes nothing and the host re-runs exactly)
    uint32_t* spec;
    unsigned* fail;         // device word, cleared by the speculative pass
    int warm;               // speculative walks start this many chunks early (IE_DEC_WARM, default 0)
    // device-chained span (ie_decode_gop): when non-null the first record is at
    // min(*dstart + start_add, nbits) -- an earlier launch's end bit -- and the span ends at most
    // `span` bits after it (start_bit is then unused); chunks past the span's end hold no record
    const uint64_t* dstart;
    uint64_t start_add, span;
};
// Table-wave geometry for chunks of C bits: chunks per wave (tm) and log2 claim slots (hbits).
void rec_table_geometry(uint32_t C, int n, int* tm, int* hbits);
int rec_group_chunks(int n);
int rec_entry_span(int n);
size_t rec_decode_lds(uint32_t C, int n);
int rec_count_seg(uint32_t C);
// Returns the number of composition levels (< 0: too many chunks).
int launch_rec_parse_decode(RecParseArgs a, const DecArgs& d, int n, hipStream_t s);
// the speculative form (a.spec, a.fail set): speculative walks, verifying count pass, decode
void launch_rec_spec_decode(const RecParseArgs& a, const DecArgs& d, int n, hipStream_t s);

// Huffman decode (ie_decode.hip): write = false runs the exact parse (per-chunk transfer tables
// over the 15 entry offsets, composed) + the counting walk + scan and leaves the symbol count in
// *total (device); write = true then emits the symbols into out.  tab: huffman_table_rows()
// 16-bit words; E: at least 256 words; ticket: 0 (left 0).  Returns the composition levels (< 0
// on error).
int huffman_decode_device(const uint32_t* W, uint64_t nbits, uint64_t start_bit, const uint16_t* lut,
                          uint64_t chunk_bits, uint64_t* entry, uint16_t* tab, uint32_t* E, unsigned* ticket,
                          uint32_t* count, uint64_t* base, unsigned* changed, uint64_t* total, uint8_t* out,
                          bool write, hipStream_t s, uint64_t out_cap = ~0ull);
size_t huffman_table_rows(uint64_t nbits, uint64_t start_bit, uint64_t chunk_bits);

// P-frame of a gop > 1 video (ie_pframe.hip): one launch sequence per frame, chained on the device.
struct PfArgs {
    const uint8_t* cur;      // the frame, rows cs apart
    uint64_t cs;
    const uint8_t* ref;      // the previous frame's buffer as the reference leaves it, rows rs apart
    uint64_t rs;
    uint8_t* rec;            // [h][w]: this frame's buffer after the P-frame pass (the next reference)
    int w, h, mbx, mby, bx;  // macroblocks per row / column (floor), microblocks per row
    int rle, merange, mv_bits;
    const EncTables* tab;
    int16_t* coef;           // [bx*by][16] quantised prediction error (natural order), 4x4 only
    uint32_t* bits;          // [bx*by] record bits, 0 = no record
    uint32_t* out;           // stream words (zero from the frame's first bit on)
    const uint64_t* start;   // device: the frame's first bit
    uint64_t* end;           // device: its end bit
    uint64_t* st;            // record tiles' chain state (look-back scan); nullptr = separate scan launches
    uint32_t tag;            // the state's epoch
    unsigned* err;           // [0]: look-back spin timeouts
};
void launch_pframe(const PfArgs& a, int n, uint64_t* tile_scratch, hipStream_t s);
// P-frame decode, first half (Block.cpp:481-496): every macroblock's motion vector read from the
// stream words (big-endian bytes) at start_bit, the previous decoded frame's block at the clamped
// vector copied into place
// gop decode: pos[0] = start, pos[1..n] = ~0 (no end yet), tot[0..n) = 0
void launch_gop_init(uint64_t* pos, uint64_t* tot, int n, uint64_t start, hipStream_t s);
// dstart non-null: the vectors start at *dstart (device, an earlier launch's end bit) in place of
// start_bit; a macroblock whose vector lies past nbits copies nothing (the caller reports it)
void launch_pframe_mvcopy(const uint8_t* stream, uint64_t start_bit, const uint64_t* dstart, uint64_t nbits, int mv_bits,
                          const uint8_t* ref, uint64_t rs, uint8_t* out, uint64_t os, int w, int h, hipStream_t s);
int pframe_tiles(int nb);    // tile_scratch entries

}  // namespace ie
