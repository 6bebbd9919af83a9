// imageencoder_amd/csrc/ie_capi.cpp -- the extern "C" boundary (include/ie_hip.h): context,
// quantisation tables, buffer staging and kernel launches.  Host code; compiled with hipcc.
#include "ie_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ie_device.h"

struct ie_pipe;  // streamed host path (below)

struct ie_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    std::string err;

    int n = 0;
    uint16_t q[64] = {};
    ie::EncTables* h_tab = nullptr;
    ie::EncTables* d_tab = nullptr;

    // decoupled look-back state
    uint64_t* d_state = nullptr;  // [kStateWordsPerTile * cap_tiles] tile chain granules (ie_common.hpp)
    size_t cap_tiles = 0;
    uint32_t tag = 0;
    unsigned long long* d_ticket = nullptr;
    unsigned long long ticket_base = 0;

    uint64_t* d_frame_start = nullptr;  // [cap_frames]
    uint64_t* d_chain_end = nullptr;    // [cap_frames]
    size_t cap_frames = 0;
    unsigned* d_err = nullptr;          // [0] look-back timeouts (cumulative)
    uint32_t* d_wave_fix = nullptr;     // [cap_tiles * waves per tile] fix-up requests of the last launch
    int last_fix_words = 0;
    unsigned err_seen[66] = {};         // counter values at the previous read
    bool use_ticket = false;            // order tiles with an atomic ticket (after a timeout)
    hipEvent_t stage_ev[4] = {};        // timing events around the last batched histogram [0,1] / pack [2,3]
    bool stage_rec[2] = {false, false};
    bool stage_timing = false;          // ie_set_stage_timing
    int fake_timeouts = 0;              // debug (IE_FAKE_TIMEOUTS): report this many look-back timeouts
    bool fake_fired = false;            // a faked timeout was reported (the redo paths dirty the output first)
    // Asynchronous launches (no read-back) since the last error read: a look-back timeout found
    // at the next read is charged to them (their output is invalid), never silently retried away.
    unsigned async_pending = 0;
    const char* async_what = nullptr;

    // staging for host-resident inputs / outputs
    uint8_t* d_in = nullptr;
    size_t cap_in = 0;
    uint8_t* d_out = nullptr;
    size_t cap_out = 0;
    uint8_t* d_scratch = nullptr;   // quantize-only stream sink
    size_t cap_scratch = 0;
    int16_t* d_coef = nullptr;
    size_t cap_coef = 0;

    uint64_t last_fallbacks = 0;

    // Huffman tables / histogram
    uint32_t* d_code = nullptr;        // [256] codes, then [256/4] packed lengths (one block)
    uint32_t* h_code = nullptr;        // pinned mirror
    uint32_t* d_hist = nullptr;        // [256]
    // batched Huffman: device + pinned staging (hist/first of every string, then the pack tables)
    uint8_t* d_batch = nullptr;
    size_t cap_batch = 0;
    uint8_t* h_batch = nullptr;
    size_t cap_hbatch = 0;
    // pipelined batches: two pinned slots for the histogram read-back and two for the pack tables,
    // each guarded by an event (no stream-wide synchronisation between batches)
    uint8_t* h_hist[2] = {};
    size_t cap_hhist[2] = {};
    hipEvent_t ev_hist[2] = {};
    int hist_count[2] = {};
    uint8_t* h_pack[2] = {};
    size_t cap_hpack[2] = {};
    hipEvent_t ev_pack[2] = {};    // the table copy out of pinned slot i (on tab_stream)
    bool pack_recorded[2] = {};
    uint8_t* d_pack[2] = {};       // device table slots
    size_t cap_dpack[2] = {};
    hipEvent_t ev_packed[2] = {};  // the pack (and prefix copies) that read device slot i
    bool packed_recorded[2] = {};
    hipStream_t tab_stream = nullptr;
    int pack_slot = 0;
    int fused_count = 0;  // > 0: the last encode (ie_encode_images_counted) left this many histograms in d_chist
    // the counted pipeline: the encoder's histograms (cleared by the first-occurrence pass that reads
    // them: chist_zero_rows), and per pinned slot the device n / first / unresolved the rare first_full
    // pass of ie_huffman_hist_batch_wait needs, with the batch it reads
    uint32_t* d_chist = nullptr;
    size_t cap_chist = 0;  // (words)
    // leading 256-word rows of d_chist known to be zero (the counted encode skips its memset when
    // its rows lie within them), and the rows that will be zero once the fused pass has read -- and
    // cleared -- the last counted encode's rows
    size_t chist_zero_rows = 0, chist_clean_after = 0;
    bool hist_skip_zero = false;  // one shot: encode() skips its histogram memset (set by the counted encode)
    uint8_t* d_cslot[2] = {};
    size_t cap_cslot[2] = {};
    bool hist_fused[2] = {};
    const uint8_t* hist_in[2] = {};
    size_t hist_pitch[2] = {};
    // decoder scratch
    uint8_t* d_dec = nullptr;          // staged stream + padding
    size_t cap_dec = 0;
    uint64_t* d_walk = nullptr;        // entry, exA, exB, base: 4 x cap_chunks
    size_t cap_walk = 0;
    uint32_t* d_count = nullptr;
    size_t cap_count = 0;
    uint16_t* d_rtab = nullptr;        // record parse: chunk transfer tables and the composites of every level
    size_t cap_rtab = 0;
    uint16_t* d_rpos = nullptr;        // record parse: record positions per chunk
    size_t cap_rpos = 0;
    uint64_t* d_misc = nullptr;        // [0] end bit, [1] changed / invalid flags or decode tickets, [2] symbol /
                                       // record count, [3] histogram ticket
    uint64_t* h_decres = nullptr;      // record decode results, pinned host memory the device writes
    uint64_t* d_decres = nullptr;      // directly ([0] end bit, [1] record total): no read-back copy
    uint16_t* d_hlut = nullptr;        // Huffman decode prefix table (32768 entries)
    size_t cap_hlut = 0;
    uint8_t* d_hout = nullptr;         // Huffman decode output staging (host destinations)
    size_t cap_hout = 0;
    uint8_t* d_pix = nullptr;
    size_t cap_pix = 0;
    int last_chunks = 0;               // chunks of the last record decode
    int last_groups = 0;               // and their groups
    int last_spec = 0;                 // 1: the last record decode was the speculative parse
    int spec_parse = 0;                // ie_set_exact_parse(ctx, 0): speculative record parse first
    int spec_warm = 0;                 // ie_set_spec_warm(ctx, w): w warm-up chunks (<= 8)
    unsigned long long* d_first = nullptr;  // [256]
    ie_pipe* pipe = nullptr;           // streamed host path of image batches (created on first use)
    // P-frame videos (ie_encode_gop): reconstructed frames (two, alternating), the prediction
    // error's coefficients and record lengths, the scan's tile sums, the frames' bit positions
    uint8_t* d_gop_rec = nullptr;
    size_t cap_gop_rec = 0;
    int16_t* d_gop_coef = nullptr;
    size_t cap_gop_coef = 0;
    uint32_t* d_gop_bits = nullptr;
    size_t cap_gop_bits = 0;
    uint64_t* d_gop_tile = nullptr;
    size_t cap_gop_tile = 0;
    uint64_t* d_gop_pos = nullptr;
    size_t cap_gop_pos = 0;
};

namespace {

constexpr int kErrWords = 66;

int fail(ie_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPCHK(ctx, expr)                                                                       \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail(ctx, IE_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
    } while (0)

bool is_device_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeDevice;
}

template <class T>
int ensure(ie_ctx* c, T*& p, size_t& cap, size_t need_elems) {
    if (cap >= need_elems && p) return IE_OK;
    if (p) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(p));
        p = nullptr;
    }
    size_t n = std::max(need_elems, cap + cap / 2);
    HIPCHK(c, hipMalloc(&p, n * sizeof(T)));
    cap = n;
    return IE_OK;
}


// pinned host staging (the stream is synchronised before an existing buffer is replaced)
int ensure_pinned(ie_ctx* c, uint8_t*& p, size_t& cap, size_t need) {
    if (cap >= need && p) return IE_OK;
    if (p) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipHostFree(p));
        p = nullptr;
    }
    const size_t n = std::max(need, cap + cap / 2);
    HIPCHK(c, hipHostMalloc(&p, n));
    cap = n;
    return IE_OK;
}

// ---- rigorous error bound of the FP32 fast path -----------------------------------------
// Trk = an exact real affine form c0 + sum_k a_k x_k of the block's RAW pixels x_k in [0, 255]
// plus a bound E on the FP32 rounding error accumulated so far.  TrkOp mirrors every operation
// of the quotient transforms in ie_dct.h: the real coefficients follow the FP32 constants
// exactly; each rounded operation adds u*(|result| + E) with |result| <= |c0 + 127.5 sum a| +
// 127.5 sum|a| (the box bound).  Results that are integers below 2^24 are exact (integ), and so
// is a product of an exact value by a power of two.
struct Trk {
    double a[64];
    double c0;
    double E;
    bool integ;
};

struct TrkOp {
    int nn;
    static constexpr double u = 1.0 / 16777216.0;  // 2^-24
    double mag(const Trk& t) const {
        double s = 0, m = 0;
        for (int k = 0; k < nn; k++) {
            s += t.a[k];
            m += std::fabs(t.a[k]);
        }
        return std::fabs(t.c0 + 127.5 * s) + 127.5 * m;
    }
    static bool is_int(double c) { return c == std::rint(c); }
    static bool is_pow2(double c) {
        int e = 0;
        return c != 0.0 && std::fabs(std::frexp(c, &e)) == 0.5;
    }
    Trk lin(const Trk& x, double cx, const Trk* y, double cy, double cadd, double Ein, bool integ, bool exact) const {
        Trk r;
        for (int k = 0; k < nn; k++) r.a[k] = cx * x.a[k] + (y ? cy * y->a[k] : 0.0);
        for (int k = nn; k < 64; k++) r.a[k] = 0.0;
        r.c0 = cx * x.c0 + (y ? cy * y->c0 : 0.0) + cadd;
        const double m = mag(r);
        r.integ = integ && m < 16777216.0;
        r.E = Ein + ((r.integ || exact) ? 0.0 : u * (m + Ein));
        return r;
    }
    Trk add(const Trk& x, const Trk& y) const { return lin(x, 1, &y, 1, 0, x.E + y.E, x.integ && y.integ, false); }
    Trk sub(const Trk& x, const Trk& y) const { return lin(x, 1, &y, -1, 0, x.E + y.E, x.integ && y.integ, false); }
    Trk mul(const Trk& x, float c) const {
        const bool exact = x.E == 0.0 && is_pow2(double(c));
        return lin(x, double(c), nullptr, 0, 0, std::fabs(double(c)) * x.E, x.integ && is_int(c), exact);
    }
    Trk fma(const Trk& x, float c, const Trk& y) const {
        return lin(x, double(c), &y, 1, 0, std::fabs(double(c)) * x.E + y.E, x.integ && y.integ && is_int(c), false);
    }
    Trk fms(const Trk& x, float c, const Trk& y) const {
        return lin(x, double(c), &y, -1, 0, std::fabs(double(c)) * x.E + y.E, x.integ && y.integ && is_int(c), false);
    }
    Trk addc(const Trk& x, float c) const { return lin(x, 1, nullptr, 0, double(c), x.E, x.integ && is_int(c), false); }
    // x * c + k (one rounding, constant k)
    Trk fmac(const Trk& x, float c, float k) const {
        return lin(x, double(c), nullptr, 0, double(k), std::fabs(double(c)) * x.E, x.integ && is_int(c) && is_int(k), false);
    }
};

inline double Cf(int i) { return i == 0 ? 0.5 : M_SQRT1_2; }  // algo.cpp:294-297

// Build the per-matrix tables.  The cos values are the reference's own expression evaluated with
// the host libm (algo.cpp:312,318-319); P, S and R are the double products it forms.  For the
// FP32 path, the tracked run of the kernel's quotient transform (quot4 / quot8 in ie_dct.h) on
// raw pixels gives per coefficient k the real affine map the FP32 code implements and its
// rounding bound E_k.  With alpha*_k the reference's map (S*P/q on centred pixels) the FP32
// quotient is within
//     bound_k = E_k + 128 * sum|alpha_k - alpha*_k| + |value of our map at x = 128| + 1e-9
// of the reference's FP64 quotient (1e-9 covers the reference's own FP64 rounding, <= 1e-10);
// |t32 - rint(t32)| >= 0.5 - 2*bound_k flags a possible tie.  Returns false if alpha deviates
// from alpha* beyond FP32 constant rounding (a transform bug).
bool build_tables(int n, const uint16_t* q, ie::EncTables* T) {
    const int nn = n * n;
    std::memset(T, 0, sizeof(*T));
    const double factor = M_PI_2 / double(n);
    for (int u = 0; u < n; u++)
        for (int i = 0; i < n; i++) T->c[u * n + i] = std::cos(double(2.0 * i + 1.0) * double(u) * factor);
    std::vector<double> sq(nn);
    for (int u = 0; u < n; u++)
        for (int v = 0; v < n; v++) {
            const int k = u * n + v;
            T->S[k] = Cf(u) * Cf(v);
            T->qd[k] = double(q[k]);
            int e2 = 0;
            T->rq[k] = (std::frexp(double(q[k]), &e2) == 0.5) ? 1.0 / double(q[k]) : 0.0;
            sq[k] = T->S[k] / T->qd[k];
            T->g[k] = float(sq[k]);
            for (int i = 0; i < n; i++)
                for (int j = 0; j < n; j++) {
                    T->P[k * nn + i * n + j] = T->c[u * n + i] * T->c[v * n + j];
                    T->R[k * nn + i * n + j] = Cf(u) * Cf(v) * T->c[u * n + i] * T->c[v * n + j];
                }
        }
    for (int k = 0; k < nn; k++) T->cf[k] = float(T->c[k]);
    for (int k = 0; k <= 8; k++) T->dct.K[k] = float(std::cos(double(k) * M_PI / 16.0));
    // 4x4 plan: K2 = cos(pi/8), K4 = cos(pi/4), K6 = cos(3pi/8); row outputs R1, R3 carry 1/K2
    {
        const double K2 = std::cos(M_PI / 8.0), K4 = std::cos(M_PI / 4.0), K6 = std::cos(3.0 * M_PI / 8.0);
        T->plan4.r = float(K6 / K2);
        if (n == 4) {
            for (int v = 0; v < 4; v++) {
                const double Kv = (v == 0) ? 1.0 : (v == 2) ? K4 : K2;
                float* G = T->plan4.col[v];
                G[0] = float(Kv * sq[0 * 4 + v]);
                G[1] = float(K4 * Kv * sq[2 * 4 + v]);
                G[2] = float(K2 * Kv * sq[1 * 4 + v]);
                G[3] = float(K6 * Kv * sq[1 * 4 + v]);
                G[4] = float(K6 * Kv * sq[3 * 4 + v]);
                G[5] = float(-K2 * Kv * sq[3 * 4 + v]);
            }
        }
    }

    // 4x4 matrix-pipe plan (quot4j): G[k][m] = S/q * the row and column basis factors of term m
    if (n == 4) {
        const double K2 = std::cos(M_PI / 8.0), K4 = std::cos(M_PI / 4.0), K6 = std::cos(3.0 * M_PI / 8.0);
        auto f = [&](int u, int m) -> double {  // factor of basis dct4j_b(u, m) in 1-D row u
            if (u == 0) return 1.0;
            if (u == 2) return K4;
            if (u == 1) return m == 0 ? K2 : K6;
            return m == 0 ? K6 : -K2;
        };
        for (int u = 0; u < 4; u++)
            for (int v = 0; v < 4; v++) {
                int m = 0;
                for (int a = 0; a < ie::dct4j_nb(u); a++)
                    for (int bb = 0; bb < ie::dct4j_nb(v); bb++) T->plan4j.G[4 * u + v][m++] = float(sq[4 * u + v] * f(u, a) * f(v, bb));
            }
        static const int B[4][4] = {{1, 1, 1, 1}, {1, -1, -1, 1}, {1, 0, 0, -1}, {0, 1, -1, 0}};
        for (int l = 0; l < 64; l++) {
            const int r = l & 31, h = l >> 5, rho = (r & 3) + 4 * (r >> 3), hr = (r >> 2) & 1;
            for (int w = 0; w < 4; w++) T->mfma_w[l][w] = 0u;
            if (h != hr) continue;
            for (int j = 0; j < 16; j++) {
                const int c = B[rho >> 2][j >> 2] * B[rho & 3][j & 3];
                T->mfma_w[l][j >> 2] |= uint32_t(uint8_t(int8_t(c))) << (8 * (j & 3));
            }
        }
    }

    // tracked run of the kernel's transform on raw pixels
    std::vector<Trk> b(nn);
    for (int k = 0; k < nn; k++) {
        for (int m = 0; m < 64; m++) b[k].a[m] = (m == k) ? 1.0 : 0.0;
        b[k].c0 = 0.0;
        b[k].E = 0.0;
        b[k].integ = true;
    }
    TrkOp op{nn};
    // the matrix-pipe form: the sixteen J exact (pixels - 128), then quot4j's FP32 stage
    std::vector<Trk> bj(nn), bh(nn);
    if (n == 4) {
        std::vector<Trk> xs(b), J(nn);
        for (int k = 0; k < nn; k++) xs[k].c0 = -128.0;
        ie::dct4j_ints(xs.data(), J.data(), op);
        for (int k = 0; k < nn; k++)
            if (!J[k].integ || J[k].E != 0.0) return false;  // the integer stage must be exact
        ie::quot4j(J.data(), bj.data(), T->plan4j, op);
        ie::quot4j<true>(J.data(), bh.data(), T->plan4j, op);
    }
    if (n == 4) ie::quot4(b.data(), T->plan4, op);
    else ie::quot8(b.data(), T->dct, T->g, op);
    // Largest record: |Q_k| <= 128 * sum_ij |S_k P_k[ij]| / q_k (|x| <= 128), so bl <= the widest
    // bits_needed over k (utils.hpp:226-243; int16 caps it at 16) and >= ffs(N*N) (the L field);
    // an RLE record is 4 + bl * (1 + N*N) bits at most (Block.cpp:372-413).
    {
        int bl = 32 - __builtin_clz(unsigned(nn));
        for (int k = 0; k < nn; k++) {
            double m = 0.0;
            for (int ij = 0; ij < nn; ij++) m += std::fabs(T->S[k] * T->P[k * nn + ij]);
            const double qmax = std::ceil(128.0 * m / T->qd[k]) + 1.0;
            const int b = (qmax >= 32768.0) ? 16 : std::min(16, (32 - __builtin_clz(unsigned(qmax))) + 1);
            bl = std::max(bl, b);
        }
        T->rec_bits = 4 + bl * (1 + nn);
    }
    if (n == 4) {  // every coefficient's FP64 row and its S, rq, qd, contiguous (encode4p_kernel's DMA)
        for (int i = 0; i < nn * nn; i++) T->rows4[i] = T->P[i];
        for (int k = 0; k < nn; k++) {
            T->rows4[nn * nn + k] = T->S[k];
            T->rows4[nn * nn + nn + k] = T->rq[k];
            T->rows4[nn * nn + 2 * nn + k] = T->qd[k];
        }
    }
    {  // the fix-up's structural rows, contiguous (encode_kernel copies them to LDS)
        const int h = n / 2, ks[3] = {h, h * n, h * n + h};
        for (int si = 0; si < 3; si++) {
            for (int ij = 0; ij < nn; ij++) T->srow[si * nn + ij] = T->P[ks[si] * nn + ij];
            T->srow[3 * nn + si] = T->S[ks[si]];
            T->srow[3 * nn + 3 + si] = T->rq[ks[si]];
            T->srow[3 * nn + 6 + si] = T->qd[ks[si]];
        }
    }
    bool ok = true;
    // per coefficient of one tracked transform: its tie limit (lim), the bound (thr), whether the
    // DC quotient is exact, and the loosest limit of the non-structural coefficients (lim_min)
    auto limits = [&](const std::vector<Trk>& tv, float* lim, float* thr, float* lim_min, int* dc_exact, float g0) {
        *dc_exact = 0;
        *lim_min = 0.5f;
        for (int k = 0; k < nn; k++) {
            const Trk& t = tv[k];
            double dev = 0.0, amax = 0.0, sa = 0.0;
            for (int m = 0; m < nn; m++) {
                const double ref = sq[k] * T->P[k * nn + m];
                dev += std::fabs(t.a[m] - ref);
                amax = std::max(amax, std::fabs(ref));
                sa += t.a[m];
            }
            if (dev > 1e-5 * (amax + 1e-30) * nn) ok = false;  // FP32 constants differ by ~1e-7 relative
            const double bound = t.E + 128.0 * dev + std::fabs(t.c0 + 128.0 * sa) + 1e-9;
            // coefficient 0: an integer sum (minus 128*N*N) scaled by a power of two is exact in FP32,
            // and the reference computes it exactly too (c[0][*] = 1, C(0)^2 = 1/4, q a power of two)
            if (k == 0 && t.E == 0.0 && double(g0) == sq[0] && TrkOp::is_pow2(sq[0])) {
                if (thr) thr[k] = -1.0f;
                lim[k] = 1.0f;  // never flagged
                *dc_exact = 1;
            } else {
                if (thr) thr[k] = float(2.0 * bound);
                lim[k] = float(0.5 - 2.0 * bound);
                // the structural coefficients (0,N/2), (N/2,0), (N/2,N/2) are flagged one by one
                const int h = n / 2;
                const bool structural = (k == h) || (k == h * n) || (k == h * n + h);
                if (!structural) *lim_min = std::min(*lim_min, lim[k]);
            }
        }
    };
    limits(b, T->lim, T->thr, &T->lim_min, &T->dc_exact, T->g[0]);
    if (n == 4) limits(bj, T->lim4j, nullptr, &T->lim_min4j, &T->dc_exact4j, T->plan4j.G[0][0]);
    if (n == 4) {  // t + 1/2: the tie test on fract(t + 1/2), limits rounded outward
        T->dc_exact4h = 0;
        T->dlo_max4h = 0.0f;
        T->dhi_min4h = 1.0f;
        for (int k = 0; k < nn; k++) {
            const Trk& t = bh[k];
            double dev = 0.0, sa = 0.0;
            for (int m = 0; m < nn; m++) {
                dev += std::fabs(t.a[m] - sq[k] * T->P[k * nn + m]);
                sa += t.a[m];
            }
            // (the map's value at x = 128 is the 1/2 itself)
            const double bound = t.E + 128.0 * dev + std::fabs(t.c0 + 128.0 * sa - 0.5) + 1e-9;
            // DC: exact in quot4j (dc_exact4j) stays exact with the 1/2 added (J0 * G (a power of two)
            // has at most 12 significant bits; the tracked fmac does not see that)
            if (k == 0 && T->dc_exact4j) {
                T->dlo4h[k] = -1.0f;  // never flagged
                T->dhi4h[k] = 2.0f;
                T->dc_exact4h = 1;
                continue;
            }
            const double d = 2.0 * bound;
            T->dlo4h[k] = std::nextafter(float(d), 1.0f);          // >= d
            T->dhi4h[k] = std::nextafter(float(1.0 - d), 0.0f);    // <= 1 - d
            const int h = n / 2;
            const bool structural = (k == h) || (k == h * n) || (k == h * n + h);
            if (!structural) {
                T->dlo_max4h = std::max(T->dlo_max4h, T->dlo4h[k]);
                T->dhi_min4h = std::min(T->dhi_min4h, T->dhi4h[k]);
            }
        }
    }
    return ok;
}

int prepare_state(ie_ctx* c, int ntiles, int nframes) {
    if (size_t(ntiles) > c->cap_tiles) {
        if (c->d_state) {
            HIPCHK(c, hipStreamSynchronize(c->stream));
            HIPCHK(c, hipFree(c->d_state));
        }
        const size_t cap = std::max<size_t>(ntiles, c->cap_tiles * 2);
        HIPCHK(c, hipMalloc(&c->d_state, size_t(ie::kStateWordsPerTile) * cap * sizeof(uint64_t)));
        if (c->d_wave_fix) HIPCHK(c, hipFree(c->d_wave_fix));
        HIPCHK(c, hipMalloc(&c->d_wave_fix, cap * 16 * sizeof(uint32_t)));
        HIPCHK(c, hipMemsetAsync(c->d_state, 0, size_t(ie::kStateWordsPerTile) * cap * sizeof(uint64_t), c->stream));
        c->cap_tiles = cap;
        c->tag = 0;
    }
    c->tag++;
    if (c->tag > 255) {
        HIPCHK(c, hipMemsetAsync(c->d_state, 0, size_t(ie::kStateWordsPerTile) * c->cap_tiles * sizeof(uint64_t), c->stream));
        c->tag = 1;
    }
    if (size_t(nframes) > c->cap_frames) {
        if (c->d_frame_start) {
            HIPCHK(c, hipStreamSynchronize(c->stream));
            HIPCHK(c, hipFree(c->d_frame_start));
            HIPCHK(c, hipFree(c->d_chain_end));
        }
        const size_t cap = std::max<size_t>(nframes, 64);
        HIPCHK(c, hipMalloc(&c->d_frame_start, cap * sizeof(uint64_t)));
        HIPCHK(c, hipMalloc(&c->d_chain_end, cap * sizeof(uint64_t)));
        c->cap_frames = cap;
    }
    return IE_OK;
}

// [0] look-back timeouts; sum of [2..65] = FP64 re-evaluations.  Synchronises the stream.
// The device counters only ever grow (no per-launch reset kernel in the launch path); a read
// reports the increments since the previous read.
// Timing marks around the batched Huffman stages (ie_last_stage_ms): event i on the context's stream.
int stage_mark(ie_ctx* c, int i) {
    if (!c->stage_timing) return IE_OK;  // (ie_set_stage_timing: off by default)
    if (!c->stage_ev[i]) HIPCHK(c, hipEventCreate(&c->stage_ev[i]));
    HIPCHK(c, hipEventRecord(c->stage_ev[i], c->stream));
    if (i & 1) c->stage_rec[i >> 1] = true;
    return IE_OK;
}

int read_errors(ie_ctx* c, unsigned* timeouts, uint64_t* fallbacks) {
    unsigned e[kErrWords];
    HIPCHK(c, hipMemcpyAsync(e, c->d_err, sizeof(e), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    uint64_t f = 0;
    if (fallbacks && c->last_fix_words) {
        std::vector<uint32_t> w(size_t(c->last_fix_words));
        HIPCHK(c, hipMemcpy(w.data(), c->d_wave_fix, w.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
        for (uint32_t v : w) f += v;
    }
    unsigned t = e[0] - c->err_seen[0];
    if (c->fake_timeouts > 0 && timeouts && !c->async_pending) {  // debug: IE_FAKE_TIMEOUTS
        c->fake_timeouts--;
        c->fake_fired = true;
        t++;
    }
    if (timeouts) *timeouts = t;
    if (fallbacks) *fallbacks = f;
    std::memcpy(c->err_seen, e, sizeof(e));
    const unsigned pending = c->async_pending;
    const char* what = c->async_what;
    c->async_pending = 0;
    c->async_what = nullptr;
    if (t && pending) {
        // a launch that returned without a read-back timed out: its output is invalid and there is
        // nothing to re-run here -- fail loudly (later launches order their tiles by ticket)
        c->use_ticket = true;
        return fail(c, IE_EDEVICE, std::string("tile look-back timed out in an earlier asynchronous ") +
                                       (what ? what : "launch") + " (" + std::to_string(pending) +
                                       " unchecked launch(es)); its output is invalid");
    }
    return IE_OK;
}

// An asynchronous launch returned without reading the error counters: the next read (ie_sync or
// any synchronous call) checks it.
void note_async(ie_ctx* c, const char* what) {
    c->async_pending++;
    c->async_what = what;
}

struct Geometry {
    int bx, by, gpr, gpf, tpf, ntiles;
};

Geometry geometry(int w, int h, int n, int nframes, int bpt = 0) {
    Geometry g;
    if (!bpt) bpt = ie::encode_blocks_per_thread(n);
    g.bx = w / n;
    g.by = h / n;
    g.gpr = (g.bx + bpt - 1) / bpt;
    g.gpf = g.gpr * g.by;
    const int tpt = ie::encode_threads_per_tile();  // groups per tile
    g.tpf = (g.gpf + tpt - 1) / tpt;
    g.ntiles = g.tpf * nframes;
    return g;
}

int check_dims(ie_ctx* c, int w, int h, int nframes) {
    if (!c->n) return fail(c, IE_ENOQUANT, "ie_set_quant has not been called");
    if (w <= 0 || h <= 0 || w % c->n || h % c->n)
        return fail(c, IE_EINVAL, "width/height must be positive multiples of the block size");
    if (w > 32767 || h > 32767) return fail(c, IE_EINVAL, "width/height exceed the 15-bit header fields");
    if (nframes <= 0) return fail(c, IE_EINVAL, "nframes must be > 0");
    return IE_OK;
}

size_t bound_bits_per_block(int n) { return 4 + 16 * size_t(n * n + 1); }

// One encode launch over device-resident frames (no staging, no synchronisation): the EncArgs
// of ie_device.h, the chain state's epoch and the launch.  start_dev (optional) makes the chain
// start at a device-resident bit position (the previous launch's chain end, ie_vstream_*);
// chain_end (optional) receives the chain end(s) instead of the context's d_chain_end.
struct Launch {
    const uint8_t* dy = nullptr;
    int w = 0, h = 0;
    size_t stride = 0, frame_pitch = 0;
    int nframes = 0, use_rle = 1, mode = IE_MODE_FAST;
    uint32_t* dout = nullptr;  // word 0 = stream bytes [0, 4) (may point before the allocation)
    size_t out_pitch = 0;      // segmented: bytes between images
    uint64_t start_bit = 0;
    const uint64_t* start_dev = nullptr;
    uint64_t* chain_end = nullptr;
    int segmented = 0;
    int16_t* coef = nullptr;
    uint32_t* hist = nullptr;
};

int launch_chain(ie_ctx* c, const Launch& L) {
    const int bpt = ie::encode_blocks_per_thread(c->n);
    const Geometry g = geometry(L.w, L.h, c->n, L.nframes, bpt);
    // a launch too small to fill the chip: its tiles reach the look-back together (deep windows)
    const bool small = g.ntiles < ie::encode_small_tiles();
    const bool vec_ok = (reinterpret_cast<uintptr_t>(L.dy) % size_t(bpt * c->n) == 0) &&
                        (L.stride % (bpt * c->n) == 0) && (L.nframes == 1 || L.frame_pitch % (bpt * c->n) == 0);
    int r;
    ie::EncArgs a{};
    a.y = L.dy;
    a.stride = L.stride;
    a.frame_pitch = L.frame_pitch;
    a.w = L.w;
    a.h = L.h;
    a.nframes = L.nframes;
    a.bx = g.bx;
    a.by = g.by;
    a.gpr = g.gpr;
    a.gpr_magic = (g.gpr > 1) ? uint32_t(((uint64_t(1) << 32) + uint64_t(g.gpr) - 1) / uint64_t(g.gpr)) : 0u;
    a.groups_per_frame = g.gpf;
    a.tiles_per_frame = g.tpf;
    a.div_frames = ie::make_fastdiv(uint32_t(L.nframes));
    a.div_tpf = ie::make_fastdiv(uint32_t(g.tpf));
    a.div_gpr = ie::make_fastdiv(uint32_t(g.gpr));
    a.ntiles = g.ntiles;
    a.rle = L.use_rle ? 1 : 0;
    a.segmented = L.segmented;
    a.vec_ok = vec_ok ? 1 : 0;
    a.out = L.dout;
    a.out_pitch_words = L.segmented ? L.out_pitch / 4 : 0;
    a.start_bit = L.start_bit;
    a.start_dev = L.start_dev;
    a.tab = c->d_tab;
    a.rec_bits = c->h_tab->rec_bits;
    a.tri = (c->n == 4 && (a.rec_bits - 4) / 17 <= 10) ? 1 : 0;  // bl_max = (rec_bits - 4) / (1 + N*N); 3 bl <= 30
    a.coef = L.coef;
    a.hist = L.hist;
#ifndef IE_PROFILE
#define IE_PROFILE 0
#endif
#ifndef IE_ABLATE_FORCE
#define IE_ABLATE_FORCE 0
#endif
    // Profiling knobs exist only in IE_PROFILE builds (tools/variants.sh): the product library
    // never reads IE_ABLATE / IE_STAMPS, so no environment variable can change its output.
#if IE_PROFILE
    static const int ablate = getenv("IE_ABLATE") ? atoi(getenv("IE_ABLATE")) : 0;
    static const char* stamp_file = getenv("IE_STAMPS");  // per-tile phase stamps
#else
    constexpr int ablate = 0;
    const char* stamp_file = nullptr;
#endif
    a.ablate = ablate | IE_ABLATE_FORCE;  // IE_ABLATE_FORCE: A/B builds of an ablation
    if ((r = prepare_state(c, g.ntiles, L.nframes))) return r;
    a.st = c->d_state;
    a.ticket = c->use_ticket ? c->d_ticket : nullptr;
    a.ticket_base = c->ticket_base;
    a.tag = c->tag;
    a.frame_start = c->d_frame_start;
    a.chain_end = L.chain_end ? L.chain_end : c->d_chain_end;
    a.err = c->d_err;
    a.wave_fix = c->d_wave_fix;
    c->last_fix_words = 0;  // (set after the launch: its kernel's waves per tile)
    if (L.hist && !c->hist_skip_zero) HIPCHK(c, hipMemsetAsync(L.hist, 0, size_t(L.nframes) * 256 * sizeof(uint32_t), c->stream));
    c->hist_skip_zero = false;  // (a re-launch clears)
    uint64_t* d_stamps = nullptr;
    if (stamp_file) {
        HIPCHK(c, hipMalloc(&d_stamps, size_t(g.ntiles) * ie::kStamps * sizeof(uint64_t)));
        HIPCHK(c, hipMemsetAsync(d_stamps, 0, size_t(g.ntiles) * ie::kStamps * sizeof(uint64_t), c->stream));
    }
    a.stamps = d_stamps;
    a.deep_lb = small ? 1 : 0;
    const int fix_per_tile = ie::launch_encode(a, c->n, L.mode == IE_MODE_EXACT, c->stream, bpt);
    c->last_fix_words = (L.mode == IE_MODE_EXACT) ? 0 : g.ntiles * fix_per_tile;
    HIPCHK(c, hipGetLastError());
    if (d_stamps) {
        std::vector<uint64_t> hs(size_t(g.ntiles) * ie::kStamps);
        HIPCHK(c, hipMemcpyAsync(hs.data(), d_stamps, hs.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(d_stamps));
        if (FILE* f = std::fopen(stamp_file, "wb")) {
            std::fwrite(hs.data(), sizeof(uint64_t), hs.size(), f);
            std::fclose(f);
        }
    }
    if (c->use_ticket) c->ticket_base += uint64_t(g.ntiles);
    return IE_OK;
}

int streamed_images(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                    int use_rle, int mode, uint8_t* out, size_t out_pitch, uint64_t start_bit, uint64_t* end_bits);
int streamed_frames(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                    int use_rle, int mode, uint8_t* out, size_t out_cap, uint64_t start_bit, uint64_t* frame_bits,
                    uint64_t* end_bit);

// Common driver of ie_encode_frames (segmented = 0) and ie_encode_images (segmented = 1).
int encode(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
           int use_rle, int mode, uint8_t* out, size_t out_cap, size_t out_pitch, uint64_t start_bit,
           int segmented, uint64_t* frame_bits, uint64_t* end_bits, int16_t* coef = nullptr,
           uint32_t* hist = nullptr) {
    c->fused_count = 0;  // any encode replaces the batch scratch's meaning
    int r = check_dims(c, w, h, nframes);
    if (r) return r;
    if (stride < size_t(w)) return fail(c, IE_EINVAL, "stride < width");
    if (nframes > 1 && frame_pitch < stride * size_t(h - 1) + size_t(w))
        return fail(c, IE_EINVAL, "frame_pitch smaller than a frame");
    if (segmented && (out_pitch % 4)) return fail(c, IE_EINVAL, "out_pitch must be a multiple of 4");
    HIPCHK(c, hipSetDevice(c->device));
    const Geometry g = geometry(w, h, c->n, nframes);
    const int nchains = segmented ? nframes : 1;

    // output bound
    const uint64_t payload_bound = uint64_t(g.bx) * g.by * bound_bits_per_block(c->n) * (segmented ? 1 : nframes);
    const uint64_t end_bound = start_bit + payload_bound;
    const size_t need_bytes = size_t((end_bound + 31) / 32) * 4;
    const size_t span = segmented ? out_pitch * size_t(nframes - 1) + need_bytes : need_bytes;
    if (segmented && out_pitch < need_bytes) return fail(c, IE_ECAP, "out_pitch below ie_stream_bound");
    if (out_cap < span) return fail(c, IE_ECAP, "output capacity below ie_stream_bound");
    const bool in_dev = is_device_ptr(y), out_dev = is_device_ptr(out);

    // Host frames in AND host streams out, several frames: the streamed path (pinned double
    // buffering, H2D / encode / D2H on three streams; ie_vstream for the concatenated chain).
    if (!in_dev && !out_dev && nframes > 1 && !coef && !hist && !c->use_ticket) {
        return segmented ? streamed_images(c, y, w, h, stride, frame_pitch, nframes, use_rle, mode, out, out_pitch,
                                           start_bit, end_bits)
                         : streamed_frames(c, y, w, h, stride, frame_pitch, nframes, use_rle, mode, out, out_cap,
                                           start_bit, frame_bits, end_bits);
    }

    // input
    const size_t in_bytes = size_t(nframes - 1) * frame_pitch + stride * size_t(h - 1) + size_t(w);
    const uint8_t* dy = y;
    if (!in_dev) {
        if ((r = ensure(c, c->d_in, c->cap_in, in_bytes))) return r;
        HIPCHK(c, hipMemcpyAsync(c->d_in, y, in_bytes, hipMemcpyHostToDevice, c->stream));
        dy = c->d_in;
    }

    // output
    uint32_t* dout;
    const uint64_t w0 = start_bit / 32;
    if (out_dev) {
        if (reinterpret_cast<uintptr_t>(out) % 4) return fail(c, IE_EINVAL, "device output must be 4-byte aligned");
        dout = reinterpret_cast<uint32_t*>(out);
    } else {
        // stage from the word holding start_bit; its leading bytes carry the caller's header
        const size_t stage = span - size_t(w0) * 4;
        if ((r = ensure(c, c->d_out, c->cap_out, stage))) return r;
        for (int f = 0; f < (segmented ? nframes : 1); f++) {
            const size_t hb = size_t(f) * out_pitch + size_t(w0) * 4;
            uint8_t word[4] = {0, 0, 0, 0};
            for (int e = 0; e < 4 && hb + e < out_cap; e++) word[e] = out[hb + e];
            // keep only the bytes before start_bit's byte plus its leading bits
            HIPCHK(c, hipMemcpyAsync(c->d_out + size_t(f) * out_pitch, word, 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
        }
        dout = reinterpret_cast<uint32_t*>(c->d_out) - w0;
    }

    Launch L;
    L.dy = dy;
    L.w = w;
    L.h = h;
    L.stride = stride;
    L.frame_pitch = frame_pitch;
    L.nframes = nframes;
    L.use_rle = use_rle;
    L.mode = mode;
    L.dout = dout;
    L.out_pitch = out_pitch;
    L.start_bit = start_bit;
    L.segmented = segmented;
    L.coef = coef;
    L.hist = hist;
    if ((r = launch_chain(c, L))) return r;

    const bool want = frame_bits || end_bits || !out_dev;
    if (!want) {
        note_async(c, hist ? "counting encode" : "encode");
        return IE_OK;
    }
    std::vector<uint64_t> fs(nframes), ce(nchains);
    HIPCHK(c, hipMemcpyAsync(fs.data(), c->d_frame_start, nframes * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(ce.data(), c->d_chain_end, nchains * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    unsigned timeouts = 0;
    if ((r = read_errors(c, &timeouts, &c->last_fallbacks))) return r;
    if (timeouts) {
        if (c->use_ticket) return fail(c, IE_EDEVICE, "tile look-back timed out");
        c->use_ticket = true;  // dispatch order did not hold: order the tiles explicitly and redo
        return encode(c, y, w, h, stride, frame_pitch, nframes, use_rle, mode, out, out_cap, out_pitch, start_bit,
                      segmented, frame_bits, end_bits, coef, hist);
    }
    if (!out_dev) {
        for (int ch = 0; ch < nchains; ch++) {
            const size_t b0 = size_t(ch) * out_pitch + size_t(start_bit / 8);
            const size_t b1 = size_t(ch) * out_pitch + size_t((ce[ch] + 7) / 8);
            const size_t off = b0 - (size_t(ch) * out_pitch + size_t(w0) * 4);
            HIPCHK(c, hipMemcpy(out + b0, c->d_out + size_t(ch) * out_pitch + off, b1 - b0, hipMemcpyDeviceToHost));
        }
    }
    if (frame_bits) {
        if (segmented) {
            for (int f = 0; f < nframes; f++) frame_bits[f] = ce[f] - fs[f];
        } else {
            for (int f = 0; f < nframes; f++) frame_bits[f] = ((f + 1 < nframes) ? fs[f + 1] : ce[0]) - fs[f];
        }
    }
    if (end_bits) {
        for (int ch = 0; ch < nchains; ch++) end_bits[ch] = ce[ch];
    }
    return IE_OK;
}

// ---- streamed host path ---------------------------------------------------------------------
// Host frames in, host streams out (the reference reads and writes whole files, utils.hpp:352-402,
// VideoBase.cpp:6-19): the batch flows through the device in sub-batches ("chunks") of a few
// frames.  Three HIP streams -- H2D (c->pipe->h2d), encode (c->stream), D2H (c->pipe->d2h) --
// with two device slots and two pinned host slots per direction: the H2D of chunk k+1, the encode
// of chunk k and the D2H of chunk k-1 run at the same time (PCIe is full duplex).  Pinned caller
// buffers (ie_host_alloc / hipHostMalloc / hipHostRegister) are DMA'd directly; pageable ones go
// through the pinned slots with a multi-threaded host copy.

bool is_pinned_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

// memcpy split over a few threads (a single core copies ~10 GB/s, PCIe moves ~50 GB/s).
void par_copy(uint8_t* dst, const uint8_t* src, size_t n) {
    constexpr size_t kPart = size_t(4) << 20;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t parts = std::min<size_t>(std::min<size_t>(hw, 8), (n + kPart - 1) / kPart);
    if (parts <= 1) {
        std::memcpy(dst, src, n);
        return;
    }
    const size_t per = (n + parts - 1) / parts;
    std::vector<std::thread> th;
    th.reserve(parts - 1);
    for (size_t i = 1; i < parts; i++) {
        const size_t b = i * per, e = std::min(n, b + per);
        if (b < e) th.emplace_back([=] { std::memcpy(dst + b, src + b, e - b); });
    }
    std::memcpy(dst, src, std::min(n, per));
    for (auto& t : th) t.join();
}

}  // namespace

struct ie_pipe {
    hipStream_t h2d = nullptr, d2h = nullptr;
    hipEvent_t ev_h2d[2] = {}, ev_enc[2] = {}, ev_d2h[2] = {};
    bool rec_enc[2] = {}, rec_d2h[2] = {}, rec_h2d[2] = {};
    uint8_t* d_in[2] = {};
    size_t cap_din[2] = {};
    uint8_t* d_out[2] = {};
    size_t cap_dout[2] = {};
    uint8_t* h_in[2] = {};
    size_t cap_hin[2] = {};
    uint8_t* h_out[2] = {};
    size_t cap_hout[2] = {};
    uint64_t* h_ends = nullptr;    // pinned [2][kMaxChunk + 1]: images: each image's chain end;
                                   // video chunks: the frame starts, then [kMaxChunk] the chain end
    uint32_t* h_hdr = nullptr;     // pinned [2][kMaxChunk] header words (the word holding start_bit)
    uint64_t* d_ends = nullptr;    // device [2]: chained launches read the previous end here
};
namespace {

using Pipe = ie_pipe;
constexpr int kMaxChunk = 64;

int pipe_new(ie_ctx* c, Pipe*& P) {
    P = new Pipe();
    HIPCHK(c, hipStreamCreateWithFlags(&P->h2d, hipStreamNonBlocking));
    HIPCHK(c, hipStreamCreateWithFlags(&P->d2h, hipStreamNonBlocking));
    for (int i = 0; i < 2; i++) {
        HIPCHK(c, hipEventCreateWithFlags(&P->ev_h2d[i], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&P->ev_enc[i], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&P->ev_d2h[i], hipEventDisableTiming));
    }
    HIPCHK(c, hipHostMalloc(&P->h_ends, 2 * (kMaxChunk + 1) * sizeof(uint64_t)));
    HIPCHK(c, hipHostMalloc(&P->h_hdr, 2 * kMaxChunk * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&P->d_ends, 2 * sizeof(uint64_t)));
    return IE_OK;
}

void pipe_free(Pipe* p) {
    if (!p) return;
    if (p->h2d) (void)hipStreamSynchronize(p->h2d);
    if (p->d2h) (void)hipStreamSynchronize(p->d2h);
    for (int i = 0; i < 2; i++) {
        (void)hipFree(p->d_in[i]);
        (void)hipFree(p->d_out[i]);
        if (p->h_in[i]) (void)hipHostFree(p->h_in[i]);
        if (p->h_out[i]) (void)hipHostFree(p->h_out[i]);
        if (p->ev_h2d[i]) (void)hipEventDestroy(p->ev_h2d[i]);
        if (p->ev_enc[i]) (void)hipEventDestroy(p->ev_enc[i]);
        if (p->ev_d2h[i]) (void)hipEventDestroy(p->ev_d2h[i]);
    }
    if (p->h_ends) (void)hipHostFree(p->h_ends);
    if (p->h_hdr) (void)hipHostFree(p->h_hdr);
    (void)hipFree(p->d_ends);
    if (p->h2d) (void)hipStreamDestroy(p->h2d);
    if (p->d2h) (void)hipStreamDestroy(p->d2h);
    delete p;
}

// The context's pipeline for streamed image batches; a new run starts with nothing pending (the
// previous one ended with a full synchronisation).
int pipe_get(ie_ctx* c, Pipe*& P) {
    if (!c->pipe) {
        int r = pipe_new(c, c->pipe);
        if (r) {
            pipe_free(c->pipe);
            c->pipe = nullptr;
            return r;
        }
    }
    P = c->pipe;
    for (int i = 0; i < 2; i++) P->rec_enc[i] = P->rec_d2h[i] = P->rec_h2d[i] = false;
    return IE_OK;
}

// device / pinned slot buffers (a slot is only resized when nothing of this run uses it yet)
int slot_dev(ie_ctx* c, uint8_t*& p, size_t& cap, size_t need) {
    if (cap >= need && p) return IE_OK;
    if (p) HIPCHK(c, hipFree(p));
    p = nullptr;
    HIPCHK(c, hipMalloc(&p, need));
    cap = need;
    return IE_OK;
}
int slot_pinned(ie_ctx* c, uint8_t*& p, size_t& cap, size_t need) {
    if (cap >= need && p) return IE_OK;
    if (p) HIPCHK(c, hipHostFree(p));
    p = nullptr;
    HIPCHK(c, hipHostMalloc(&p, need));
    cap = need;
    return IE_OK;
}

// frames per chunk: ~8 MiB of pixels (at least 1, at most kMaxChunk), and at least two chunks
// (IE_CHUNK_MB overrides the target: a tuning aid, the output does not depend on it)
int chunk_frames(size_t frame_bytes, int nframes) {
    const char* e = getenv("IE_CHUNK_MB");
    const size_t target = (e && atof(e) > 0) ? size_t(atof(e) * 1048576.0) : size_t(8) << 20;
    int k = int(std::max<size_t>(1, target / std::max<size_t>(1, frame_bytes)));
    k = std::min(k, kMaxChunk);
    k = std::min(k, (nframes + 1) / 2);
    return std::max(k, 1);
}

// Upload chunk `k` (frames f0 .. f0+nf-1) into device slot s on the H2D stream.
int pipe_upload(ie_ctx* c, Pipe* P, int s, const uint8_t* y, size_t frame_pitch, size_t in_bytes, int f0,
                bool pinned_in) {
    // d_in[s] is free once the encode of the chunk that last used it is done
    if (P->rec_enc[s]) HIPCHK(c, hipStreamWaitEvent(P->h2d, P->ev_enc[s], 0));
    const uint8_t* src = y + size_t(f0) * frame_pitch;
    if (pinned_in) {
        HIPCHK(c, hipMemcpyAsync(P->d_in[s], src, in_bytes, hipMemcpyHostToDevice, P->h2d));
    } else {
        if (P->rec_h2d[s]) HIPCHK(c, hipEventSynchronize(P->ev_h2d[s]));  // h_in[s] drained
        par_copy(P->h_in[s], src, in_bytes);
        HIPCHK(c, hipMemcpyAsync(P->d_in[s], P->h_in[s], in_bytes, hipMemcpyHostToDevice, P->h2d));
    }
    HIPCHK(c, hipEventRecord(P->ev_h2d[s], P->h2d));
    P->rec_h2d[s] = true;
    return IE_OK;
}

int streamed_images(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                    int use_rle, int mode, uint8_t* out, size_t out_pitch, uint64_t start_bit, uint64_t* end_bits) {
    // Three host threads keep the three streams busy: the uploader issues chunk k's H2D, this
    // thread chunk k's encode, the downloader chunk k's stream D2H.  A copy from or to PAGEABLE
    // memory is synchronous for its calling thread (the runtime stages it), so each direction has
    // its own thread and both PCIe directions stay busy; pinned memory is DMA'd directly.
    Pipe* P;
    int r;
    if ((r = pipe_get(c, P))) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int K = chunk_frames(stride * size_t(h), nframes);
    const int nchunks = (nframes + K - 1) / K;
    const size_t in_bytes = size_t(K - 1) * frame_pitch + stride * size_t(h - 1) + size_t(w);
    const uint64_t w0 = start_bit / 32;
    const size_t b0 = size_t(start_bit / 8);
    const size_t stage = out_pitch * size_t(K - 1) + (out_pitch - size_t(w0) * 4);  // slot: from word w0 of image 0
    for (int s = 0; s < 2; s++) {
        if ((r = slot_dev(c, P->d_in[s], P->cap_din[s], in_bytes))) return r;
        if ((r = slot_dev(c, P->d_out[s], P->cap_dout[s], stage))) return r;
    }
    std::vector<uint64_t> ends(size_t(nframes), 0);
    // hand-offs between the three threads: counters of chunks whose H2D / encode / D2H are
    // issued, waited on by spinning (a condition variable's wake-up costs tens of microseconds
    // per hand-off, several per chunk)
    std::atomic<int> uploaded{0}, enqueued{0}, downloaded{0};
    std::atomic<int> err{IE_OK};
    std::mutex mu;
    std::string msg;
    auto set_err = [&](int code, const std::string& m) {
        std::lock_guard<std::mutex> lk(mu);
        int ok = IE_OK;
        if (err.compare_exchange_strong(ok, code)) msg = m;
    };
    auto wait_for = [&](const std::atomic<int>& counter, int value) {  // false: another thread failed
        while (counter.load(std::memory_order_acquire) < value) {
            if (err.load(std::memory_order_relaxed) != IE_OK) return false;
            std::this_thread::yield();
        }
        return err.load(std::memory_order_relaxed) == IE_OK;
    };
    auto publish = [&](std::atomic<int>& counter) { counter.fetch_add(1, std::memory_order_release); };
#define TCHK(expr)                                                                   \
    do {                                                                             \
        hipError_t e_ = (expr);                                                      \
        if (e_ != hipSuccess) {                                                      \
            set_err(IE_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
            return;                                                                  \
        }                                                                            \
    } while (0)
    // the three roles, per chunk
    auto upload = [&](int k) {
        const int s = k & 1, f0 = k * K, nf = std::min(K, nframes - f0);
        if (!wait_for(enqueued, k - 1)) return;  // d_in[s]'s previous reader (chunk k-2) is launched
        if (k >= 2) TCHK(hipStreamWaitEvent(P->h2d, P->ev_enc[s], 0));
        const size_t ib = size_t(nf - 1) * frame_pitch + stride * size_t(h - 1) + size_t(w);
        TCHK(hipMemcpyAsync(P->d_in[s], y + size_t(f0) * frame_pitch, ib, hipMemcpyHostToDevice, P->h2d));
        TCHK(hipEventRecord(P->ev_h2d[s], P->h2d));
        publish(uploaded);
    };
    auto download = [&](int j) {
        const int s = j & 1, f0 = j * K, nf = std::min(K, nframes - f0);
        if (!wait_for(enqueued, j + 1)) return;
        TCHK(hipEventSynchronize(P->ev_enc[s]));  // its end bits are in h_ends[s] (written by the encoder)
        const uint64_t* he = P->h_ends + s * (kMaxChunk + 1);
        for (int i = 0; i < nf; i++) {
            const uint64_t e = he[i];
            ends[size_t(f0 + i)] = e;
            const size_t n = size_t((e + 7) / 8) - b0;
            const uint8_t* src = P->d_out[s] + size_t(i) * out_pitch + (b0 - size_t(w0) * 4);
            if (n) TCHK(hipMemcpyAsync(out + size_t(f0 + i) * out_pitch + b0, src, n, hipMemcpyDeviceToHost, P->d2h));
        }
        TCHK(hipEventRecord(P->ev_d2h[s], P->d2h));
        publish(downloaded);
    };
    auto encode_chunk = [&](int k) {
        const int s = k & 1, f0 = k * K, nf = std::min(K, nframes - f0);
        // chunk k-2 (slot s) fully out: its streams downloaded (d_out[s]) and its ends read (h_ends[s])
        if (!wait_for(uploaded, k + 1) || !wait_for(downloaded, k - 1)) return;
        TCHK(hipStreamWaitEvent(c->stream, P->ev_h2d[s], 0));
        if (k >= 2) TCHK(hipStreamWaitEvent(c->stream, P->ev_d2h[s], 0));
        // each image's word holding start_bit (the caller's header bits), read by the device from
        // page-locked memory (h_hdr[s] is free: chunk k-2's encode has completed)
        uint32_t* hw = P->h_hdr + s * kMaxChunk;
        for (int i = 0; i < nf; i++) std::memcpy(&hw[i], out + size_t(f0 + i) * out_pitch + size_t(w0) * 4, 4);
        ie::launch_word_scatter(hw, reinterpret_cast<uint32_t*>(P->d_out[s]), out_pitch / 4, nf, c->stream);
        Launch L;
        L.dy = P->d_in[s];
        L.w = w;
        L.h = h;
        L.stride = stride;
        L.frame_pitch = frame_pitch;
        L.nframes = nf;
        L.use_rle = use_rle;
        L.mode = mode;
        L.dout = reinterpret_cast<uint32_t*>(P->d_out[s]) - w0;
        L.out_pitch = out_pitch;
        L.start_bit = start_bit;
        L.segmented = 1;
        // each image's end bit goes straight to page-locked host memory (no small SDMA read-back
        // queued behind the stream downloads)
        L.chain_end = P->h_ends + s * (kMaxChunk + 1);
        const int rl = launch_chain(c, L);
        if (rl != IE_OK) return set_err(rl, c->err);
        TCHK(hipEventRecord(P->ev_enc[s], c->stream));
        note_async(c, "streamed encode");
        publish(enqueued);
    };
    if (is_pinned_ptr(y) && is_pinned_ptr(out)) {
        // pinned both ways: every copy is asynchronous, one thread issues everything in order
        for (int k = 0; k < nchunks && err.load() == IE_OK; k++) {
            upload(k);
            encode_chunk(k);
            if (k >= 1) download(k - 1);
        }
        if (err.load() == IE_OK) download(nchunks - 1);
    } else {
        const int dev = c->device;
        std::thread uploader([&] {
            if (hipSetDevice(dev) != hipSuccess) return set_err(IE_EHIP, "hipSetDevice (uploader)");
            for (int k = 0; k < nchunks && err.load() == IE_OK; k++) upload(k);
        });
        std::thread downloader([&] {
            if (hipSetDevice(dev) != hipSuccess) return set_err(IE_EHIP, "hipSetDevice (downloader)");
            for (int j = 0; j < nchunks && err.load() == IE_OK; j++) download(j);
        });
        for (int k = 0; k < nchunks && err.load() == IE_OK; k++) encode_chunk(k);
        uploader.join();
        downloader.join();
    }
#undef TCHK
    (void)hipStreamSynchronize(P->h2d);
    (void)hipStreamSynchronize(P->d2h);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (err.load() != IE_OK) return fail(c, err.load(), msg);
    unsigned timeouts = 0;
    r = read_errors(c, &timeouts, &c->last_fallbacks);
    if (r == IE_EDEVICE || (r == IE_OK && timeouts)) {
        // a tile look-back timed out (dispatch order did not hold): redo the batch through the
        // staged path with ticket-ordered tiles
        c->use_ticket = true;
        return encode(c, y, w, h, stride, frame_pitch, nframes, use_rle, mode, out, out_pitch * size_t(nframes),
                      out_pitch, start_bit, 1, nullptr, end_bits);
    }
    if (r) return r;
    if (end_bits) std::memcpy(end_bits, ends.data(), ends.size() * sizeof(uint64_t));
    return IE_OK;
}

}  // namespace

// ---- streamed gop=1 video (ie_vstream_*) ----------------------------------------------------
// One bit-contiguous chain (Frame.cpp:31-45, VideoEncoder.cpp:83-91) grown chunk by chunk on the
// device: chunk k's launch starts at chunk k-1's chain end read on the device (start_dev), so the
// host never waits for an encode before launching the next; the finished bytes leave through the
// D2H stream while later chunks encode.
struct ie_vstream {
    ie_ctx* c = nullptr;
    int w = 0, h = 0, rle = 1, mode = IE_MODE_FAST;
    size_t stride = 0, frame_pitch = 0;
    uint64_t start_bit = 0;
    int max_frames = 0, frames = 0;  // capacity, frames pushed
    int K = 1;                       // frames per chunk
    uint8_t* d_stream = nullptr;     // the whole stream from byte 0 (the caller's head included)
    size_t cap = 0;
    int chunks = 0;                  // chunks launched
    int harvested = 0;               // chunks whose frame starts / end are known on the host
    uint64_t done_bits = 0;          // chain end of the last harvested chunk
    uint64_t pulled = 0;             // bytes [0, pulled) handed out by ie_vstream_pull
    int chunk_f0[2] = {}, chunk_nf[2] = {};
    std::vector<uint64_t> fs;        // absolute start bit of every harvested frame
    ie_pipe* P = nullptr;            // its own streams, events and slots
};

namespace {

// The host side of chunk j (the oldest unharvested one): its frame starts and chain end.
int vs_harvest(ie_vstream* v) {
    ie_ctx* c = v->c;
    Pipe* P = v->P;
    const int j = v->harvested, s = j & 1;
    HIPCHK(c, hipEventSynchronize(P->ev_enc[s]));
    const uint64_t* hs = P->h_ends + s * (kMaxChunk + 1);
    for (int i = 0; i < v->chunk_nf[s]; i++) v->fs[size_t(v->chunk_f0[s] + i)] = hs[i];
    v->done_bits = hs[kMaxChunk];
    v->harvested = j + 1;
    return IE_OK;
}

// One chunk: upload, then a launch continuing the chain on the device.
int vs_chunk(ie_vstream* v, const uint8_t* frames, int nf, bool pinned_in) {
    ie_ctx* c = v->c;
    Pipe* P = v->P;
    const int k = v->chunks, s = k & 1;
    while (k - v->harvested >= 2) {  // slot s's read-back area still holds chunk k-2's ends
        int r = vs_harvest(v);
        if (r) return r;
    }
    const size_t ib = size_t(nf - 1) * v->frame_pitch + v->stride * size_t(v->h - 1) + size_t(v->w);
    int r;
    if ((r = pipe_upload(c, P, s, frames, v->frame_pitch, ib, 0, pinned_in))) return r;
    HIPCHK(c, hipStreamWaitEvent(c->stream, P->ev_h2d[s], 0));
    Launch L;
    L.dy = P->d_in[s];
    L.w = v->w;
    L.h = v->h;
    L.stride = v->stride;
    L.frame_pitch = v->frame_pitch;
    L.nframes = nf;
    L.use_rle = v->rle;
    L.mode = v->mode;
    L.dout = reinterpret_cast<uint32_t*>(v->d_stream);
    L.start_bit = v->start_bit;
    L.start_dev = k ? P->d_ends + ((k - 1) & 1) : nullptr;
    L.chain_end = P->d_ends + s;
    if ((r = launch_chain(c, L))) return r;
    uint64_t* hs = P->h_ends + s * (kMaxChunk + 1);
    HIPCHK(c, hipMemcpyAsync(hs, c->d_frame_start, size_t(nf) * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(hs + kMaxChunk, P->d_ends + s, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipEventRecord(P->ev_enc[s], c->stream));
    P->rec_enc[s] = true;
    note_async(c, "streamed video encode");
    v->chunk_f0[s] = v->frames;
    v->chunk_nf[s] = nf;
    v->frames += nf;
    v->chunks = k + 1;
    return IE_OK;
}

// Copy stream bytes [v->pulled, b1) to dst (host, pinned or pageable) through the D2H stream:
// pinned destinations directly, pageable ones in 16 MiB pieces through two pinned slots (the
// host copies piece i out while piece i+1 is in flight).
int vs_copy_out(ie_vstream* v, uint8_t* dst, uint64_t b1) {
    ie_ctx* c = v->c;
    Pipe* P = v->P;
    if (b1 <= v->pulled) return IE_OK;
    const size_t n = size_t(b1 - v->pulled);
    const uint8_t* src = v->d_stream + v->pulled;
    // the bytes were written by the launches up to the last harvested chunk (on c->stream)
    HIPCHK(c, hipStreamWaitEvent(P->d2h, P->ev_enc[(v->harvested - 1) & 1], 0));
    if (is_pinned_ptr(dst)) {
        HIPCHK(c, hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, P->d2h));
        HIPCHK(c, hipStreamSynchronize(P->d2h));
    } else {
        constexpr size_t kPiece = size_t(16) << 20;
        int r;
        for (int s = 0; s < 2; s++)
            if ((r = slot_pinned(c, P->h_out[s], P->cap_hout[s], std::min(n, kPiece)))) return r;
        const size_t pieces = (n + kPiece - 1) / kPiece;
        for (size_t i = 0; i <= pieces; i++) {
            if (i < pieces) {  // slot i&1 was emptied at step i-1
                const size_t o = i * kPiece, len = std::min(kPiece, n - o);
                HIPCHK(c, hipMemcpyAsync(P->h_out[i & 1], src + o, len, hipMemcpyDeviceToHost, P->d2h));
                HIPCHK(c, hipEventRecord(P->ev_d2h[i & 1], P->d2h));
            }
            if (i >= 1) {
                const size_t j = i - 1, o = j * kPiece, len = std::min(kPiece, n - o);
                HIPCHK(c, hipEventSynchronize(P->ev_d2h[j & 1]));
                par_copy(dst + o, P->h_out[j & 1], len);
            }
        }
    }
    v->pulled = b1;
    return IE_OK;
}

}  // namespace

extern "C" {

int ie_vstream_open(ie_ctx* c, int w, int h, size_t stride, size_t frame_pitch, int use_rle, int mode,
                    const uint8_t* head, uint64_t start_bit, int max_frames, ie_vstream** out) {
    if (!c || !out || max_frames <= 0 || (start_bit && !head)) return IE_EINVAL;
    *out = nullptr;
    int r = check_dims(c, w, h, max_frames);
    if (r) return r;
    if (stride < size_t(w)) return fail(c, IE_EINVAL, "stride < width");
    if (frame_pitch < stride * size_t(h - 1) + size_t(w)) return fail(c, IE_EINVAL, "frame_pitch smaller than a frame");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    ie_vstream* v = new ie_vstream();
    if ((r = pipe_new(c, v->P))) {
        pipe_free(v->P);
        delete v;
        return r;
    }
    Pipe* P = v->P;
    v->c = c;
    v->w = w;
    v->h = h;
    v->stride = stride;
    v->frame_pitch = frame_pitch;
    v->rle = use_rle ? 1 : 0;
    v->mode = mode;
    v->start_bit = start_bit;
    v->max_frames = max_frames;
    v->K = chunk_frames(stride * size_t(h), 1 << 20);
    v->fs.assign(size_t(max_frames), 0);
    v->done_bits = start_bit;
    v->cap = ie_stream_bound(w, h, c->n, max_frames, start_bit);
    const size_t in_bytes = size_t(v->K - 1) * frame_pitch + stride * size_t(h - 1) + size_t(w);
    auto bad = [&](int code) {
        (void)hipFree(v->d_stream);
        pipe_free(v->P);
        delete v;
        return code;
    };
    if (hipMalloc(&v->d_stream, v->cap) != hipSuccess) return bad(fail(c, IE_EHIP, "hipMalloc(video stream)"));
    for (int s = 0; s < 2; s++) {
        if ((r = slot_dev(c, P->d_in[s], P->cap_din[s], in_bytes))) return bad(r);
        if ((r = slot_pinned(c, P->h_in[s], P->cap_hin[s], in_bytes))) return bad(r);
    }
    // the caller's head: bytes [0, ceil(start_bit/8)), bits from start_bit on cleared; the word
    // holding start_bit is completed by the first chunk's first tile
    const size_t hb = size_t((start_bit + 7) / 8);
    std::vector<uint8_t> hd(hb + 8, 0);
    if (hb) std::memcpy(hd.data(), head, hb);
    if (start_bit % 8) hd[hb - 1] &= uint8_t(0xFF00u >> (start_bit % 8));
    if (hipMemsetAsync(v->d_stream, 0, std::min(v->cap, hb + 8), c->stream) != hipSuccess ||
        (hb && hipMemcpyAsync(v->d_stream, hd.data(), hb, hipMemcpyHostToDevice, c->stream) != hipSuccess) ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return bad(fail(c, IE_EHIP, "video stream head upload"));
    *out = v;
    return IE_OK;
}

int ie_vstream_push(ie_vstream* v, const uint8_t* frames, int nframes) {
    if (!v || (!frames && nframes)) return IE_EINVAL;
    ie_ctx* c = v->c;
    if (nframes < 0 || v->frames + nframes > v->max_frames)
        return fail(c, IE_ECAP, "more frames pushed than ie_vstream_open's max_frames");
    if (ie_is_device_ptr(frames)) return fail(c, IE_EINVAL, "ie_vstream_push takes host frames");
    HIPCHK(c, hipSetDevice(c->device));
    // the previous push's pinned frames may still be in flight: they are released now
    HIPCHK(c, hipStreamSynchronize(v->P->h2d));
    const bool pinned = is_pinned_ptr(frames);
    for (int f = 0; f < nframes; f += v->K) {
        const int r = vs_chunk(v, frames + size_t(f) * v->frame_pitch, std::min(v->K, nframes - f), pinned);
        if (r) return r;
    }
    return IE_OK;
}

int ie_vstream_pull(ie_vstream* v, uint8_t* dst, size_t cap, size_t* nbytes) {
    if (!v || !nbytes || (!dst && cap)) return IE_EINVAL;
    *nbytes = 0;
    // every chunk but the newest is complete or nearly so: harvest them (the newest keeps encoding)
    while (v->harvested < v->chunks - 1) {
        const int r = vs_harvest(v);
        if (r) return r;
    }
    const uint64_t b1 = v->done_bits / 8;  // whole bytes (the partial one follows with the next chunk)
    if (b1 <= v->pulled) return IE_OK;
    if (b1 - v->pulled > cap) return fail(v->c, IE_ECAP, "pull buffer smaller than the finished bytes");
    const uint64_t b0 = v->pulled;
    const int r = vs_copy_out(v, dst, b1);
    if (r) return r;
    *nbytes = size_t(b1 - b0);
    return IE_OK;
}

int ie_vstream_finish(ie_vstream* v, uint8_t* dst, size_t cap, size_t* nbytes, uint64_t* end_bit,
                      uint64_t* frame_bits) {
    if (!v || (!dst && cap)) return IE_EINVAL;
    ie_ctx* c = v->c;
    if (nbytes) *nbytes = 0;
    int r;
    while (v->harvested < v->chunks)
        if ((r = vs_harvest(v))) return r;
    unsigned timeouts = 0;
    if ((r = read_errors(c, &timeouts, &c->last_fallbacks))) return r;
    if (timeouts) return fail(c, IE_EDEVICE, "tile look-back timed out in a streamed video chunk");
    const uint64_t end = v->done_bits, b1 = (end + 7) / 8;
    if (dst) {
        if (b1 - v->pulled > cap) return fail(c, IE_ECAP, "finish buffer smaller than the remaining bytes");
        const uint64_t b0 = v->pulled;
        if ((r = vs_copy_out(v, dst, b1))) return r;
        if (nbytes) *nbytes = size_t(b1 - b0);
    }
    if (end_bit) *end_bit = end;
    if (frame_bits)
        for (int f = 0; f < v->frames; f++)
            frame_bits[f] = ((f + 1 < v->frames) ? v->fs[size_t(f + 1)] : end) - v->fs[size_t(f)];
    return IE_OK;
}

int ie_last_decode_info(ie_ctx* c, int* chunks, int* levels) {
    if (!c) return IE_EINVAL;
    if (chunks) *chunks = c->last_chunks;
    if (levels) *levels = c->last_groups;
    return IE_OK;
}

int ie_set_exact_parse(ie_ctx* c, int exact) {
    if (!c) return IE_EINVAL;
    c->spec_parse = exact != 0 ? 0 : 1;  // any nonzero value: the exact parse
    return IE_OK;
}

int ie_set_spec_warm(ie_ctx* c, int warm) {
    if (!c) return IE_EINVAL;
    c->spec_warm = warm < 0 ? 0 : (warm > 8 ? 8 : warm);  // clamped before use: no negation
    return IE_OK;
}

int ie_last_decode_spec(ie_ctx* c) { return c ? c->last_spec : 0; }

const uint8_t* ie_vstream_device(const ie_vstream* v) { return v ? v->d_stream : nullptr; }

int ie_vstream_close(ie_vstream* v) {
    if (!v) return IE_OK;
    ie_ctx* c = v->c;
    (void)hipStreamSynchronize(c->stream);
    pipe_free(v->P);
    (void)hipFree(v->d_stream);
    delete v;
    return IE_OK;
}

int ie_host_alloc(ie_ctx* c, size_t bytes, void** out) {
    if (!c || !out) return IE_EINVAL;
    *out = nullptr;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipHostMalloc(out, bytes ? bytes : 4));
    return IE_OK;
}

int ie_host_free(ie_ctx* c, void* p) {
    if (!c) return IE_EINVAL;
    if (!p) return IE_OK;
    HIPCHK(c, hipHostFree(p));
    return IE_OK;
}

}  // extern "C"

namespace {

// ie_encode_frames with host frames and a host stream: the video stream pipeline, pulled into the
// caller's buffer as the chunks finish.
int streamed_frames(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                    int use_rle, int mode, uint8_t* out, size_t out_cap, uint64_t start_bit, uint64_t* frame_bits,
                    uint64_t* end_bit) {
    ie_vstream* v = nullptr;
    int r = ie_vstream_open(c, w, h, stride, frame_pitch, use_rle, mode, out, start_bit, nframes, &v);
    if (r) return r;
    size_t got = 0;
    for (int f = 0; f < nframes && r == IE_OK; f += v->K) {
        const int nf = std::min(v->K, nframes - f);
        if ((r = ie_vstream_push(v, y + size_t(f) * frame_pitch, nf))) break;
        const uint64_t b0 = v->pulled;
        if ((r = ie_vstream_pull(v, out + b0, out_cap - size_t(b0), &got))) break;
    }
    uint64_t end = 0;
    if (r == IE_OK) {
        const uint64_t b0 = v->pulled;
        r = ie_vstream_finish(v, out + b0, out_cap - size_t(b0), &got, &end, frame_bits);
    }
    ie_vstream_close(v);
    if (r == IE_EDEVICE && !c->use_ticket) {  // a look-back timeout: redo through the staged path
        c->use_ticket = true;
        return encode(c, y, w, h, stride, frame_pitch, nframes, use_rle, mode, out, out_cap, 0, start_bit, 0,
                      frame_bits, end_bit);
    }
    if (r) return r;
    if (end_bit) *end_bit = end;
    return IE_OK;
}


// Variable-length re-encode of n bytes (Huffman.cpp:314-319) into one stream from start_bit.
int pack(ie_ctx* c, const uint8_t* bytes, size_t n, const uint32_t* code, const uint8_t* len, uint8_t* out,
         size_t out_cap, uint64_t start_bit, uint64_t* end_bit) {
    HIPCHK(c, hipSetDevice(c->device));
    int r;
    unsigned maxlen = 0;
    for (int b = 0; b < 256; b++) {
        if (len[b] > 32) return fail(c, IE_EINVAL, "code length above 32 bits");
        maxlen = std::max<unsigned>(maxlen, len[b]);
    }
    const uint64_t end_bound = start_bit + uint64_t(maxlen) * n;
    const size_t need_bytes = size_t((end_bound + 31) / 32) * 4;
    if (out_cap < need_bytes) return fail(c, IE_ECAP, "output capacity below start_bit + max_len * n bits");
    // code table through pinned memory (the caller's arrays may be gone when the copy runs)
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::memcpy(c->h_code, code, 256 * sizeof(uint32_t));
    std::memcpy(reinterpret_cast<uint8_t*>(c->h_code + 256), len, 256);
    HIPCHK(c, hipMemcpyAsync(c->d_code, c->h_code, 2 * 256 * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    const uint8_t* din = bytes;
    if (n && !is_device_ptr(bytes)) {
        if ((r = ensure(c, c->d_in, c->cap_in, n))) return r;
        HIPCHK(c, hipMemcpyAsync(c->d_in, bytes, n, hipMemcpyHostToDevice, c->stream));
        din = c->d_in;
    }
    const bool out_dev = is_device_ptr(out);
    const uint64_t w0 = start_bit / 32;
    uint32_t* dout;
    if (out_dev) {
        if (reinterpret_cast<uintptr_t>(out) % 4) return fail(c, IE_EINVAL, "device output must be 4-byte aligned");
        dout = reinterpret_cast<uint32_t*>(out);
    } else {
        if ((r = ensure(c, c->d_out, c->cap_out, need_bytes - size_t(w0) * 4))) return r;
        uint8_t word[4] = {0, 0, 0, 0};
        for (int e = 0; e < 4 && size_t(w0) * 4 + e < out_cap; e++) word[e] = out[size_t(w0) * 4 + e];
        HIPCHK(c, hipMemcpyAsync(c->d_out, word, 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        dout = reinterpret_cast<uint32_t*>(c->d_out) - w0;
    }
    uint64_t end = start_bit;
    if (n) {
        const uint64_t tb = uint64_t(ie::pack_tile_bytes(int(maxlen)));
        const int ntiles = int((n + tb - 1) / tb);
        if ((r = prepare_state(c, ntiles, 1))) return r;
        ie::PackArgs a{};
        a.in = din;
        a.n = n;
        a.code = c->d_code;
        a.len = reinterpret_cast<const uint8_t*>(c->d_code + 256);
        a.ntiles = ntiles;
        a.out = dout;
        a.start_bit = start_bit;
        a.st = c->d_state;
        a.ticket = c->use_ticket ? c->d_ticket : nullptr;
        a.ticket_base = c->ticket_base;
        a.tag = c->tag;
        a.chain_end = c->d_chain_end;
        a.err = c->d_err;
        a.maxlen = int(maxlen);
        ie::launch_pack(a, c->stream);  // (no stage events: ie_last_stage_ms reports the batched calls)
        HIPCHK(c, hipGetLastError());
        if (c->use_ticket) c->ticket_base += uint64_t(ntiles);
        if (!end_bit && out_dev) {
            note_async(c, "Huffman pack");
            return IE_OK;
        }
        HIPCHK(c, hipMemcpyAsync(&end, c->d_chain_end, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
        unsigned timeouts = 0;
        if ((r = read_errors(c, &timeouts, nullptr))) return r;
        if (timeouts) {
            if (c->use_ticket) return fail(c, IE_EDEVICE, "tile look-back timed out");
            c->use_ticket = true;
            return pack(c, bytes, n, code, len, out, out_cap, start_bit, end_bit);
        }
    }
    if (!out_dev && end > start_bit) {
        const size_t b0 = size_t(start_bit / 8), b1 = size_t((end + 7) / 8);
        HIPCHK(c, hipMemcpy(out + b0, c->d_out + (b0 - size_t(w0) * 4), b1 - b0, hipMemcpyDeviceToHost));
    }
    if (end_bit) *end_bit = end;
    return IE_OK;
}

}  // namespace

extern "C" {

int ie_create(int device, ie_ctx** out) {
    if (!out) return IE_EINVAL;
    *out = nullptr;
    ie_ctx* c = new ie_ctx();
    c->device = device;
    int r = IE_OK;
    auto chk = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && r == IE_OK) r = fail(c, IE_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    };
    chk(hipSetDevice(device), "hipSetDevice");
    // A BLOCKING stream: it orders with the legacy default (NULL) stream, so device buffers a caller
    // (e.g. PyTorch's default stream) filled just before a call are complete when the call's kernels
    // read them, and vice versa.  (Callers with their own streams use ie_set_stream.)
    if (r == IE_OK) chk(hipStreamCreateWithFlags(&c->own, hipStreamDefault), "hipStreamCreate");
    c->stream = c->own;
    // Debug switch: order tiles by the atomic ticket from the first launch (exercises the
    // timeout-recovery path, which dispatch order otherwise never needs)
    if (const char* ft = getenv("IE_FORCE_TICKET")) c->use_ticket = atoi(ft) != 0;
    // Debug switch: the next k synchronous error checks report a look-back timeout (exercises the
    // redo-in-ticket-mode paths and their output clearing)
    if (const char* ft = getenv("IE_FAKE_TIMEOUTS")) c->fake_timeouts = atoi(ft);
    if (r == IE_OK) chk(hipMalloc(&c->d_tab, sizeof(ie::EncTables)), "hipMalloc(tables)");
    if (r == IE_OK) chk(hipHostMalloc(&c->h_tab, sizeof(ie::EncTables)), "hipHostMalloc(tables)");
    if (r == IE_OK) chk(hipMalloc(&c->d_ticket, sizeof(unsigned long long)), "hipMalloc(ticket)");
    if (r == IE_OK) chk(hipMemset(c->d_ticket, 0, sizeof(unsigned long long)), "hipMemset(ticket)");
    if (r == IE_OK) chk(hipMalloc(&c->d_err, kErrWords * sizeof(unsigned)), "hipMalloc(err)");
    if (r == IE_OK) chk(hipMemset(c->d_err, 0, kErrWords * sizeof(unsigned)), "hipMemset(err)");
    if (r == IE_OK) chk(hipMalloc(&c->d_code, 2 * 256 * sizeof(uint32_t)), "hipMalloc(code)");
    if (r == IE_OK) chk(hipHostMalloc(&c->h_code, 2 * 256 * sizeof(uint32_t)), "hipHostMalloc(code)");
    if (r == IE_OK) chk(hipMalloc(&c->d_hist, 256 * sizeof(uint32_t)), "hipMalloc(hist)");
    if (r == IE_OK) chk(hipMalloc(&c->d_misc, 8 * sizeof(uint64_t)), "hipMalloc(misc)");
    if (r == IE_OK) chk(hipMalloc(&c->d_first, 256 * sizeof(unsigned long long)), "hipMalloc(first)");
    if (r != IE_OK) {
        std::fprintf(stderr, "ie_create: %s\n", c->err.c_str());
        ie_destroy(c);
        return r;
    }
    *out = c;
    return IE_OK;
}

int ie_destroy(ie_ctx* c) {
    if (!c) return IE_OK;
    (void)hipSetDevice(c->device);
    if (c->own) (void)hipStreamSynchronize(c->own);
    if (c->stream && c->stream != c->own) (void)hipStreamSynchronize(c->stream);
    if (c->tab_stream) {
        (void)hipStreamSynchronize(c->tab_stream);
        (void)hipStreamDestroy(c->tab_stream);
    }
    (void)hipFree(c->d_tab);
    (void)hipHostFree(c->h_tab);
    (void)hipFree(c->d_state);
    (void)hipFree(c->d_ticket);
    (void)hipFree(c->d_frame_start);
    (void)hipFree(c->d_chain_end);
    (void)hipFree(c->d_err);
    (void)hipFree(c->d_wave_fix);
    (void)hipFree(c->d_in);
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_scratch);
    (void)hipFree(c->d_code);
    (void)hipHostFree(c->h_code);
    (void)hipFree(c->d_hist);
    (void)hipFree(c->d_batch);
    (void)hipHostFree(c->h_batch);
    (void)hipFree(c->d_chist);
    for (int i = 0; i < 2; i++) {
        (void)hipFree(c->d_cslot[i]);
        if (c->h_hist[i]) (void)hipHostFree(c->h_hist[i]);
        if (c->h_pack[i]) (void)hipHostFree(c->h_pack[i]);
        if (c->ev_hist[i]) (void)hipEventDestroy(c->ev_hist[i]);
        if (c->ev_pack[i]) (void)hipEventDestroy(c->ev_pack[i]);
        if (c->ev_packed[i]) (void)hipEventDestroy(c->ev_packed[i]);
        (void)hipFree(c->d_pack[i]);
    }
    for (hipEvent_t e : c->stage_ev)
        if (e) (void)hipEventDestroy(e);
    (void)hipFree(c->d_first);
    (void)hipFree(c->d_dec);
    (void)hipFree(c->d_walk);
    (void)hipFree(c->d_count);
    (void)hipFree(c->d_rtab);
    (void)hipFree(c->d_rpos);
    (void)hipFree(c->d_misc);
    if (c->h_decres) (void)hipHostFree(c->h_decres);
    (void)hipFree(c->d_hlut);
    (void)hipFree(c->d_hout);
    (void)hipFree(c->d_pix);
    (void)hipFree(c->d_coef);
    (void)hipFree(c->d_gop_rec);
    (void)hipFree(c->d_gop_coef);
    (void)hipFree(c->d_gop_bits);
    (void)hipFree(c->d_gop_tile);
    (void)hipFree(c->d_gop_pos);
    pipe_free(c->pipe);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
    return IE_OK;
}

const char* ie_last_error(const ie_ctx* c) { return c ? c->err.c_str() : "null context"; }

int ie_set_stream(ie_ctx* c, void* s) {
    if (!c) return IE_EINVAL;
    c->stream = s ? static_cast<hipStream_t>(s) : c->own;
    return IE_OK;
}

int ie_sync(ie_ctx* c) {
    if (!c) return IE_EINVAL;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    unsigned timeouts = 0;
    int r = read_errors(c, &timeouts, nullptr);  // fails if an unchecked launch timed out
    if (r) return r;
    if (timeouts) {  // (no asynchronous launch pending: a synchronous caller already re-ran it)
        c->use_ticket = true;
        return fail(c, IE_EDEVICE, "tile look-back timed out");
    }
    return IE_OK;
}

int ie_set_quant(ie_ctx* c, const uint16_t* q, int n) {
    if (!c || !q) return IE_EINVAL;
    if (n != 4 && n != 8) return fail(c, IE_EINVAL, "block size must be 4 or 8");
    for (int k = 0; k < n * n; k++)
        if (q[k] == 0) return fail(c, IE_EINVAL, "quantisation matrix entries must be > 0");
    if (c->n == n && std::memcmp(c->q, q, sizeof(uint16_t) * n * n) == 0) return IE_OK;  // unchanged
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));  // tables may be in use by a running launch
    if (!build_tables(n, q, c->h_tab)) return fail(c, IE_EINVAL, "FP32 transform does not match the reference map");
    HIPCHK(c, hipMemcpy(c->d_tab, c->h_tab, sizeof(ie::EncTables), hipMemcpyHostToDevice));
    c->n = n;
    std::memcpy(c->q, q, sizeof(uint16_t) * n * n);
    return IE_OK;
}

int ie_set_stage_timing(ie_ctx* c, int on) {
    if (!c) return IE_EINVAL;
    c->stage_timing = on != 0;
    if (!c->stage_timing) c->stage_rec[0] = c->stage_rec[1] = false;  // (stale marks are not reported)
    return IE_OK;
}

int ie_last_stage_ms(ie_ctx* c, int stage, float* ms) {
    if (!c || !ms || stage < 0 || stage > 1) return IE_EINVAL;
    if (!c->stage_rec[stage]) return fail(c, IE_EINVAL, "no batched Huffman stage recorded yet");
    HIPCHK(c, hipEventSynchronize(c->stage_ev[2 * stage + 1]));
    HIPCHK(c, hipEventElapsedTime(ms, c->stage_ev[2 * stage], c->stage_ev[2 * stage + 1]));
    return IE_OK;
}

int ie_cos_table(ie_ctx* c, double* out) {
    if (!c || !out) return IE_EINVAL;
    if (c->n == 0) return fail(c, IE_ENOQUANT, "ie_set_quant not called");
    // read back from the DEVICE table: the values every kernel's FP64 path multiplies with
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(out, reinterpret_cast<const char*>(c->d_tab) + offsetof(ie::EncTables, c),
                        sizeof(double) * size_t(c->n) * size_t(c->n), hipMemcpyDeviceToHost));
    return IE_OK;
}

size_t ie_stream_bound(int w, int h, int n, int nframes, uint64_t start_bit) {
    if ((n != 4 && n != 8) || w <= 0 || h <= 0 || nframes <= 0) return 0;
    const uint64_t bits = start_bit + uint64_t(w / n) * (h / n) * bound_bits_per_block(n) * nframes;
    return size_t((bits + 31) / 32) * 4;
}

int ie_encode_frames(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                     int use_rle, int mode, uint8_t* out, size_t out_cap, uint64_t start_bit, uint64_t* frame_bits,
                     uint64_t* end_bit) {
    if (!c || !y || !out) return IE_EINVAL;
    return encode(c, y, w, h, stride, frame_pitch, nframes, use_rle, mode, out, out_cap, 0, start_bit, 0,
                  frame_bits, end_bit);
}

// bits_needed of an int16 (utils.hpp:226-243): Frame::MVEC_BIT_SIZE = bits_needed(merange) (VideoBase.cpp:42)
static int mvec_bits(int merange) {
    int b = 1;
    const int16_t v = int16_t(merange);
    while (int16_t(int16_t((v & ((1 << b) - 1)) << (16 - b)) >> (16 - b)) != v) b++;
    return b;
}

size_t ie_gop_stream_bound(int w, int h, int n, int nframes, int merange, uint64_t start_bit) {
    if ((n != 4 && n != 8) || w <= 0 || h <= 0 || nframes <= 0 || merange < 0 || merange > 32767) return 0;
    const uint64_t per_frame = uint64_t(w / n) * (h / n) * bound_bits_per_block(n) +
                               uint64_t(w / 16) * (h / 16) * 2u * uint64_t(mvec_bits(merange));
    return size_t((start_bit + per_frame * uint64_t(nframes) + 31) / 32) * 4 + 8;
}

// The frame loop of VideoEncoder.cpp:83-91 with I- and P-frames (VideoBase.cpp:96-122): I-frames
// through the block encoder, P-frames through ie_pframe.hip; every frame starts at the previous
// frame's end bit read on the device, and a P-frame's reference is the previous frame's buffer as
// the reference leaves it (an I-frame's own pixels, a P-frame's reconstruction).
int ie_encode_gop(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes, int gop,
                  int merange, int use_rle, int mode, uint8_t* out, size_t out_cap, uint64_t start_bit,
                  uint64_t* frame_bits, uint64_t* end_bit) {
    if (!c || !y || !out) return IE_EINVAL;
    int r = check_dims(c, w, h, nframes);
    if (r) return r;
    gop = std::max(1, gop);
    if (merange < 0 || merange > 32767) return fail(c, IE_EINVAL, "merange must be in [0, 32767] (15-bit header field)");
    if (stride < size_t(w)) return fail(c, IE_EINVAL, "stride < width");
    if (nframes > 1 && frame_pitch < stride * size_t(h - 1) + size_t(w))
        return fail(c, IE_EINVAL, "frame_pitch smaller than a frame");
    const bool has_p = gop > 1 && nframes > 1;
    if (has_p && w % 16 && h / 16 >= 2)
        return fail(c, IE_EINVAL, "P-frames need W % 16 == 0 when H >= 32: the reference builds its macroblocks "
                                  "from misplaced, overlapping rows there (ImageBase.cpp:223-227)");
    const size_t need = ie_gop_stream_bound(w, h, c->n, nframes, merange, start_bit);
    if (out_cap < need) return fail(c, IE_ECAP, "output capacity below ie_gop_stream_bound");
    HIPCHK(c, hipSetDevice(c->device));
    const bool in_dev = is_device_ptr(y), out_dev = is_device_ptr(out);

    const uint8_t* dy = y;
    if (!in_dev) {
        const size_t in_bytes = size_t(nframes - 1) * frame_pitch + stride * size_t(h - 1) + size_t(w);
        if ((r = ensure(c, c->d_in, c->cap_in, in_bytes))) return r;
        HIPCHK(c, hipMemcpyAsync(c->d_in, y, in_bytes, hipMemcpyHostToDevice, c->stream));
        dy = c->d_in;
    }
    uint32_t* dout;
    if (out_dev) {
        if (reinterpret_cast<uintptr_t>(out) % 4) return fail(c, IE_EINVAL, "device output must be 4-byte aligned");
        dout = reinterpret_cast<uint32_t*>(out);
    } else {
        // zeroed staging (the P-frame records are ORed in) holding the caller's leading bytes
        if ((r = ensure(c, c->d_out, c->cap_out, need))) return r;
        HIPCHK(c, hipMemsetAsync(c->d_out, 0, need, c->stream));
        const size_t hb = size_t((start_bit + 7) / 8);
        if (hb) HIPCHK(c, hipMemcpyAsync(c->d_out, out, hb, hipMemcpyHostToDevice, c->stream));
        dout = reinterpret_cast<uint32_t*>(c->d_out);
    }
    const int n = c->n, bx = w / n, nb = bx * (h / n);
    if (has_p) {
        if ((r = ensure(c, c->d_gop_rec, c->cap_gop_rec, 2 * size_t(w) * h))) return r;
        if ((r = ensure(c, c->d_gop_coef, c->cap_gop_coef, size_t(nb) * 16))) return r;
        if ((r = ensure(c, c->d_gop_bits, c->cap_gop_bits, size_t(nb)))) return r;
        if ((r = ensure(c, c->d_gop_tile, c->cap_gop_tile, size_t(ie::pframe_tiles(nb)) + 1))) return r;
    }
    if ((r = ensure(c, c->d_gop_pos, c->cap_gop_pos, size_t(nframes) + 1))) return r;
    HIPCHK(c, hipMemcpy(c->d_gop_pos, &start_bit, sizeof(uint64_t), hipMemcpyHostToDevice));

    const uint8_t* ref = nullptr;
    size_t rs = 0;
    for (int f = 0; f < nframes; f++) {
        const uint8_t* cf = dy + size_t(f) * frame_pitch;
        if (f % gop == 0) {
            Launch L;
            L.dy = cf;
            L.w = w;
            L.h = h;
            L.stride = stride;
            L.nframes = 1;
            L.use_rle = use_rle;
            L.mode = mode;
            L.dout = dout;
            L.start_bit = start_bit;
            L.start_dev = c->d_gop_pos + f;
            L.chain_end = c->d_gop_pos + f + 1;
            if ((r = launch_chain(c, L))) return r;
            ref = cf;
            rs = stride;
        } else {
            ie::PfArgs a{};
            a.cur = cf;
            a.cs = stride;
            a.ref = ref;
            a.rs = rs;
            a.rec = c->d_gop_rec + size_t(f & 1) * size_t(w) * h;
            a.w = w;
            a.h = h;
            a.mbx = w / 16;
            a.mby = h / 16;
            a.bx = bx;
            a.rle = use_rle ? 1 : 0;
            a.merange = merange;
            a.mv_bits = mvec_bits(merange);
            a.tab = c->d_tab;
            a.coef = c->d_gop_coef;
            a.bits = c->d_gop_bits;
            a.out = dout;
            a.start = c->d_gop_pos + f;
            a.end = c->d_gop_pos + f + 1;
            if (n == 4 && !c->use_ticket) {  // the record tiles' scan by look-back (one launch)
                if ((r = prepare_state(c, ie::pframe_tiles(nb), 1))) return r;
                a.st = c->d_state;
                a.tag = c->tag;
                a.err = c->d_err;
            }
            ie::launch_pframe(a, n, c->d_gop_tile, c->stream);
            HIPCHK(c, hipGetLastError());
            ref = a.rec;
            rs = size_t(w);
        }
    }
    std::vector<uint64_t> pos(size_t(nframes) + 1);
    HIPCHK(c, hipMemcpyAsync(pos.data(), c->d_gop_pos, pos.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    unsigned timeouts = 0;
    if ((r = read_errors(c, &timeouts, nullptr))) return r;
    if (timeouts) {
        if (c->use_ticket) return fail(c, IE_EDEVICE, "tile look-back timed out");
        c->use_ticket = true;  // an I-frame's tiles did not run in order: redo in ticket mode
        if (out_dev) {
            // the first attempt ORed vectors and P-frame records at positions derived from a bad end
            // bit: clear the caller's stream from start_bit on (the bits before it are the caller's)
            const size_t b0 = size_t(start_bit / 8), b1 = size_t((start_bit + 7) / 8);
            if (c->fake_fired) {  // debug: a faked timeout stands for a bad first attempt -- leave junk
                c->fake_fired = false;
                HIPCHK(c, hipMemsetAsync(out + b0 + (b1 > b0 ? 1 : 0), 0xA5, need - b1, c->stream));
                if (b1 > b0) {
                    uint8_t lead = 0;
                    HIPCHK(c, hipMemcpyAsync(&lead, out + b0, 1, hipMemcpyDeviceToHost, c->stream));
                    HIPCHK(c, hipStreamSynchronize(c->stream));
                    lead |= uint8_t(0xFFu >> (start_bit % 8));
                    HIPCHK(c, hipMemcpyAsync(out + b0, &lead, 1, hipMemcpyHostToDevice, c->stream));
                }
            }
            if (need > b1) HIPCHK(c, hipMemsetAsync(out + b1, 0, need - b1, c->stream));
            if (b1 > b0) {
                uint8_t lead = 0;
                HIPCHK(c, hipMemcpyAsync(&lead, out + b0, 1, hipMemcpyDeviceToHost, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
                lead &= uint8_t(0xFF00u >> (start_bit % 8));
                HIPCHK(c, hipMemcpyAsync(out + b0, &lead, 1, hipMemcpyHostToDevice, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
            }
        }
        return ie_encode_gop(c, y, w, h, stride, frame_pitch, nframes, gop, merange, use_rle, mode, out, out_cap,
                             start_bit, frame_bits, end_bit);
    }
    if (!out_dev) {
        const size_t b0 = size_t(start_bit / 8), b1 = size_t((pos[nframes] + 7) / 8);
        HIPCHK(c, hipMemcpy(out + b0, c->d_out + b0, b1 - b0, hipMemcpyDeviceToHost));
    }
    if (frame_bits)
        for (int f = 0; f < nframes; f++) frame_bits[f] = pos[f + 1] - pos[f];
    if (end_bit) *end_bit = pos[nframes];
    return IE_OK;
}

int ie_encode_images(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                     int use_rle, int mode, uint8_t* out, size_t out_pitch, uint64_t start_bit, uint64_t* end_bits) {
    if (!c || !y || !out) return IE_EINVAL;
    return encode(c, y, w, h, stride, frame_pitch, nframes, use_rle, mode, out, out_pitch * size_t(nframes),
                  out_pitch, start_bit, 1, nullptr, end_bits);
}

int ie_encode_images_counted(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                             int use_rle, int mode, uint8_t* out, size_t out_pitch, uint64_t start_bit) {
    if (!c || !y || !out || nframes <= 0) return IE_EINVAL;
    // no fused variant (EXACT mode, 8x8 -- its registers are full --, host output): the histogram
    // pass counts later
    if (mode == IE_MODE_EXACT || c->n != 4 || !is_device_ptr(out))
        return ie_encode_images(c, y, w, h, stride, frame_pitch, nframes, use_rle, mode, out, out_pitch, start_bit,
                                nullptr);
    // the counts go to d_chist, where ie_huffman_hist_batch_ends_async reads (and clears) them: the
    // memset before the launch only when they are not known to be zero
    const size_t K = size_t(nframes);
    int r;
    if (c->cap_chist < K * 256 || !c->d_chist) {
        if ((r = ensure(c, c->d_chist, c->cap_chist, K * 256))) return r;
        HIPCHK(c, hipMemsetAsync(c->d_chist, 0, c->cap_chist * sizeof(uint32_t), c->stream));
        c->chist_zero_rows = c->cap_chist / 256;
    }
    // rows [0, K) are counted into: skip their memset only when all of them are known zero (rows
    // of an earlier, larger batch that no fused pass cleared may hold stale counts)
    c->hist_skip_zero = K <= c->chist_zero_rows;
    c->chist_clean_after = c->hist_skip_zero ? c->chist_zero_rows : K;
    c->chist_zero_rows = 0;  // dirty until the fused pass reads this batch
    r = encode(c, y, w, h, stride, frame_pitch, nframes, use_rle, mode, out, out_pitch * K, out_pitch, start_bit, 1,
               nullptr, nullptr, nullptr, c->d_chist);
    c->hist_skip_zero = false;
    if (r == IE_OK) c->fused_count = nframes;
    return r;
}

int ie_quantize_frames(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                       int mode, int16_t* coef) {
    if (!c || !y || !coef) return IE_EINVAL;
    int r = check_dims(c, w, h, nframes);
    if (r) return r;
    const size_t bound = ie_stream_bound(w, h, c->n, nframes, 0);
    if ((r = ensure(c, c->d_scratch, c->cap_scratch, bound))) return r;
    const size_t ncoef = size_t(nframes) * (w / c->n) * (h / c->n) * c->n * c->n;
    const bool dev = is_device_ptr(coef);
    int16_t* dc = coef;
    if (!dev) {
        if ((r = ensure(c, c->d_coef, c->cap_coef, ncoef))) return r;
        dc = c->d_coef;
    }
    uint64_t end = 0;
    r = encode(c, y, w, h, stride, frame_pitch, nframes, 1, mode, c->d_scratch, bound, 0, 0, 0, nullptr, &end, dc);
    if (r) return r;
    if (!dev) HIPCHK(c, hipMemcpy(coef, dc, ncoef * sizeof(int16_t), hipMemcpyDeviceToHost));
    return IE_OK;
}

int ie_last_fallbacks(ie_ctx* c, uint64_t* count) {
    if (!c || !count) return IE_EINVAL;
    unsigned timeouts = 0;
    int r = read_errors(c, &timeouts, &c->last_fallbacks);  // the last encode launch's requests
    if (r) return r;
    *count = c->last_fallbacks;
    if (timeouts) return fail(c, IE_EDEVICE, "tile look-back timed out");
    return IE_OK;
}

int ie_is_device_ptr(const void* p) { return is_device_ptr(p) ? 1 : 0; }

int ie_malloc(ie_ctx* c, size_t bytes, void** out) {
    if (!c || !out) return IE_EINVAL;
    *out = nullptr;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMalloc(out, bytes ? bytes : 4));
    return IE_OK;
}

int ie_free(ie_ctx* c, void* p) {
    if (!c) return IE_EINVAL;
    if (!p) return IE_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipFree(p));
    return IE_OK;
}

int ie_memcpy(ie_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c || (bytes && (!dst || !src))) return IE_EINVAL;
    if (!bytes) return IE_OK;
    const bool dd = is_device_ptr(dst), sd = is_device_ptr(src);
    const hipMemcpyKind k = dd ? (sd ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice)
                               : (sd ? hipMemcpyDeviceToHost : hipMemcpyHostToHost);
    if (k == hipMemcpyHostToHost) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        std::memcpy(dst, src, bytes);
        return IE_OK;
    }
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, k, c->stream));
    if (k != hipMemcpyDeviceToDevice) HIPCHK(c, hipStreamSynchronize(c->stream));
    return IE_OK;
}

int ie_memset(ie_ctx* c, void* dst, int value, size_t bytes) {
    if (!c || (bytes && !dst)) return IE_EINVAL;
    if (!bytes) return IE_OK;
    if (!is_device_ptr(dst)) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        std::memset(dst, value, bytes);
        return IE_OK;
    }
    HIPCHK(c, hipMemsetAsync(dst, value, bytes, c->stream));
    return IE_OK;
}

int ie_huffman_hist(ie_ctx* c, const uint8_t* bytes, size_t n, uint32_t* hist, uint64_t* first_pos) {
    if (!c || (!bytes && n) || !hist || !first_pos) return IE_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    int r;
    const uint8_t* din = bytes;
    if (n && !is_device_ptr(bytes)) {
        if ((r = ensure(c, c->d_in, c->cap_in, n))) return r;
        HIPCHK(c, hipMemcpyAsync(c->d_in, bytes, n, hipMemcpyHostToDevice, c->stream));
        din = c->d_in;
    }
    HIPCHK(c, hipMemsetAsync(c->d_hist, 0, 256 * sizeof(uint32_t), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_first, 0xFF, 256 * sizeof(unsigned long long), c->stream));
    if (n) ie::launch_hist(din, n, c->d_hist, c->d_first, reinterpret_cast<unsigned*>(c->d_misc + 3), c->stream);
    HIPCHK(c, hipGetLastError());
    const hipMemcpyKind k1 = is_device_ptr(hist) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    const hipMemcpyKind k2 = is_device_ptr(first_pos) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    HIPCHK(c, hipMemcpyAsync(hist, c->d_hist, 256 * sizeof(uint32_t), k1, c->stream));
    HIPCHK(c, hipMemcpyAsync(first_pos, c->d_first, 256 * sizeof(uint64_t), k2, c->stream));
    if (k1 == hipMemcpyDeviceToHost || k2 == hipMemcpyDeviceToHost) HIPCHK(c, hipStreamSynchronize(c->stream));
    return IE_OK;
}

int ie_huffman_pack(ie_ctx* c, const uint8_t* bytes, size_t n, const uint32_t* code, const uint8_t* len,
                    uint8_t* out, size_t out_cap, uint64_t start_bit, uint64_t* end_bit) {
    if (!c || (!bytes && n) || !code || !len || !out) return IE_EINVAL;
    return pack(c, bytes, n, code, len, out, out_cap, start_bit, end_bit);
}

int ie_bitcopy(ie_ctx* c, const uint8_t* bytes, size_t n, uint8_t* out, size_t out_cap, uint64_t start_bit) {
    if (!c || (!bytes && n) || !out) return IE_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t end = start_bit + 8 * uint64_t(n);
    const size_t need_bytes = size_t((end + 31) / 32) * 4;  // whole words: the last one is zero-padded
    if (out_cap < need_bytes) return fail(c, IE_ECAP, "output capacity below ceil((start_bit + 8n) / 32) words");
    if (!n) return IE_OK;
    int r;
    const uint8_t* din = bytes;
    if (!is_device_ptr(bytes)) {
        if ((r = ensure(c, c->d_in, c->cap_in, n))) return r;
        HIPCHK(c, hipMemcpyAsync(c->d_in, bytes, n, hipMemcpyHostToDevice, c->stream));
        din = c->d_in;
    }
    const uint64_t w0 = start_bit / 32;
    if (is_device_ptr(out)) {
        if (reinterpret_cast<uintptr_t>(out) % 4) return fail(c, IE_EINVAL, "device output must be 4-byte aligned");
        // device to device: asynchronous on the context's stream
        ie::launch_bitshift(din, n, reinterpret_cast<uint32_t*>(out), start_bit, c->stream);
        HIPCHK(c, hipGetLastError());
        if (din == bytes) return IE_OK;
        HIPCHK(c, hipStreamSynchronize(c->stream));  // the staged input must outlive the copy
        return IE_OK;
    }
    // host output: stage from the word holding start_bit (its leading bytes keep the caller's bits)
    if ((r = ensure(c, c->d_out, c->cap_out, need_bytes - size_t(w0) * 4))) return r;
    uint8_t word[4] = {0, 0, 0, 0};
    for (int e = 0; e < 4 && size_t(w0) * 4 + e < out_cap; e++) word[e] = out[size_t(w0) * 4 + e];
    HIPCHK(c, hipMemcpyAsync(c->d_out, word, 4, hipMemcpyHostToDevice, c->stream));
    ie::launch_bitshift(din, n, reinterpret_cast<uint32_t*>(c->d_out) - w0, start_bit, c->stream);
    HIPCHK(c, hipGetLastError());
    const size_t b0 = size_t(start_bit / 8), b1 = size_t((end + 7) / 8);
    HIPCHK(c, hipMemcpyAsync(out + b0, c->d_out + (b0 - size_t(w0) * 4), b1 - b0, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return IE_OK;
}

int ie_huffman_hist_batch(ie_ctx* c, const uint8_t* in, size_t in_pitch, const uint64_t* n, int count,
                          uint32_t* hist, uint64_t* first_pos) {
    if (c) c->fused_count = 0;
    if (!c || !in || !n || count <= 0 || !hist || !first_pos) return IE_EINVAL;
    if (!is_device_ptr(in)) return fail(c, IE_EINVAL, "batched Huffman input must be device memory");
    HIPCHK(c, hipSetDevice(c->device));
    uint64_t maxn = 0;
    for (int k = 0; k < count; k++) {
        if (k + 1 < count && n[k] > in_pitch) return fail(c, IE_EINVAL, "string longer than the input pitch");
        maxn = std::max(maxn, n[k]);
    }
    const size_t hb = size_t(count) * 256 * sizeof(uint32_t), fb = size_t(count) * 256 * sizeof(uint64_t);
    const size_t nb = size_t(count) * sizeof(uint64_t), ub = size_t(count) * sizeof(unsigned);
    int r;
    if ((r = ensure(c, c->d_batch, c->cap_batch, hb + fb + nb + ub))) return r;
    if ((r = ensure_pinned(c, c->h_batch, c->cap_hbatch, nb))) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));  // the pinned staging may still feed a copy
    std::memcpy(c->h_batch, n, nb);
    uint32_t* dh = reinterpret_cast<uint32_t*>(c->d_batch);
    auto* df = reinterpret_cast<unsigned long long*>(c->d_batch + hb);
    auto* dn = reinterpret_cast<uint64_t*>(c->d_batch + hb + fb);
    HIPCHK(c, hipMemcpyAsync(dn, c->h_batch, nb, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemsetAsync(dh, 0, hb, c->stream));
    HIPCHK(c, hipMemsetAsync(df, 0xFF, fb, c->stream));
    auto* du = reinterpret_cast<unsigned*>(c->d_batch + hb + fb + nb);
    ie::launch_hist_batch(in, in_pitch, dn, maxn, count, dh, df, du, c->stream);
    HIPCHK(c, hipGetLastError());
    const hipMemcpyKind k1 = is_device_ptr(hist) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    const hipMemcpyKind k2 = is_device_ptr(first_pos) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    HIPCHK(c, hipMemcpyAsync(hist, dh, hb, k1, c->stream));
    HIPCHK(c, hipMemcpyAsync(first_pos, df, fb, k2, c->stream));
    if (k1 == hipMemcpyDeviceToHost || k2 == hipMemcpyDeviceToHost) HIPCHK(c, hipStreamSynchronize(c->stream));
    return IE_OK;
}

const uint64_t* ie_last_end_bits(ie_ctx* c) { return c ? c->d_chain_end : nullptr; }

int ie_huffman_hist_batch_ends(ie_ctx* c, const uint8_t* in, size_t in_pitch, const uint64_t* end_bits, int count,
                               uint32_t* hist, uint64_t* first_pos) {
    if (c) c->fused_count = 0;
    if (!c || !in || !end_bits || count <= 0 || !hist || !first_pos) return IE_EINVAL;
    if (!is_device_ptr(in) || !is_device_ptr(end_bits))
        return fail(c, IE_EINVAL, "batched Huffman input and end bits must be device memory");
    HIPCHK(c, hipSetDevice(c->device));
    const size_t hb = size_t(count) * 256 * sizeof(uint32_t), fb = size_t(count) * 256 * sizeof(uint64_t);
    const size_t nb = size_t(count) * sizeof(uint64_t), ub = size_t(count) * sizeof(unsigned);
    int r;
    if ((r = ensure(c, c->d_batch, c->cap_batch, hb + fb + nb + ub))) return r;
    uint32_t* dh = reinterpret_cast<uint32_t*>(c->d_batch);
    auto* df = reinterpret_cast<unsigned long long*>(c->d_batch + hb);
    auto* dn = reinterpret_cast<uint64_t*>(c->d_batch + hb + fb);
    auto* du = reinterpret_cast<unsigned*>(c->d_batch + hb + fb + nb);
    ie::launch_ends_to_bytes(end_bits, uint64_t(in_pitch), count, dn, c->stream, dh, df);
    ie::launch_hist_batch(in, in_pitch, dn, uint64_t(in_pitch), count, dh, df, du, c->stream);
    HIPCHK(c, hipGetLastError());
    const hipMemcpyKind k1 = is_device_ptr(hist) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    const hipMemcpyKind k2 = is_device_ptr(first_pos) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    HIPCHK(c, hipMemcpyAsync(hist, dh, hb, k1, c->stream));
    HIPCHK(c, hipMemcpyAsync(first_pos, df, fb, k2, c->stream));
    if (k1 == hipMemcpyDeviceToHost || k2 == hipMemcpyDeviceToHost) HIPCHK(c, hipStreamSynchronize(c->stream));
    return IE_OK;
}

int ie_huffman_hist_batch_ends_async(ie_ctx* c, const uint8_t* in, size_t in_pitch, const uint64_t* end_bits,
                                     int count, int slot) {
    if (!c || !in || !end_bits || count <= 0 || slot < 0 || slot > 1) return IE_EINVAL;
    if (!is_device_ptr(in) || !is_device_ptr(end_bits))
        return fail(c, IE_EINVAL, "batched Huffman input and end bits must be device memory");
    HIPCHK(c, hipSetDevice(c->device));
    // counts left by ie_encode_images_counted for exactly this batch: only the first positions remain
    const bool fused = c->fused_count == count;
    c->fused_count = 0;
    const size_t hb = size_t(count) * 256 * sizeof(uint32_t), fb = size_t(count) * 256 * sizeof(uint64_t);
    const size_t nb = size_t(count) * sizeof(uint64_t), ub = size_t(count) * sizeof(unsigned);
    int r;
    if ((r = ensure_pinned(c, c->h_hist[slot], c->cap_hhist[slot], hb + fb + ub))) return r;
    if (!c->ev_hist[slot]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_hist[slot], hipEventDisableTiming));
    c->hist_fused[slot] = fused;
    c->hist_in[slot] = in;
    c->hist_pitch[slot] = in_pitch;
    if (fused) {
        // counts from the encoder (cleared as they are read), lengths from the end bits, results
        // straight into the pinned slot: ONE launch, no memset, no copy
        if ((r = ensure(c, c->d_cslot[slot], c->cap_cslot[slot], fb + nb + ub))) return r;
        uint8_t* hp = nullptr;
        HIPCHK(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&hp), c->h_hist[slot], 0));
        uint8_t* ds = c->d_cslot[slot];
        if ((r = stage_mark(c, 0))) return r;
        ie::launch_first_counted(in, in_pitch, end_bits, uint64_t(in_pitch), count, c->d_chist,
                                 reinterpret_cast<uint64_t*>(ds + fb), reinterpret_cast<unsigned long long*>(ds),
                                 reinterpret_cast<unsigned*>(ds + fb + nb), reinterpret_cast<uint32_t*>(hp),
                                 reinterpret_cast<unsigned long long*>(hp + hb), reinterpret_cast<unsigned*>(hp + hb + fb),
                                 c->stream);
        HIPCHK(c, hipGetLastError());
        c->chist_zero_rows = c->chist_clean_after;  // (the pass cleared rows [0, count))
        if ((r = stage_mark(c, 1))) return r;
        HIPCHK(c, hipEventRecord(c->ev_hist[slot], c->stream));
        c->hist_count[slot] = count;
        return IE_OK;
    }
    if ((r = ensure(c, c->d_batch, c->cap_batch, hb + fb + nb + ub))) return r;
    uint32_t* dh = reinterpret_cast<uint32_t*>(c->d_batch);
    auto* df = reinterpret_cast<unsigned long long*>(c->d_batch + hb);
    auto* dn = reinterpret_cast<uint64_t*>(c->d_batch + hb + fb);
    auto* du = reinterpret_cast<unsigned*>(c->d_batch + hb + fb + nb);
    if ((r = stage_mark(c, 0))) return r;
    ie::launch_ends_to_bytes(end_bits, uint64_t(in_pitch), count, dn, c->stream, dh, df);
    ie::launch_hist_batch(in, in_pitch, dn, uint64_t(in_pitch), count, dh, df, du, c->stream, true);
    HIPCHK(c, hipGetLastError());
    if ((r = stage_mark(c, 1))) return r;
    // histograms and first positions are contiguous on the device: one read-back
    HIPCHK(c, hipMemcpyAsync(c->h_hist[slot], c->d_batch, hb + fb, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipEventRecord(c->ev_hist[slot], c->stream));
    c->hist_count[slot] = count;
    return IE_OK;
}

int ie_huffman_hist_batch_wait(ie_ctx* c, int slot, uint32_t* hist, uint64_t* first_pos) {
    if (!c || slot < 0 || slot > 1 || !hist || !first_pos) return IE_EINVAL;
    if (!c->ev_hist[slot] || !c->hist_count[slot]) return fail(c, IE_EINVAL, "no histogram pending in this slot");
    HIPCHK(c, hipEventSynchronize(c->ev_hist[slot]));
    const int K = c->hist_count[slot];
    const size_t hb = size_t(K) * 256 * sizeof(uint32_t), fb = size_t(K) * 256 * sizeof(uint64_t);
    const size_t nb = size_t(K) * sizeof(uint64_t);
    std::memcpy(hist, c->h_hist[slot], hb);
    std::memcpy(first_pos, c->h_hist[slot] + hb, fb);
    c->hist_count[slot] = 0;
    if (c->hist_fused[slot]) {
        // a string whose first-occurrence scan stopped short (a value first seen past its first
        // 64 chunks): the full pass over the batch, then the device's positions
        const unsigned* un = reinterpret_cast<const unsigned*>(c->h_hist[slot] + hb + fb);
        bool any = false;
        uint64_t maxn = 0;
        for (int k = 0; k < K; k++) any |= un[k] != 0u;
        if (any) {
            uint64_t* nn = reinterpret_cast<uint64_t*>(c->d_cslot[slot] + fb);
            for (int k = 0; k < K; k++) {
                uint64_t s = 0;
                for (int b = 0; b < 256; b++) s += hist[256 * k + b];
                maxn = std::max(maxn, s);
            }
            uint8_t* hp = nullptr;
            HIPCHK(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&hp), c->h_hist[slot], 0));
            // on the side stream, ordered after the batch's histogram only: work the caller queued on
            // c->stream since _async (e.g. the next batch's encode) is neither waited for nor
            // delayed, and only this launch and its read-back are synchronised
            if (!c->tab_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->tab_stream, hipStreamNonBlocking));
            HIPCHK(c, hipStreamWaitEvent(c->tab_stream, c->ev_hist[slot], 0));
            ie::launch_first_full_batch(c->hist_in[slot], c->hist_pitch[slot], nn, maxn, K, reinterpret_cast<const uint32_t*>(hp),
                                        reinterpret_cast<unsigned long long*>(c->d_cslot[slot]),
                                        reinterpret_cast<const unsigned*>(c->d_cslot[slot] + fb + nb), c->tab_stream);
            HIPCHK(c, hipGetLastError());
            HIPCHK(c, hipMemcpyAsync(first_pos, c->d_cslot[slot], fb, hipMemcpyDeviceToHost, c->tab_stream));
            HIPCHK(c, hipStreamSynchronize(c->tab_stream));
        }
    }
    return IE_OK;
}

int ie_huffman_pack_batch(ie_ctx* c, const uint8_t* in, size_t in_pitch, const uint64_t* n, int count,
                          const uint32_t* code, const uint8_t* len, const uint8_t* prefix, size_t prefix_pitch,
                          uint8_t* out, size_t out_pitch, const uint64_t* start_bit, uint64_t* end_bit) {
    if (!c || !in || !n || count <= 0 || !code || !len || !out || !start_bit || (!prefix && prefix_pitch))
        return IE_EINVAL;
    if (!is_device_ptr(in) || !is_device_ptr(out))
        return fail(c, IE_EINVAL, "batched Huffman input and output must be device memory");
    if (reinterpret_cast<uintptr_t>(out) % 4 || out_pitch % 4)
        return fail(c, IE_EINVAL, "output and its pitch must be 4-byte aligned");
    HIPCHK(c, hipSetDevice(c->device));
    // layout of the staged tables: tiles[count (+1 unused)] n[count] start[count] code[count*256]
    // prefix[count][pw] (words) len[count*256]
    uint64_t pw = 1, ntiles = 0;
    std::vector<uint64_t> ts(size_t(count) + 1);
    unsigned maxlen_all = 0;  // one tile shape for the whole batch
    for (int k = 0; k < count * 256; k++) maxlen_all = std::max<unsigned>(maxlen_all, len[k]);
    const uint64_t tb = uint64_t(ie::pack_tile_bytes(int(maxlen_all)));
    for (int k = 0; k < count; k++) {
        if (k + 1 < count && n[k] > in_pitch) return fail(c, IE_EINVAL, "string longer than the input pitch");
        unsigned maxlen = 0;
        for (int b = 0; b < 256; b++) {
            if (len[256 * k + b] > 32) return fail(c, IE_EINVAL, "code length above 32 bits");
            maxlen = std::max<unsigned>(maxlen, len[256 * k + b]);
        }
        const uint64_t end_bound = start_bit[k] + uint64_t(maxlen) * n[k];
        if (out_pitch < size_t((end_bound + 31) / 32) * 4)
            return fail(c, IE_ECAP, "output pitch below start_bit + max_len * n bits");
        if (start_bit[k] && !prefix) return fail(c, IE_EINVAL, "start_bit > 0 needs a prefix");
        if ((start_bit[k] + 7) / 8 > prefix_pitch && start_bit[k]) return fail(c, IE_EINVAL, "prefix pitch too small");
        pw = std::max<uint64_t>(pw, start_bit[k] / 32 + 1);
        ts[size_t(k)] = (n[k] + tb - 1) / tb;  // tiles of string k
        ntiles = std::max<uint64_t>(ntiles, ts[size_t(k)]);
    }
    ntiles *= uint64_t(count);  // interleaved: tile t -> string t % count (pack_kernel)
    ts[size_t(count)] = 0;
    if (ntiles > uint64_t(INT32_MAX)) return fail(c, IE_EINVAL, "batch too large");
    const size_t K = size_t(count);
    const size_t o_ts = 0, o_n = o_ts + 8 * (K + 1), o_st = o_n + 8 * K, o_code = o_st + 8 * K;
    const size_t o_pre = o_code + 4 * 256 * K, o_len = o_pre + 4 * size_t(pw) * K, total = o_len + 256 * K;
    int r;
    // two pinned staging slots and two device table slots in turn: wait only for this slot's
    // previous copy, not the stream.  The copy runs on a side stream as soon as the tables exist
    // (beside whatever the context's stream is running, e.g. the next batch's encode); the pack
    // waits for it by event, and the copy into a device slot waits for the pack that last read it.
    const int ps = c->pack_slot;
    c->pack_slot ^= 1;
    if (c->pack_recorded[ps]) HIPCHK(c, hipEventSynchronize(c->ev_pack[ps]));
    if ((r = ensure_pinned(c, c->h_pack[ps], c->cap_hpack[ps], total))) return r;
    if (c->cap_dpack[ps] < total && c->d_pack[ps]) HIPCHK(c, hipStreamSynchronize(c->stream));
    if ((r = ensure(c, c->d_pack[ps], c->cap_dpack[ps], total))) return r;
    if (!c->ev_pack[ps]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_pack[ps], hipEventDisableTiming));
    if (!c->ev_packed[ps]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_packed[ps], hipEventDisableTiming));
    if (!c->tab_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->tab_stream, hipStreamNonBlocking));
    uint8_t* h = c->h_pack[ps];
    std::memcpy(h + o_ts, ts.data(), 8 * (K + 1));
    std::memcpy(h + o_n, n, 8 * K);
    std::memcpy(h + o_st, start_bit, 8 * K);
    std::memcpy(h + o_code, code, 4 * 256 * K);
    std::memcpy(h + o_len, len, 256 * K);
    std::memset(h + o_pre, 0, 4 * size_t(pw) * K);
    for (size_t k = 0; k < K; k++) {
        const uint64_t sb = start_bit[k];
        if (!sb) continue;
        uint8_t* d = h + o_pre + 4 * size_t(pw) * k;
        const size_t nbytes = size_t((sb + 7) / 8);
        std::memcpy(d, prefix + k * prefix_pitch, nbytes);
        if (sb % 8) d[nbytes - 1] &= uint8_t(0xFF00u >> (sb % 8));  // bits from start_bit on are the packer's
    }
    if (c->packed_recorded[ps]) HIPCHK(c, hipStreamWaitEvent(c->tab_stream, c->ev_packed[ps], 0));
    HIPCHK(c, hipMemcpyAsync(c->d_pack[ps], h, total, hipMemcpyHostToDevice, c->tab_stream));
    HIPCHK(c, hipEventRecord(c->ev_pack[ps], c->tab_stream));
    c->pack_recorded[ps] = true;
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_pack[ps], 0));
    const uint8_t* d = c->d_pack[ps];
    // strings without bytes: the prefix alone
    for (size_t k = 0; k < K; k++)
        if (n[k] == 0)
            HIPCHK(c, hipMemcpyAsync(out + k * out_pitch, d + o_pre + 4 * size_t(pw) * k, 4 * size_t(start_bit[k] / 32 + 1),
                                     hipMemcpyDeviceToDevice, c->stream));
    if (ntiles) {
        if ((r = prepare_state(c, int(ntiles), count))) return r;
        ie::PackArgs a{};
        a.in = in;
        a.code = reinterpret_cast<const uint32_t*>(d + o_code);
        a.len = d + o_len;
        a.ntiles = int(ntiles);
        a.out = reinterpret_cast<uint32_t*>(out);
        a.st = c->d_state;
        a.ticket = c->use_ticket ? c->d_ticket : nullptr;
        a.ticket_base = c->ticket_base;
        a.tag = c->tag;
        a.chain_end = c->d_chain_end;
        a.err = c->d_err;
        a.count = count;
        a.tiles = reinterpret_cast<const uint64_t*>(d + o_ts);
        a.bn = reinterpret_cast<const uint64_t*>(d + o_n);
        a.bstart = reinterpret_cast<const uint64_t*>(d + o_st);
        a.in_pitch = in_pitch;
        a.out_pitch_words = out_pitch / 4;
        a.prefix_pitch_words = pw;
        a.prefix = reinterpret_cast<const uint32_t*>(d + o_pre);
        a.maxlen = int(maxlen_all);
        if ((r = stage_mark(c, 2))) return r;
        ie::launch_pack(a, c->stream);
        if ((r = stage_mark(c, 3))) return r;
        HIPCHK(c, hipGetLastError());
        if (c->use_ticket) c->ticket_base += ntiles;
    }
    HIPCHK(c, hipEventRecord(c->ev_packed[ps], c->stream));  // (the table slot's readers are done)
    c->packed_recorded[ps] = true;
    if (!end_bit) {
        if (ntiles) note_async(c, "Huffman batch pack");
        return IE_OK;
    }
    std::vector<uint64_t> ends(K);
    if (ntiles) HIPCHK(c, hipMemcpyAsync(ends.data(), c->d_chain_end, 8 * K, hipMemcpyDeviceToHost, c->stream));
    unsigned timeouts = 0;
    if ((r = read_errors(c, &timeouts, nullptr))) return r;
    if (timeouts) {
        if (c->use_ticket) return fail(c, IE_EDEVICE, "tile look-back timed out");
        c->use_ticket = true;
        return ie_huffman_pack_batch(c, in, in_pitch, n, count, code, len, prefix, prefix_pitch, out, out_pitch,
                                     start_bit, end_bit);
    }
    for (size_t k = 0; k < K; k++) end_bit[k] = n[k] ? ends[k] : start_bit[k];
    return IE_OK;
}

int ie_huffman_table(const uint8_t* in, size_t len, uint64_t start_bit, uint16_t* lut, uint64_t* code_start) {
    if ((!in && len) || !lut || !code_start) return IE_EINVAL;
    // MSB-first reads (BitStreamReader::get, BitStream.cpp:14-40); past the end: malformed
    uint64_t pos = start_bit;
    bool over = false;
    auto get = [&](unsigned nb) {
        uint32_t v = 0;
        for (unsigned k = 0; k < nb; k++, pos++) {
            if (pos >= uint64_t(len) * 8) {
                over = true;
                return 0u;
            }
            v = (v << 1) | ((in[pos >> 3] >> (7 - (pos & 7))) & 1u);
        }
        return v;
    };
    // Huffman::buildTree (Huffman.cpp:120-143): groups of {1, count:7, bits:4} headers, each
    // followed by count {key:8, code:bits} entries, ended by a '0' bit; treeAddLeaf (:143-173)
    // grows the tree along the code's bits MSB first (bits = 0 hangs the leaf on the root's left)
    struct Node {
        int child[2] = {-1, -1};
        int sym = -1;
    };
    std::vector<Node> tree(1);
    bool any = false;
    // (an empty stream, or one ending right after its last group, reads as the stop bit)
    while (pos < uint64_t(len) * 8 && get(1)) {
        uint32_t cnt = get(7);
        const uint32_t bl = get(4);
        while (cnt-- && !over) {
            const uint32_t key = get(8), word = get(bl);
            any = true;
            int cur = 0;
            const int steps = bl ? int(bl) : 1;
            for (int b = steps - 1; b >= 0; b--) {
                const int dir = bl ? int((word >> b) & 1u) : 0;
                if (tree[size_t(cur)].child[dir] < 0) {
                    tree[size_t(cur)].child[dir] = int(tree.size());
                    tree.emplace_back();
                }
                cur = tree[size_t(cur)].child[dir];
            }
            tree[size_t(cur)].sym = int(key);
        }
        if (over) return IE_EFORMAT;
    }
    if (over) return IE_EFORMAT;
    *code_start = pos;
    if (!any) return 1;  // no dictionary: the data follows uncompressed (Huffman.cpp:361-371)
    // lut[p] = sym | len << 8 for the leaf the 15-bit string p walks to (codes are <= 15 bits: a
    // 4-bit length field, Huffman.cpp:41-42); 0 where the walk leaves the tree
    constexpr int K = 15;
    std::fill(lut, lut + (size_t(1) << K), uint16_t(0));
    std::vector<std::pair<int, int>> stack{{0, 0}};
    std::vector<uint32_t> path(tree.size(), 0);
    while (!stack.empty()) {
        const auto [nd, depth] = stack.back();
        stack.pop_back();
        const Node& t = tree[size_t(nd)];
        if (t.child[0] < 0 && t.child[1] < 0) {
            if (depth == 0 || depth > K || t.sym < 0) continue;  // a lone root / over-long code: no entry
            const uint32_t lo = path[size_t(nd)] << (K - depth), span = 1u << (K - depth);
            for (uint32_t q = 0; q < span; q++) lut[lo + q] = uint16_t(uint32_t(t.sym) | (uint32_t(depth) << 8));
            continue;
        }
        for (int d = 0; d < 2; d++)
            if (t.child[d] >= 0) {
                path[size_t(t.child[d])] = (path[size_t(nd)] << 1) | uint32_t(d);
                stack.push_back({t.child[d], depth + 1});
            }
    }
    return IE_OK;
}

int ie_huffman_decode(ie_ctx* c, const uint8_t* in, size_t len, uint64_t start_bit, const uint16_t* lut,
                      uint8_t* out, size_t out_cap, size_t* nout) {
    if (!c || !in || !lut || !nout) return IE_EINVAL;
    *nout = 0;
    if (start_bit > uint64_t(len) * 8) return fail(c, IE_EINVAL, "start_bit beyond the stream");
    HIPCHK(c, hipSetDevice(c->device));
    int r;
    // the kernels read the stream only through their LDS staging, which stops at its last byte: a
    // 4-byte-aligned device stream is read in place, and a device table too (no copies)
    const uint8_t* src = in;
    if (!is_device_ptr(in) || reinterpret_cast<uintptr_t>(in) % 4) {
        const size_t padded = (len + 3) / 4 * 4 + 16;
        if ((r = ensure(c, c->d_dec, c->cap_dec, padded))) return r;
        if (len)
            HIPCHK(c, hipMemcpyAsync(c->d_dec, in, len, is_device_ptr(in) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                                     c->stream));
        src = c->d_dec;
    }
    const uint16_t* dlut = lut;
    if (!is_device_ptr(lut) || reinterpret_cast<uintptr_t>(lut) % 2) {
        if ((r = ensure(c, c->d_hlut, c->cap_hlut, size_t(32768)))) return r;
        HIPCHK(c, hipMemcpyAsync(c->d_hlut, lut, 32768 * sizeof(uint16_t),
                                 is_device_ptr(lut) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
        dlut = c->d_hlut;
    }
    const uint64_t nbits = uint64_t(len) * 8;
    // walk chunk of the Huffman decode; IE_HUF_CHUNK overrides (tuning aid).  1024 bits measured
    // best on a 4K payload (tools/gpu_huf_chunk.sh: 0.30-0.32 ms against 0.34 at 512, 0.37 at 768
    // and 2048, 0.55 at 4096)
    static const uint64_t huf_chunk = getenv("IE_HUF_CHUNK") ? strtoull(getenv("IE_HUF_CHUNK"), nullptr, 10) : 1024;
    // (at most 2048: the per-chunk symbol counts and middle offsets are u16, and huf_emit_kernel's
    // LDS grows ~33 bytes per chunk bit -- 4096-bit chunks would not fit gfx950's 160 KB)
    const uint64_t chunk_bits = std::min<uint64_t>(2048, std::max<uint64_t>(256, huf_chunk));
    const size_t nchunks = size_t((nbits - start_bit + chunk_bits - 1) / chunk_bits);
    if (!nchunks) return IE_OK;
    // d_walk: [cap] entries, [cap] symbol bases, then 128 words of top-level entries (256 x u32)
    if ((r = ensure(c, c->d_walk, c->cap_walk, 2 * nchunks + 130))) return r;
    // per-chunk symbol counts, then the walk workgroups' totals (ie::kTPB chunks each)
    if ((r = ensure(c, c->d_count, c->cap_count, nchunks + (nchunks + ie::kTPB - 1) / ie::kTPB + 1))) return r;
    if ((r = ensure(c, c->d_rtab, c->cap_rtab, ie::huffman_table_rows(nbits, start_bit, chunk_bits) + 2))) return r;
    uint64_t* wk = c->d_walk;
    const size_t cap = (c->cap_walk - 130) / 2;
    unsigned* flags = reinterpret_cast<unsigned*>(c->d_misc + 1);
    uint32_t* E = reinterpret_cast<uint32_t*>(wk + 2 * cap);
    unsigned* ticket = reinterpret_cast<unsigned*>(c->d_misc + 5);
    HIPCHK(c, hipMemsetAsync(c->d_misc, 0, 6 * sizeof(uint64_t), c->stream));
    const uint32_t* W = reinterpret_cast<const uint32_t*>(src);
    const int rounds = ie::huffman_decode_device(W, nbits, start_bit, dlut, chunk_bits, wk, c->d_rtab, E, ticket,
                                                 c->d_count, wk + cap, flags, c->d_misc + 2, nullptr, false,
                                                 c->stream);
    if (rounds < 0) return fail(c, IE_EHIP, "Huffman decode walk failed");
    HIPCHK(c, hipGetLastError());
    if (is_device_ptr(out)) {
        // device output: the emit follows at once, bounded by out_cap (a symbol past it is not
        // written and flags the launch), and the total and flags come back in ONE read
        ie::huffman_decode_device(W, nbits, start_bit, dlut, chunk_bits, wk, c->d_rtab, E, ticket, c->d_count,
                                  wk + cap, flags, c->d_misc + 2, out, true, c->stream, uint64_t(out_cap));
        HIPCHK(c, hipGetLastError());
        uint64_t rb[2] = {0, 0};  // d_misc[1]: the two flag words, d_misc[2]: the total
        HIPCHK(c, hipMemcpyAsync(rb, c->d_misc + 1, sizeof(rb), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        *nout = size_t(rb[1]);
        if (uint32_t(rb[0] >> 32)) return fail(c, IE_EFORMAT, "Huffman stream holds a bit string no code prefixes");
        if (rb[1] > out_cap) return fail(c, IE_ECAP, "output capacity below the decoded symbol count");
        return IE_OK;
    }
    uint64_t total = 0;
    HIPCHK(c, hipMemcpyAsync(&total, c->d_misc + 2, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *nout = size_t(total);
    if (total > out_cap) return fail(c, IE_ECAP, "output capacity below the decoded symbol count");
    const bool out_dev = is_device_ptr(out);
    uint8_t* dout = out;
    if (!out_dev) {
        if ((r = ensure(c, c->d_hout, c->cap_hout, size_t(total) + 1))) return r;
        dout = c->d_hout;
    }
    ie::huffman_decode_device(W, nbits, start_bit, dlut, chunk_bits, wk, c->d_rtab, E, ticket, c->d_count,
                              wk + cap, flags, c->d_misc + 2, dout, true, c->stream);
    HIPCHK(c, hipGetLastError());
    unsigned f[2] = {0, 0};
    HIPCHK(c, hipMemcpyAsync(f, flags, sizeof(f), hipMemcpyDeviceToHost, c->stream));
    if (!out_dev && total) HIPCHK(c, hipMemcpyAsync(out, dout, size_t(total), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (f[1]) return fail(c, IE_EFORMAT, "Huffman stream holds a bit string no code prefixes");
    return IE_OK;
}

}  // extern "C"

namespace {
// host pixel destinations: copy only the pixel rows (bytes between rows / frames belong to the caller)
int finish_decode(ie_ctx* c, uint8_t* out, const uint8_t* dpix, bool out_dev, int nframes, int w, int h, size_t stride,
                  size_t frame_pitch, uint64_t end, uint64_t* end_bit) {
    if (!out_dev) {
        for (int f = 0; f < nframes; f++)
            HIPCHK(c, hipMemcpy2D(out + size_t(f) * frame_pitch, stride, dpix + size_t(f) * frame_pitch, stride,
                                  size_t(w), size_t(h), hipMemcpyDeviceToHost));
    }
    if (end_bit) *end_bit = end;
    return IE_OK;
}

// Chunk plan of a record span (span bits from the first record, nblocks records) and the
// parse buffers it needs: fills a's chunking fields and scratch pointers, *levels = composition
// levels.  The record stream's own fields (words, nbits, start_bit, dstart, total, end_out) are
// the caller's.
#ifndef IE_GOP_CAPC
#define IE_GOP_CAPC 1  // 0: (A/B builds) gop decode chunks sized by the I-frame bound alone
#endif
int plan_records(ie_ctx* c, uint64_t span, uint64_t nblocks, ie::RecParseArgs& a, size_t* spec_at_out, int* levels_out,
                 uint64_t cmax = uint64_t(1) << 15) {
    const int n = c->n;
    int r;
    // chunking: about R records per chunk (IE_DEC_R; default 24 for 4x4, 28 for 8x8: measured
    // with 32-table composition groups on 4K noise / mixed / gradient / flat frames and the
    // reference's ex1 / ex4 -- 4x4 against 16, 24, 32, 48: ex4 126 -> 115 us, mixed 197 -> 191 us,
    // noise and flat unchanged; 8x8 against 20-32: noise 342 -> 258 us, ex1 376 -> 269 us,
    // gradient 209 -> 181 us, flat 101 -> 112 us; 8x8 noise alone is erratic in R, 2.6x slower at
    // 24) so that every chunk's walks are short; C a multiple of 32, at least
    // 256 bits, at most 2^15 (16-bit record positions; a table wave's LDS -- the chunk's bits and
    // valid-header bitmap -- stays small)
    const int G = ie::rec_group_chunks(n), D = ie::rec_entry_span(n);
    static const char* rs = getenv("IE_DEC_R");
    const uint64_t recs = rs ? std::max<uint64_t>(1, strtoull(rs, nullptr, 10)) : (n == 4 ? 24 : 28);
    const uint64_t want = std::max<uint64_t>((nblocks + recs - 1) / recs, 1);
    uint64_t C = (span + want - 1) / want;
    C = std::min<uint64_t>(std::max<uint64_t>((C + 31) / 32 * 32, 256), std::max<uint64_t>(cmax / 32 * 32, 256));
    const uint64_t nch = std::max<uint64_t>((span + C - 1) / C, 1);
    // levels: ceil(n / G) composites per level until at most G remain (G^4 chunks at most)
    size_t tab_rows = 0;
    int levels = 0;
    for (uint64_t cur = nch;; cur = (cur + G - 1) / G) {
        tab_rows += cur;
        levels++;
        if ((cur + G - 1) / G <= uint64_t(G)) {
            tab_rows += (cur + G - 1) / G;
            break;
        }
    }
    if (levels > ie::kRecMaxLevels || nch > uint64_t(INT32_MAX))
        return fail(c, IE_EINVAL, "stream too long for one decode call");
    const int nchunks = int(nch);
    if ((r = ensure(c, c->d_rtab, c->cap_rtab, tab_rows * D))) return r;
    // d_walk (8-byte words): [nchunks / 2] in-workgroup record bases, [G / 2] top-level entries,
    // [nchunks / 2] chunk counts, [nchunks / 2] count-pass workgroup totals (a workgroup covers at
    // least 4 chunks)
    const size_t e_at = size_t(nchunks) / 2 + 1, cnt_at = e_at + size_t(G) / 2 + 1;
    const size_t wg_at = cnt_at + size_t(nchunks) / 2 + 1;
    const size_t spec_at = wg_at + size_t(nchunks) / 2 + 2;  // [nchunks / 2] speculative exits
    if ((r = ensure(c, c->d_walk, c->cap_walk, spec_at + size_t(nchunks) / 2 + 1))) return r;
    if ((r = ensure(c, c->d_rpos, c->cap_rpos, size_t(nchunks) * ie::kRecPosCap))) return r;
    a.C = uint32_t(C);
    a.nchunks = nchunks;
    a.tab = c->d_rtab;
    a.seg = ie::rec_count_seg(uint32_t(C));
    a.lbase = reinterpret_cast<uint32_t*>(c->d_walk);
    a.wgsum = reinterpret_cast<uint32_t*>(c->d_walk + wg_at);
    a.E = reinterpret_cast<uint32_t*>(c->d_walk + e_at);
    a.cnt = reinterpret_cast<uint32_t*>(c->d_walk + cnt_at);
    a.pos = c->d_rpos;
    a.ticket = reinterpret_cast<unsigned*>(c->d_misc + 1);
    if (spec_at_out) *spec_at_out = spec_at;
    *levels_out = levels;
    return IE_OK;
}

// add_base: P-frame error -- the decoded error is added to the pixels already in `out`
#if IE_PROFILE  // host-side phase times of the record decode (IE_DEC_HOST=1): entry, launches, sync
struct DecHostTimes {
    double pre = 0, launch = 0, sync = 0;
    long n = 0;
    ~DecHostTimes() {
        if (n) fprintf(stderr, "[dec host] %ld calls: before the first launch %.1f us, launches %.1f us, sync %.1f us\n", n,
                       pre / n, launch / n, sync / n);
    }
};
static DecHostTimes g_dht;
static double dht_now() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define DHT(x) const double x = dht_now()
#else
#define DHT(x)
#endif
int decode_frames_impl(ie_ctx* c, const uint8_t* in, size_t len, uint64_t start_bit, int w, int h, int nframes,
                       int use_rle, uint8_t* out, size_t stride, size_t frame_pitch, uint64_t* end_bit, int add_base) {
    DHT(t0);
    int r = check_dims(c, w, h, nframes);
    if (r) return r;
    if (stride < size_t(w)) return fail(c, IE_EINVAL, "stride < width");
    if (nframes > 1 && frame_pitch < stride * size_t(h - 1) + size_t(w))
        return fail(c, IE_EINVAL, "frame_pitch smaller than a frame");
    if (start_bit > uint64_t(len) * 8) return fail(c, IE_EINVAL, "start_bit beyond the stream");
    HIPCHK(c, hipSetDevice(c->device));
    const int n = c->n;
    // stream: a 16-byte aligned device stream is read in place (the kernels read it with 16-byte
    // vector loads of whole aligned words up to the one holding the last byte -- never past its
    // page -- and clear the bits past the stream themselves); anything else is staged (device
    // copy or H2D) with zero padding
    const uint8_t* words = in;
    if (!is_device_ptr(in) || (reinterpret_cast<uintptr_t>(in) & 15u)) {
        const size_t padded = (len + 3) / 4 * 4 + 16;
        if ((r = ensure(c, c->d_dec, c->cap_dec, padded))) return r;
        HIPCHK(c, hipMemsetAsync(c->d_dec + (len / 4) * 4, 0, padded - (len / 4) * 4, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->d_dec, in, len, is_device_ptr(in) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                                 c->stream));
        words = c->d_dec;
    }
    const uint64_t nbits = uint64_t(len) * 8;
    const uint64_t span = nbits - start_bit;
    const uint64_t nblocks = uint64_t(nframes) * (w / n) * (h / n);
    ie::RecParseArgs pa{};
    size_t spec_at = 0;
    int levels = 0;
    if ((r = plan_records(c, span, nblocks, pa, &spec_at, &levels))) return r;
    const int nchunks = pa.nchunks;
    const size_t pix_bytes = size_t(nframes - 1) * frame_pitch + stride * size_t(h - 1) + size_t(w);
    const bool out_dev = is_device_ptr(out);
    uint8_t* dpix = out;
    if (!out_dev) {
        if ((r = ensure(c, c->d_pix, c->cap_pix, pix_bytes))) return r;
        dpix = c->d_pix;
    }
    ie::DecArgs da{};
    da.add_base = add_base;
    da.nframes = nframes;
    da.bx = w / n;
    da.by = h / n;
    da.rle = use_rle ? 1 : 0;
    da.out = dpix;
    da.stride = stride;
    da.frame_pitch = frame_pitch;
    da.tab = c->d_tab;
    pa.words = reinterpret_cast<const uint32_t*>(words);
    pa.nbits = nbits;
    pa.start_bit = start_bit;
    pa.rle = da.rle;
    if (!c->h_decres) {
        void* hp = nullptr;
        HIPCHK(c, hipHostMalloc(&hp, 64, hipHostMallocMapped | hipHostMallocCoherent));
        c->h_decres = static_cast<uint64_t*>(hp);
        void* dp = nullptr;
        HIPCHK(c, hipHostGetDevicePointer(&dp, hp, 0));
        c->d_decres = static_cast<uint64_t*>(dp);
    }
    pa.total = c->d_decres + 1;
    pa.end_out = c->d_decres;
    // (d_misc needs no clearing: the last chunk's decode wave always writes the record total, and
    // the end bit is read only when that total covers the last block, whose decode writes it)
#if IE_PROFILE  // walk statistics of the table pass (profiling builds only)
    static const bool dstats = getenv("IE_DEC_STATS") != nullptr;
    if (dstats) {
        pa.stats = reinterpret_cast<unsigned long long*>(c->d_misc + 3);  // [3..7]
        HIPCHK(c, hipMemsetAsync(c->d_misc + 3, 0, 5 * sizeof(uint64_t), c->stream));
    }
    static const char* dstamps = getenv("IE_DEC_STAMPS");  // file: [table waves][8] u64 per call
    uint64_t* d_ws = nullptr;
    int tm_ = 1, hb_ = 0;
    ie::rec_table_geometry(pa.C, n, &tm_, &hb_);
    const size_t nws = size_t(nchunks + tm_ - 1) / size_t(tm_) * 8;
    if (dstamps) {
        HIPCHK(c, hipMalloc(&d_ws, nws * 8));
        HIPCHK(c, hipMemsetAsync(d_ws, 0, nws * 8, c->stream));
        pa.wstamp = reinterpret_cast<unsigned long long*>(d_ws);
    }
#endif
    DHT(t1);
    // Optional speculative parse first (ie_decode.hip rec_spec_kernel; ie_set_exact_parse(ctx, 0)
    // or IE_DEC_SPEC=1): each chunk's entry is where a walk from an earlier chunk's first bit left
    // it, verified by the count pass; on any mismatch (e.g. periodic content, whose wrong-phase
    // walks never meet the true path) nothing was decoded and the exact parse over composed
    // transfer tables runs.  Off by default: measured on 4K frames and the reference's example
    // images it wins only on flat content -- a wrong-phase walk takes ~35 steps to
    // meet the true path and the slowest of ~16 000 chunks sets the pass's time.
    static const char* es = getenv("IE_DEC_SPEC");
    const bool spec = (es && atoi(es) != 0) || c->spec_parse;
    bool exact = !spec;
    c->last_spec = 0;
    if (spec) {
        pa.spec = reinterpret_cast<uint32_t*>(c->d_walk + spec_at);
        pa.fail = reinterpret_cast<unsigned*>(c->d_misc + 2);
        // warm-up chunks: a speculative walk crosses this many whole chunks (about 32 (4x4) / 16
        // (8x8) records each) before the chunk whose exit it reports (IE_DEC_WARM)
        static const char* ew = getenv("IE_DEC_WARM");
        const int warm = c->spec_warm ? c->spec_warm : (ew ? std::max(0, std::min(8, atoi(ew))) : 0);
        // rec_spec_kernel stages seg + warm chunks per wave in LDS: keep a wave within 12 KB
        const int room = int((uint64_t(12 * 1024) * 8 - 256) / uint64_t(pa.C)) - pa.seg;
        pa.warm = std::max(0, std::min(warm, room));
        ie::launch_rec_spec_decode(pa, da, n, c->stream);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->h_decres[1] == ~0ull) {
            exact = true;
            pa.spec = nullptr;
            pa.fail = nullptr;
        } else {
            c->last_spec = 1;
            levels = 0;
        }
    }
    DHT(t2);
    if (exact) {
        if (ie::launch_rec_parse_decode(pa, da, n, c->stream) < 0) return fail(c, IE_EINVAL, "stream too long for one decode call");
        HIPCHK(c, hipGetLastError());
    }
    c->last_chunks = nchunks;
    c->last_groups = levels;
    HIPCHK(c, hipStreamSynchronize(c->stream));
#if IE_PROFILE
    {
        DHT(t3);
        g_dht.pre += t1 - t0;
        g_dht.launch += t2 - t1;
        g_dht.sync += t3 - t2;
        g_dht.n++;
    }
#endif
    const uint64_t end = c->h_decres[0], total = c->h_decres[1];
#if IE_PROFILE
    if (dstats) {
        uint64_t st[5];
        HIPCHK(c, hipMemcpy(st, c->d_misc + 3, sizeof(st), hipMemcpyDeviceToHost));
        fprintf(stderr, "[dec] chunks %d C %u: lane-steps %.1f/chunk, beyond-window %.1f/chunk, unmerged walks %.2f/chunk, "
                "wave max steps avg %.1f max %llu\n", nchunks, unsigned(pa.C), double(st[0]) / nchunks, double(st[1]) / nchunks,
                double(st[2]) / nchunks, double(st[3]) / nchunks, (unsigned long long)st[4]);
        HIPCHK(c, hipMemsetAsync(c->d_misc + 3, 0, sizeof(uint64_t), c->stream));
    }
    if (d_ws) {
        std::vector<uint64_t> hws(nws);
        HIPCHK(c, hipMemcpy(hws.data(), d_ws, nws * 8, hipMemcpyDeviceToHost));
        HIPCHK(c, hipFree(d_ws));
        if (FILE* f = fopen(dstamps, "ab")) {
            fwrite(hws.data(), 8, nws, f);
            fclose(f);
        }
    }
#endif
    if (total < nblocks || end > nbits) return fail(c, IE_EFORMAT, "stream ends before the last block");
    return finish_decode(c, out, dpix, out_dev, nframes, w, h, stride, frame_pitch, end, end_bit);
}
}  // namespace

extern "C" {

int ie_decode_frames(ie_ctx* c, const uint8_t* in, size_t len, uint64_t start_bit, int w, int h, int nframes,
                     int use_rle, uint8_t* out, size_t stride, size_t frame_pitch, uint64_t* end_bit) {
    if (!c || !in || !out) return IE_EINVAL;
    return decode_frames_impl(c, in, len, start_bit, w, h, nframes, use_rle, out, stride, frame_pitch, end_bit, 0);
}

// Video decode with P-frames (VideoDecoder.cpp:28-58, Frame.cpp:47-127): frame by frame, each
// starting at the previous frame's end; a P-frame's motion vectors and reference-block copies
// (pf_mvcopy_kernel), then its records (every microblock's) decoded onto the copied pixels.
// Device-chained: every frame's launches read its first bit from the device word the previous
// frame's decode wrote (pos[f], RecParseArgs::dstart), with chunks planned from the frame's bound
// rather than its span, so the whole call is enqueued at once and the host waits once, at the end,
// for the end bits and record totals it checks.
int ie_decode_gop(ie_ctx* c, const uint8_t* in, size_t len, uint64_t start_bit, int w, int h, int nframes, int gop,
                  int merange, int use_rle, int motioncomp, uint8_t* out, size_t stride, size_t frame_pitch,
                  uint64_t* end_bit) {
    if (!c || !in || !out) return IE_EINVAL;
    int r = check_dims(c, w, h, nframes);
    if (r) return r;
    gop = std::max(1, gop);
    if (merange < 0 || merange > 32767) return fail(c, IE_EINVAL, "merange must be in [0, 32767]");
    if (stride < size_t(w)) return fail(c, IE_EINVAL, "stride < width");
    if (nframes > 1 && frame_pitch < stride * size_t(h - 1) + size_t(w))
        return fail(c, IE_EINVAL, "frame_pitch smaller than a frame");
    if (gop > 1 && nframes > 1 && (w % 16 || h % 16))
        return fail(c, IE_EINVAL, "P-frames decode for W and H multiples of 16 only: the reference's macroblocks are "
                                  "misplaced otherwise and its uncovered microblocks read records never written");
    if (start_bit > uint64_t(len) * 8) return fail(c, IE_EINVAL, "start_bit beyond the stream");
    HIPCHK(c, hipSetDevice(c->device));
    // the stream once on the device (16-byte aligned, zero padding for the vector reads), the
    // frames decoded into a device buffer (P-frames read their predecessor there)
    const size_t padded = (len + 3) / 4 * 4 + 16;
    if ((r = ensure(c, c->d_in, c->cap_in, padded))) return r;
    HIPCHK(c, hipMemsetAsync(c->d_in + (len / 4) * 4, 0, padded - (len / 4) * 4, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_in, in, len, is_device_ptr(in) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                             c->stream));
    const bool out_dev = is_device_ptr(out);
    const size_t pix_bytes = size_t(nframes - 1) * frame_pitch + stride * size_t(h - 1) + size_t(w);
    uint8_t* dpix = out;
    if (!out_dev) {
        if ((r = ensure(c, c->d_gop_rec, c->cap_gop_rec, pix_bytes))) return r;
        dpix = c->d_gop_rec;
    }
    const int n = c->n, mv = mvec_bits(merange);
    const uint64_t nbits = uint64_t(len) * 8;
    const uint64_t nmb = uint64_t(w / 16) * (h / 16), mvb = nmb * 2u * uint64_t(mv);
    const uint64_t nblocks = uint64_t(w / n) * (h / n);
    const uint64_t rec_bound = nblocks * bound_bits_per_block(n);
    // per-frame device words: pos[0..nframes] first bits (pos[f + 1] = frame f's end), tot[f]
    // records on frame f's true path; then the host copy of both
    const size_t nw = 2 * size_t(nframes) + 1;
    if ((r = ensure(c, c->d_gop_pos, c->cap_gop_pos, nw))) return r;
    uint64_t* pos = c->d_gop_pos;
    uint64_t* tot = pos + nframes + 1;
    ie::launch_gop_init(pos, tot, nframes, start_bit, c->stream);
    HIPCHK(c, hipGetLastError());
    // one chunk plan for every frame: its bound (plus a P-frame's vectors), so the grids and
    // scratch do not depend on where a frame ends
    ie::RecParseArgs pa{};
    int levels = 0;
    // (gop > 1: the plan is sized by the I-frame bound, but a P-frame's records are a few bits each
    // -- at most kRecPosCap records per chunk (5 bits each at least with RLE: 4 header bits and
    // one value bit) keeps its chunks on the listed-positions decode instead of the re-walk)
    const uint64_t min_rec = use_rle ? 5u : uint64_t(4 + n * n);
    const uint64_t cmax = (gop > 1 && IE_GOP_CAPC) ? uint64_t(ie::kRecPosCap) * min_rec : (uint64_t(1) << 15);
    if ((r = plan_records(c, rec_bound, nblocks, pa, nullptr, &levels, cmax))) return r;
    pa.words = reinterpret_cast<const uint32_t*>(c->d_in);
    pa.nbits = nbits;
    pa.rle = use_rle ? 1 : 0;
    pa.span = rec_bound;
    if (gop > 1 && nframes > 1 && !motioncomp)
        if ((r = ensure(c, c->d_gop_coef, c->cap_gop_coef, (stride * size_t(h) + 1) / 2))) return r;
    for (int f = 0; f < nframes; f++) {
        uint8_t* fo = dpix + size_t(f) * frame_pitch;
        const bool iframe = (f % gop) == 0;
        if (!iframe) {
            ie::launch_pframe_mvcopy(c->d_in, 0, pos + f, nbits, mv, fo - frame_pitch, stride, fo, stride, w, h, c->stream);
            HIPCHK(c, hipGetLastError());
        }
        ie::DecArgs da{};
        da.nframes = 1;
        da.bx = w / n;
        da.by = h / n;
        da.rle = pa.rle;
        da.tab = c->d_tab;
        if (!iframe && !motioncomp) {
            // the error is read (the stream must be consumed) but not applied: decode into scratch
            da.out = reinterpret_cast<uint8_t*>(c->d_gop_coef);
            da.add_base = 0;
        } else {
            da.out = fo;
            da.add_base = iframe ? 0 : 1;
        }
        da.stride = stride;
        da.frame_pitch = 0;
        pa.dstart = pos + f;
        pa.start_add = iframe ? 0 : mvb;
        pa.total = tot + f;
        pa.end_out = pos + f + 1;
        if (ie::launch_rec_parse_decode(pa, da, n, c->stream) < 0) return fail(c, IE_EINVAL, "stream too long for one decode call");
        HIPCHK(c, hipGetLastError());
    }
    std::vector<uint64_t> hp(nw);
    HIPCHK(c, hipMemcpyAsync(hp.data(), pos, nw * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->last_chunks = pa.nchunks;
    c->last_groups = levels;
    c->last_spec = 0;
    for (int f = 0; f < nframes; f++) {
        if ((f % gop) != 0 && hp[f] + mvb > nbits) return fail(c, IE_EFORMAT, "stream ends in the motion vectors");
        if (hp[nframes + 1 + f] < nblocks || hp[f + 1] > nbits) return fail(c, IE_EFORMAT, "stream ends before the last block");
    }
    if (!out_dev)
        for (int f = 0; f < nframes; f++)
            HIPCHK(c, hipMemcpy2D(out + size_t(f) * frame_pitch, stride, dpix + size_t(f) * frame_pitch, stride,
                                  size_t(w), size_t(h), hipMemcpyDeviceToHost));
    if (end_bit) *end_bit = hp[nframes];
    return IE_OK;
}

}  // extern "C"
