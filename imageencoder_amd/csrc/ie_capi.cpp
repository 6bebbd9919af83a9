// imageencoder_amd/csrc/ie_capi.cpp -- the extern "C" boundary (include/ie_hip.h): context,
// quantisation tables, buffer staging and kernel launches.  Host code; compiled with hipcc.
#include "ie_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ie_device.h"

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
    uint64_t* d_state = nullptr;  // [2 * cap_tiles]
    size_t cap_tiles = 0;
    uint32_t tag = 0;
    unsigned long long* d_ticket = nullptr;
    unsigned long long ticket_base = 0;

    uint64_t* d_frame_start = nullptr;  // [cap_frames]
    uint64_t* d_chain_end = nullptr;    // [cap_frames]
    size_t cap_frames = 0;
    unsigned* d_err = nullptr;          // [0] look-back timeouts, [1] fallbacks

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
};

namespace {

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

inline double Cf(int i) { return i == 0 ? 0.5 : M_SQRT1_2; }  // algo.cpp:294-297

// Build the per-matrix tables.  The cos values are the reference's own expression evaluated
// with the host libm (algo.cpp:312,318-319); P, S and R are the double products it forms.
// thr[k] bounds |t32 - T| where t32 is the kernel's FP32 quotient for coefficient k and T the
// reference's FP64 quotient: a forward error bound of the separable FMA chains of
// encode_kernel (row pass over j, column pass over i, one scale), for |x| <= 128, doubled.
void build_tables(int n, const uint16_t* q, ie::EncTables* T) {
    const int nn = n * n;
    std::memset(T, 0, sizeof(*T));
    const double factor = M_PI_2 / double(n);
    for (int u = 0; u < n; u++)
        for (int i = 0; i < n; i++) T->c[u * n + i] = std::cos(double(2.0 * i + 1.0) * double(u) * factor);
    for (int u = 0; u < n; u++)
        for (int v = 0; v < n; v++) {
            const int k = u * n + v;
            T->S[k] = Cf(u) * Cf(v);
            T->qd[k] = double(q[k]);
            for (int i = 0; i < n; i++)
                for (int j = 0; j < n; j++) {
                    T->P[k * nn + i * n + j] = T->c[u * n + i] * T->c[v * n + j];
                    T->R[k * nn + i * n + j] = Cf(u) * Cf(v) * T->c[u * n + i] * T->c[v * n + j];
                }
        }
    for (int k = 0; k < nn; k++) T->cf[k] = float(T->c[k]);

    const double uf = std::ldexp(1.0, -24), X = 128.0;
    double My[8], Ey[8];
    bool exy[8];
    for (int v = 0; v < n; v++) {
        double M = 0, E = 0;
        bool ex = true;
        for (int j = 0; j < n; j++) {
            const double cd = T->c[v * n + j], dc = std::fabs(double(T->cf[v * n + j]) - cd);
            ex = ex && (cd == 1.0);
            M += std::fabs(cd) * X;
            E += dc * X;
            if (!ex) E += uf * (M + E);
        }
        My[v] = M;
        Ey[v] = ex ? 0.0 : E;
        exy[v] = ex;
    }
    for (int u = 0; u < n; u++)
        for (int v = 0; v < n; v++) {
            const int k = u * n + v;
            double M = 0, E = 0;
            bool ex = exy[v];
            for (int i = 0; i < n; i++) {
                const double cd = T->c[u * n + i], cfv = T->cf[u * n + i];
                ex = ex && (cd == 1.0);
                M += std::fabs(cd) * My[v];
                E += std::fabs(cfv) * Ey[v] + std::fabs(cfv - cd) * My[v];
                if (!ex) E += uf * (M + E);
            }
            const double sq = T->S[k] / T->qd[k];
            const float g = float(sq);
            T->g[k] = g;
            const double dg = std::fabs(double(g) - sq) + 1e-15 * sq;
            double bound = std::fabs(double(g)) * E + M * dg + uf * std::fabs(double(g)) * (M + E);
            // the reference's own FP64 rounding (<= NN terms of |P x| <= 128, relative 2^-53 each)
            bound += 1e-9;
            // exact when every step is: integer sums (rows/cols of ones), a power-of-two scale and
            // divisor, so both the reference and the FP32 path compute the quotient exactly
            int e2 = 0;
            const double m2 = std::frexp(sq, &e2);
            const bool pow2 = (m2 == 0.5);
            if (ex && pow2 && double(g) == sq) {
                T->thr[k] = -1.0f;
            } else {
                T->thr[k] = float(2.0 * bound);
            }
        }
}

int prepare_state(ie_ctx* c, int ntiles, int nframes) {
    if (size_t(ntiles) > c->cap_tiles) {
        if (c->d_state) {
            HIPCHK(c, hipStreamSynchronize(c->stream));
            HIPCHK(c, hipFree(c->d_state));
        }
        const size_t cap = std::max<size_t>(ntiles, c->cap_tiles * 2);
        HIPCHK(c, hipMalloc(&c->d_state, 2 * cap * sizeof(uint64_t)));
        HIPCHK(c, hipMemsetAsync(c->d_state, 0, 2 * cap * sizeof(uint64_t), c->stream));
        c->cap_tiles = cap;
        c->tag = 0;
    }
    c->tag++;
    if (c->tag > 255) {
        HIPCHK(c, hipMemsetAsync(c->d_state, 0, 2 * c->cap_tiles * sizeof(uint64_t), c->stream));
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
    HIPCHK(c, hipMemsetAsync(c->d_err, 0, 2 * sizeof(unsigned), c->stream));
    return IE_OK;
}

struct Geometry {
    int bx, by, gpr, gpf, tpf, ntiles;
};

Geometry geometry(int w, int h, int n, int nframes) {
    Geometry g;
    const int bpt = (n == 4) ? 4 : 1;
    g.bx = w / n;
    g.by = h / n;
    g.gpr = (g.bx + bpt - 1) / bpt;
    g.gpf = g.gpr * g.by;
    g.tpf = (g.gpf + ie::kTPB - 1) / ie::kTPB;
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

// Common driver of ie_encode_frames (segmented = 0) and ie_encode_images (segmented = 1).
int encode(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
           int use_rle, int mode, uint8_t* out, size_t out_cap, size_t out_pitch, uint64_t start_bit,
           int segmented, uint64_t* frame_bits, uint64_t* end_bits, int16_t* coef = nullptr) {
    int r = check_dims(c, w, h, nframes);
    if (r) return r;
    if (stride < size_t(w)) return fail(c, IE_EINVAL, "stride < width");
    if (nframes > 1 && frame_pitch < stride * size_t(h - 1) + size_t(w))
        return fail(c, IE_EINVAL, "frame_pitch smaller than a frame");
    if (segmented && (out_pitch % 4)) return fail(c, IE_EINVAL, "out_pitch must be a multiple of 4");
    HIPCHK(c, hipSetDevice(c->device));
    const Geometry g = geometry(w, h, c->n, nframes);
    const int nchains = segmented ? nframes : 1;

    // input
    const size_t in_bytes = size_t(nframes - 1) * frame_pitch + stride * size_t(h - 1) + size_t(w);
    const uint8_t* dy = y;
    if (!is_device_ptr(y)) {
        if ((r = ensure(c, c->d_in, c->cap_in, in_bytes))) return r;
        HIPCHK(c, hipMemcpyAsync(c->d_in, y, in_bytes, hipMemcpyHostToDevice, c->stream));
        dy = c->d_in;
    }
    const int bpt = (c->n == 4) ? 4 : 1;
    const bool vec_ok = (reinterpret_cast<uintptr_t>(dy) % 16 == 0) && (stride % (bpt * c->n) == 0) &&
                        (nframes == 1 || frame_pitch % (bpt * c->n) == 0);

    // output
    const uint64_t payload_bound = uint64_t(g.bx) * g.by * bound_bits_per_block(c->n) * (segmented ? 1 : nframes);
    const uint64_t end_bound = start_bit + payload_bound;
    const size_t need_bytes = size_t((end_bound + 31) / 32) * 4;
    const size_t span = segmented ? out_pitch * size_t(nframes - 1) + need_bytes : need_bytes;
    if (segmented && out_pitch < need_bytes) return fail(c, IE_ECAP, "out_pitch below ie_stream_bound");
    if (out_cap < span) return fail(c, IE_ECAP, "output capacity below ie_stream_bound");
    const bool out_dev = is_device_ptr(out);
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

    if ((r = prepare_state(c, g.ntiles, nframes))) return r;
    ie::EncArgs a{};
    a.y = dy;
    a.stride = stride;
    a.frame_pitch = frame_pitch;
    a.w = w;
    a.h = h;
    a.nframes = nframes;
    a.bx = g.bx;
    a.by = g.by;
    a.gpr = g.gpr;
    a.groups_per_frame = g.gpf;
    a.tiles_per_frame = g.tpf;
    a.ntiles = g.ntiles;
    a.rle = use_rle ? 1 : 0;
    a.segmented = segmented;
    a.vec_ok = vec_ok ? 1 : 0;
    a.out = dout;
    a.out_pitch_words = segmented ? out_pitch / 4 : 0;
    a.start_bit = start_bit;
    a.st_agg = c->d_state;
    a.st_inc = c->d_state + c->cap_tiles;
    a.ticket = c->d_ticket;
    a.ticket_base = c->ticket_base;
    a.tag = c->tag;
    a.frame_start = c->d_frame_start;
    a.chain_end = c->d_chain_end;
    a.err = c->d_err;
    a.tab = c->d_tab;
    a.coef = coef;
    ie::launch_encode(a, c->n, mode == IE_MODE_EXACT, c->stream);
    HIPCHK(c, hipGetLastError());
    c->ticket_base += uint64_t(g.ntiles);

    const bool want = frame_bits || end_bits || !out_dev;
    if (!want) return IE_OK;
    std::vector<uint64_t> fs(nframes), ce(nchains);
    unsigned errs[2];
    HIPCHK(c, hipMemcpyAsync(fs.data(), c->d_frame_start, nframes * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(ce.data(), c->d_chain_end, nchains * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(errs, c->d_err, sizeof(errs), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->last_fallbacks = errs[1];
    if (errs[0]) return fail(c, IE_EDEVICE, "tile look-back timed out");
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
    if (r == IE_OK) chk(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking), "hipStreamCreate");
    c->stream = c->own;
    if (r == IE_OK) chk(hipMalloc(&c->d_tab, sizeof(ie::EncTables)), "hipMalloc(tables)");
    if (r == IE_OK) chk(hipHostMalloc(&c->h_tab, sizeof(ie::EncTables)), "hipHostMalloc(tables)");
    if (r == IE_OK) chk(hipMalloc(&c->d_ticket, sizeof(unsigned long long)), "hipMalloc(ticket)");
    if (r == IE_OK) chk(hipMemset(c->d_ticket, 0, sizeof(unsigned long long)), "hipMemset(ticket)");
    if (r == IE_OK) chk(hipMalloc(&c->d_err, 4 * sizeof(unsigned)), "hipMalloc(err)");
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
    (void)hipFree(c->d_tab);
    (void)hipHostFree(c->h_tab);
    (void)hipFree(c->d_state);
    (void)hipFree(c->d_ticket);
    (void)hipFree(c->d_frame_start);
    (void)hipFree(c->d_chain_end);
    (void)hipFree(c->d_err);
    (void)hipFree(c->d_in);
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_scratch);
    (void)hipFree(c->d_coef);
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
    return IE_OK;
}

int ie_set_quant(ie_ctx* c, const uint16_t* q, int n) {
    if (!c || !q) return IE_EINVAL;
    if (n != 4 && n != 8) return fail(c, IE_EINVAL, "block size must be 4 or 8");
    for (int k = 0; k < n * n; k++)
        if (q[k] == 0) return fail(c, IE_EINVAL, "quantisation matrix entries must be > 0");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));  // tables may be in use by a running launch
    build_tables(n, q, c->h_tab);
    HIPCHK(c, hipMemcpy(c->d_tab, c->h_tab, sizeof(ie::EncTables), hipMemcpyHostToDevice));
    c->n = n;
    std::memcpy(c->q, q, sizeof(uint16_t) * n * n);
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

int ie_encode_images(ie_ctx* c, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                     int use_rle, int mode, uint8_t* out, size_t out_pitch, uint64_t start_bit, uint64_t* end_bits) {
    if (!c || !y || !out) return IE_EINVAL;
    return encode(c, y, w, h, stride, frame_pitch, nframes, use_rle, mode, out, out_pitch * size_t(nframes),
                  out_pitch, start_bit, 1, nullptr, end_bits);
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
    unsigned errs[2];
    HIPCHK(c, hipMemcpyAsync(errs, c->d_err, sizeof(errs), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->last_fallbacks = errs[1];
    *count = errs[1];
    if (errs[0]) return fail(c, IE_EDEVICE, "tile look-back timed out");
    return IE_OK;
}

}  // extern "C"
