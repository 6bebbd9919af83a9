// oracle/ie_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see ie_oracle.h).
//
// A clean-room restatement of the reference's per-block codec, written from the specification
// in SURVEY.md Appendix A and checked bit-for-bit against golden vectors produced by the
// reference itself (oracle/_ref, tests/golden/).  Each function cites the reference lines whose
// behaviour it restates.  It is deliberately simple: FP64 in the reference's exact operation
// order (this file is compiled with -ffp-contract=off so no FMA can re-associate anything),
// a serial MSB-first bit writer, and the Huffman pass re-expressed with the same libstdc++
// containers the reference uses so that hash-map iteration order -- which decides the emitted
// dictionary order -- is reproduced.
#include "ie_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <queue>
#include <unordered_map>
#include <vector>

namespace {

// ---------------------------------------------------------------- bit IO (BitStream.cpp:14-77)
struct BitWriter {
    uint8_t* buf;
    size_t cap;  // bytes
    uint64_t pos;
    bool overflow = false;
    BitWriter(uint8_t* b, size_t c, uint64_t p) : buf(b), cap(c), pos(p) {}
    // put(len, val): the low `len` bits of val, MSB first (BitStream.cpp:73-77)
    void put(int len, uint32_t val) {
        for (int p = 0; p < len; p++) {
            const uint32_t bit = (val >> (len - 1 - p)) & 1u;
            const uint64_t byte = pos >> 3;
            if (byte >= cap) { overflow = true; pos++; continue; }
            const uint8_t m = uint8_t(1u << (7 - (pos & 7)));
            if (bit) buf[byte] |= m; else buf[byte] &= uint8_t(~m);
            pos++;
        }
    }
};

struct BitReader {
    const uint8_t* buf;
    size_t size;  // bytes
    uint64_t pos = 0;
    BitReader(const uint8_t* b, size_t s) : buf(b), size(s) {}
    // get_bit returns 0 past the end (BitStream.cpp:14-28)
    uint32_t bit() {
        const uint64_t byte = pos >> 3;
        if (byte >= size) return 0;
        const uint32_t v = (buf[byte] >> (7 - (pos & 7))) & 1u;
        pos++;
        return v;
    }
    uint32_t get(int l) {
        uint32_t v = 0;
        for (int i = 0; i < l; i++) v |= bit() << (l - i - 1);
        return v;
    }
};

// ffs = bit length; the reference computes 32 - __builtin_clz(v), which is undefined at 0 and
// yields 1 in every real build (utils.hpp:210-216).
inline int ffs_ref(uint32_t v) {
    if (v == 0) return 1;
    return 32 - __builtin_clz(v);
}

// utils.hpp:226-243, verbatim semantics
inline int bits_needed_ref(int16_t value) {
    int bits = 1;
    while (int16_t(int16_t((value & ((1 << bits) - 1)) << (16 - bits)) >> (16 - bits)) != value) bits++;
    return bits;
}

// utils.hpp:265-269
inline int16_t shift_signed16(uint32_t value, int src_bits) {
    const int sh = 16 - src_bits;
    return int16_t(int16_t(uint16_t(value << sh)) >> sh);
}

inline double C(int i) { return i == 0 ? 0.5 : M_SQRT1_2; }  // algo.cpp:294-297 (N=4 constants for every N)

struct Tables {
    int n;
    std::vector<double> c;    // c[u][i]
    std::vector<double> P;    // P[(u*n+v)*n*n + i*n+j] = c[u][i]*c[v][j]            (fwd term)
    std::vector<double> S;    // S[u*n+v] = C(u)*C(v)
    std::vector<double> R;    // R[(u*n+v)*n*n + i*n+j] = ((C(u)*C(v))*c[u][i])*c[v][j] (inv term)
    std::vector<int> zz;      // zig-zag -> row-major index
    explicit Tables(int n_) : n(n_) {
        const int nn = n * n;
        c.resize(nn);
        ieo_cos_table(n, c.data());
        P.resize(size_t(nn) * nn);
        R.resize(size_t(nn) * nn);
        S.resize(nn);
        for (int u = 0; u < n; u++)
            for (int v = 0; v < n; v++) {
                S[u * n + v] = C(u) * C(v);
                for (int i = 0; i < n; i++)
                    for (int j = 0; j < n; j++) {
                        P[size_t(u * n + v) * nn + i * n + j] = c[u * n + i] * c[v * n + j];
                        R[size_t(u * n + v) * nn + i * n + j] = C(u) * C(v) * c[u * n + i] * c[v * n + j];
                    }
            }
        zz.resize(nn);
        ieo_zigzag(n, zz.data());
    }
};

// Block<N>::processDCTDivQ (Block.cpp:139-153) + algo::transformDCT (algo.cpp:309-331).
void quantize_block(const Tables& T, const uint8_t* p, size_t stride, const double* qd, int16_t* out) {
    const int n = T.n, nn = n * n;
    double x[64];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) x[i * n + j] = double(p[i * stride + j]) + double(-128);
    for (int uv = 0; uv < nn; uv++) {
        const double* Puv = &T.P[size_t(uv) * nn];
        double acc = 0.0;
        for (int k = 0; k < nn; k++) acc = acc + Puv[k] * x[k];
        const double D = acc * T.S[uv];
        out[uv] = int16_t(std::round(D / qd[uv]));
    }
}

struct BlockCode {
    int bl;   // field width (only the low 4 bits are stored)
    int lw;   // number of coefficient fields emitted
};

// Block::createRLESequence (Block.cpp:186-232) + the length rule of streamEncoded (:383-397).
BlockCode size_block(const Tables& T, const int16_t* coef, int rle) {
    const int nn = T.n * T.n;
    int L = 0, maxbits = 0;
    for (int k = 0; k < nn; k++) {
        const int16_t v = coef[T.zz[k]];
        if (v != 0) {
            L = k + 1;
            maxbits = std::max(maxbits, bits_needed_ref(v));
        }
    }
    BlockCode bc;
    bc.bl = std::max(maxbits, ffs_ref(uint32_t(L)));
    if (!rle) {
        bc.lw = nn;
    } else if (L == nn && coef[T.zz[nn - 2]] == 0) {
        // the last data element and the zeroes before it are dropped (Block.cpp:388-390)
        int prev = 0;
        for (int k = 0; k < nn - 1; k++)
            if (coef[T.zz[k]] != 0) prev = k + 1;
        bc.lw = prev;
    } else {
        bc.lw = L;
    }
    return bc;
}

// Block::streamEncoded (Block.cpp:372-413)
void emit_block(const Tables& T, const int16_t* coef, int rle, BitWriter& w) {
    const BlockCode bc = size_block(T, coef, rle);
    w.put(4, uint32_t(bc.bl));
    if (rle) w.put(bc.bl, uint32_t(bc.lw));
    for (int k = 0; k < bc.lw; k++) w.put(bc.bl, uint32_t(int32_t(coef[T.zz[k]])));
}

int64_t encode_frames(const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                      int n, const uint16_t* q, int rle, uint8_t* out, size_t cap, uint64_t start_bit,
                      uint64_t* frame_bits) {
    if ((n != 4 && n != 8) || w <= 0 || h <= 0 || w % n || h % n) return -1;
    Tables T(n);
    const int nn = n * n;
    double qd[64];
    for (int k = 0; k < nn; k++) qd[k] = double(q[k]);
    const int bx = w / n, by = h / n;
    const size_t nb = size_t(bx) * by;
    std::vector<int16_t> coef(nb * nn);
    BitWriter wr(out, cap, start_bit);
    for (int f = 0; f < nframes; f++) {
        const uint8_t* fy = y + size_t(f) * frame_pitch;
        // block (bx_, by_) row r starts at buf + by_*n*n*bx + bx_*n + r*w (ImageBase.cpp:187-194)
#pragma omp parallel for schedule(static)
        for (long b = 0; b < long(nb); b++) {
            const int bxi = int(b % bx), byi = int(b / bx);
            quantize_block(T, fy + size_t(byi) * n * stride + size_t(bxi) * n, stride, qd, &coef[size_t(b) * nn]);
        }
        const uint64_t s = wr.pos;
        for (size_t b = 0; b < nb; b++) emit_block(T, &coef[b * nn], rle, wr);
        if (frame_bits) frame_bits[f] = wr.pos - s;
    }
    if (wr.overflow) return -2;
    return int64_t(wr.pos);
}

// ------------------------------------------------------------ P-frames (gop > 1)
// The 9-point pattern of algo.cpp:90-100 (index 0 = the centre).
const int kMerSx[9] = {0, 1, 1, 0, -1, -1, -1, 0, 1};
const int kMerSy[9] = {0, 0, 1, 1, 1, 0, -1, -1, -1};
constexpr int kMB = 16;  // dc::MacroBlockSize (Block.hpp:14)

inline int clamp_i16(int v, int lo, int hi) { return int(std::clamp(int16_t(v), int16_t(lo), int16_t(hi))); }

// sum |cur - ref| over the 16x16 macroblock (Block.cpp:241-254)
uint64_t mb_sad(const uint8_t* cur, size_t cs, const uint8_t* ref, size_t rs) {
    uint64_t d = 0;
    for (int y = 0; y < kMB; y++)
        for (int x = 0; x < kMB; x++) d += uint64_t(std::abs(int(cur[y * cs + x]) - int(ref[y * rs + x])));
    return d;
}

// One P-frame (Frame.cpp:160-243): motion search per macroblock (Block.cpp:267-339 over the
// pattern tree of algo.cpp:119-139, walked without materialising it: child p of the node at
// (x, y) with radius r sits at (x + sx[p] r, y + sy[p] r), radius r / 2; r == 0 is a leaf),
// the prediction error per 4x4 microblock through processDCTDivQ / createRLESequence /
// processIDCTMulQ (ImageBase.cpp:266-306), the reference block copied into the frame
// (copyBlockMatrixTo) and expandDifferences (Block.cpp:110-119) over every microblock.
// cur is read, rec receives the frame as the reference leaves it in its buffer (the next frame's
// reference).  Writes the mvecs, then the microblock records.
void pframe(const Tables& T, const double* qd, const uint8_t* cur, size_t cs, const uint8_t* ref, size_t rs,
            uint8_t* rec, int w, int h, int rle, int merange, BitWriter& wr) {
    const int n = T.n, nn = n * n;
    const int mbx = w / kMB, mby = h / kMB;  // ImageBase.cpp:213-214 (floor)
    const int bx = w / n;
    const int mv_bits = bits_needed_ref(int16_t(merange));  // VideoBase.cpp:42
    // microblocks are built BEFORE any macroblock copy: expanded = the frame's own pixels
    std::vector<double> E(size_t(w) * h);
    for (size_t i = 0; i < size_t(w) * h; i++) E[i] = double(cur[(i / w) * cs + i % w]);
    std::vector<uint8_t> M(size_t(w) * h);  // the frame buffer (matrix) as the macroblock loop leaves it
    for (int y = 0; y < h; y++) std::memcpy(&M[size_t(y) * w], cur + size_t(y) * cs, size_t(w));
    std::vector<int16_t> coef(size_t(bx) * (h / n) * nn, 0);
    std::vector<char> has_rle(size_t(bx) * (h / n), 0);
    // micro_per_macro_row (ImageBase.cpp:271): integer division, 0 for 8x8 blocks
    const int mpr = (kMB * kMB / nn) / n;
    for (int mb = 0; mb < mbx * mby; mb++) {
        const int mx = (mb % mbx) * kMB, my = (mb / mbx) * kMB;
        const uint8_t* cb = cur + size_t(my) * cs + mx;
        // search: the first best block is the one at ABSOLUTE (0, 0) (Block.cpp:272-274)
        int cx = 0, cy = 0, r = merange / 2;
        int bbx = clamp_i16(0, 0, w - kMB), bby = clamp_i16(0, 0, h - kMB);
        uint64_t best = UINT64_MAX;
        while (r != 0) {
            int np = -1, nbx = 0, nby = 0;
            uint64_t nd = best;
            for (int p = 0; p < 9; p++) {
                const int px = clamp_i16(int16_t(cx + kMerSx[p] * r + mx), 0, w - kMB);
                const int py = clamp_i16(int16_t(cy + kMerSy[p] * r + my), 0, h - kMB);
                if (p > 0 && px == mx && py == my) continue;  // Block.cpp:297-301
                const uint64_t d = mb_sad(cb, cs, ref + size_t(py) * rs + px, rs);
                if (d <= nd) { np = p; nd = d; nbx = px; nby = py; }
            }
            if (np < 0) break;
            cx += kMerSx[np] * r;
            cy += kMerSy[np] * r;
            r /= 2;
            best = nd;
            bbx = nbx;
            bby = nby;
        }
        // prediction error (expandDifferenceWith, Block.cpp:256-265) per microblock
        for (int y = 0; y < mpr; y++)
            for (int x = 0; x < mpr; x++) {
                double xs[64];
                for (int i = 0; i < n; i++)
                    for (int j = 0; j < n; j++) {
                        const int yy = y * n + i, xx = x * n + j;
                        const double diff = double(cb[size_t(yy) * cs + xx]) - double(ref[size_t(bby + yy) * rs + bbx + xx]);
                        xs[i * n + j] = diff + double(-128);
                    }
                const size_t b = size_t(my / n + y) * bx + size_t(mx / n + x);
                int16_t* o = &coef[b * nn];
                for (int uv = 0; uv < nn; uv++) {
                    const double* Puv = &T.P[size_t(uv) * nn];
                    double acc = 0.0;
                    for (int k = 0; k < nn; k++) acc = acc + Puv[k] * xs[k];
                    o[uv] = int16_t(std::round((acc * T.S[uv]) / qd[uv]));
                }
                has_rle[b] = 1;
                // processIDCTMulQ (Block.cpp:162-177): the decoded error + 128 replaces expanded
                double yq[64], t[64];
                for (int k = 0; k < nn; k++) { yq[k] = double(o[k]) * qd[k]; t[k] = 0.0; }
                for (int uv = 0; uv < nn; uv++) {
                    const double* Ruv = &T.R[size_t(uv) * nn];
                    for (int ij = 0; ij < nn; ij++) t[ij] = t[ij] + Ruv[ij] * yq[uv];
                }
                for (int i = 0; i < n; i++)
                    for (int j = 0; j < n; j++)
                        E[size_t(my + y * n + i) * w + mx + x * n + j] = t[i * n + j] + double(128);
            }
        // the reference block at the motion vector replaces the macroblock (Frame.cpp:220-225)
        const int ccx = clamp_i16(int16_t(mx + cx), 0, w - kMB), ccy = clamp_i16(int16_t(my + cy), 0, h - kMB);
        for (int y = 0; y < kMB; y++)
            std::memcpy(&M[size_t(my + y) * w + mx], ref + size_t(ccy + y) * rs + ccx, kMB);
        wr.put(mv_bits, uint32_t(int32_t(int16_t(cx))));  // streamMVec (Block.cpp:415-423)
        wr.put(mv_bits, uint32_t(int32_t(int16_t(cy))));
    }
    // expandDifferences over every microblock (Frame.cpp:234-242); only those a macroblock
    // covered have an RLE sequence to stream (Block.cpp:373-375)
    for (size_t i = 0; i < size_t(w) * h; i++)
        rec[i] = uint8_t(std::clamp(double(M[i]) + E[i], 0.0, 255.0));
    for (size_t b = 0; b < has_rle.size(); b++)
        if (has_rle[b]) emit_block(T, &coef[b * nn], rle, wr);
}

// The frame loop of VideoEncoder.cpp:83-91 with gop (VideoBase.cpp:96-122, VideoBase.hpp:32):
// frame f is an I-frame when f % gop == 0; a P-frame's reference is the previous frame's buffer
// as that frame's processing left it (an I-frame leaves its pixels untouched).
int64_t encode_gop(const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes, int n,
                   const uint16_t* q, int rle, int gop, int merange, uint8_t* out, size_t cap, uint64_t start_bit,
                   uint64_t* frame_bits) {
    if ((n != 4 && n != 8) || w <= 0 || h <= 0 || w % n || h % n) return -1;
    gop = std::max(1, gop);
    // P-frames with W % 16 != 0 and two or more macroblock rows: the reference reads its
    // macroblocks from misplaced, overlapping rows (ImageBase.cpp:223-227) in a racy OpenMP loop
    if (gop > 1 && nframes > 1 && w % kMB && h / kMB >= 2) return -1;
    Tables T(n);
    double qd[64];
    for (int k = 0; k < n * n; k++) qd[k] = double(q[k]);
    BitWriter wr(out, cap, start_bit);
    std::vector<uint8_t> rec[2] = {std::vector<uint8_t>(size_t(w) * h), std::vector<uint8_t>(size_t(w) * h)};
    const uint8_t* ref = nullptr;
    size_t rs = 0;
    for (int f = 0; f < nframes; f++) {
        const uint8_t* fy = y + size_t(f) * frame_pitch;
        const uint64_t s = wr.pos;
        if (f % gop == 0) {
            const int64_t e = encode_frames(fy, w, h, stride, 0, 1, n, q, rle, out, cap, wr.pos, nullptr);
            if (e < 0) return e;
            wr.pos = uint64_t(e);  // encode_frames wrote through its own writer
            ref = fy;
            rs = stride;
        } else {
            std::vector<uint8_t>& rb = rec[f & 1];
            pframe(T, qd, fy, stride, ref, rs, rb.data(), w, h, rle, merange, wr);
            ref = rb.data();
            rs = size_t(w);
        }
        if (frame_bits) frame_bits[f] = wr.pos - s;
    }
    if (wr.overflow) return -2;
    return int64_t(wr.pos);
}

// ------------------------------------------------------------ Huffman (Huffman.hpp / .cpp)
struct Node {
    const uint8_t data;
    const size_t freq;
    Node* left;
    Node* right;
    Node(uint8_t d, size_t f = 1, Node* l = nullptr, Node* r = nullptr) : data(d), freq(f), left(l), right(r) {}
    ~Node() { delete left; delete right; }
    bool leaf() const { return !left && !right; }
    struct cmp {
        bool operator()(const Node* a, const Node* b) const { return a->freq > b->freq; }
    };
};
struct Codeword { uint32_t word, len; };

void build_dict(const Node* nd, std::vector<bool> s, std::unordered_map<uint8_t, Codeword>& dict) {
    if (!nd) return;
    if (nd->leaf()) {
        uint32_t w = 0;
        for (bool b : s) w = (w << 1u) | uint32_t(b);
        dict[nd->data] = Codeword{w, uint32_t(s.size())};
        return;
    }
    std::vector<bool> ls(s);
    ls.push_back(false);
    s.push_back(true);
    build_dict(nd->left, ls, dict);
    build_dict(nd->right, s, dict);
}

// Huffman<uint8_t>::encode (Huffman.cpp:233-344).  The reference inserts byte values into an
// unordered_map in first-occurrence order; the same container fed the same insertion sequence
// iterates identically, and that order decides the priority-queue push order, the tree, the
// DFS dict order and, through an unstable std::sort, the emitted dictionary order.
int64_t huffman_encode(const uint8_t* in, size_t n, std::vector<uint8_t>& outv) {
    std::unordered_map<uint8_t, uint32_t> freqs;
    for (size_t i = 0; i < n; i++) freqs[in[i]]++;
    std::priority_queue<Node*, std::vector<Node*>, Node::cmp> pq;
    for (const auto& pr : freqs) pq.push(new Node(pr.first, pr.second));
    if (pq.empty()) {  // empty input: the reference would dereference an empty queue
        outv.assign(1, 0);
        return 1;
    }
    while (pq.size() > 1) {
        Node* l = pq.top(); pq.pop();
        Node* r = pq.top(); pq.pop();
        pq.push(new Node(uint8_t(-1), l->freq + r->freq, l, r));
    }
    Node* root = pq.top();
    std::unordered_map<uint8_t, Codeword> dict;
    build_dict(root, std::vector<bool>(), dict);
    std::vector<std::pair<uint8_t, Codeword>> sorted(dict.begin(), dict.end());
    std::sort(sorted.begin(), sorted.end(),
              [](const std::pair<uint8_t, Codeword>& a, const std::pair<uint8_t, Codeword>& b) {
                  return a.second.len > b.second.len;
              });
    std::unordered_map<uint32_t, uint32_t> bit_freqs;
    for (const auto& wd : sorted) bit_freqs[wd.second.len]++;
    size_t dict_bits = 8 * dict.size() + 12 * bit_freqs.size() + 1;
    for (const auto& f : bit_freqs) dict_bits += size_t(f.first) * f.second;
    uint64_t data_bits = 0;
    for (const auto& pr : freqs) data_bits += uint64_t(pr.second) * dict[pr.first].len;

    const size_t cap = (dict_bits + n * 8) / 8 + 1;
    outv.assign(cap + 8, 0);
    BitWriter w(outv.data(), cap, 0);
    uint32_t seq = 0, bl = 0;
    for (const auto& wd : sorted) {
        if (seq == 0) {
            bl = wd.second.len;
            seq = bit_freqs[bl];
            w.put(8, 0x80u | (seq & 0x7Fu));  // group header (Huffman.cpp:39-43)
            w.put(4, bl & 0xFu);
        }
        w.put(8, wd.first);
        w.put(int(bl), wd.second.word);
        seq--;
    }
    w.put(1, 0);  // stop bit
    for (size_t i = 0; i < n; i++) {
        const Codeword& cw = dict[in[i]];
        w.put(int(cw.len), cw.word);
    }
    delete root;
    (void)data_bits;
    const size_t total = (w.pos + 7) / 8;
    if (n < total) {
        // no gain: '0' + the input bytes (Huffman.cpp:329-341).  The reference writes the final
        // bit one byte past its allocation; the extra byte's other 7 bits are observed 0.
        outv.assign(n + 1, 0);
        BitWriter r(outv.data(), n + 1, 0);
        r.put(1, 0);
        for (size_t i = 0; i < n; i++) r.put(8, in[i]);
        return int64_t(n + 1);
    }
    outv.resize(total);
    return int64_t(total);
}

// Huffman<uint8_t>::decode (Huffman.cpp:120-204, 354-402): returns the decoded byte stream and
// the bit position at which the caller continues (passthrough keeps the original buffer).
struct HNode { int child[2] = {-1, -1}; int sym = -1; };

bool huffman_decode(const uint8_t* in, size_t len, std::vector<uint8_t>& outv, uint64_t& start_pos, bool& passthrough) {
    BitReader rd(in, len);
    std::vector<HNode> tree(1);
    bool any = false;
    while (rd.bit()) {
        uint32_t seq = rd.get(7), bl = rd.get(4);
        while (seq--) {
            const uint32_t key = rd.get(8), word = rd.get(int(bl));
            any = true;
            int cur = 0;
            for (int b = int(bl) - 1; b >= 0; b--) {
                const int dir = (word >> b) & 1;
                if (tree[cur].child[dir] < 0) {
                    tree[cur].child[dir] = int(tree.size());
                    tree.emplace_back();
                }
                cur = tree[cur].child[dir];
            }
            tree[cur].sym = int(key);
        }
    }
    if (!any) {
        passthrough = true;
        start_pos = rd.pos;
        return true;
    }
    passthrough = false;
    // a lone 0-bit code leaves the root a leaf: the reference's treeAddLeaf is undefined there
    // (Huffman.cpp:155-172) and its walk would emit forever; report it as malformed
    if (tree[0].child[0] < 0 && tree[0].child[1] < 0) return false;
    const uint64_t raw_bits = uint64_t(len) * 8;
    outv.clear();
    while (rd.pos < raw_bits) {
        int cur = 0;
        while (tree[cur].child[0] >= 0 || tree[cur].child[1] >= 0) {
            const int nx = tree[cur].child[rd.bit()];
            if (nx < 0) return false;  // not a code of the dictionary
            cur = nx;
        }
        outv.push_back(uint8_t(tree[cur].sym));
    }
    start_pos = 0;
    return true;
}

}  // namespace

// ====================================================================== extern "C" surface
extern "C" {

void ieo_cos_table(int n, double* c) {
    const double factor = M_PI_2 / double(n);
    for (int u = 0; u < n; u++)
        for (int i = 0; i < n; i++) c[u * n + i] = std::cos(double(2.0 * i + 1.0) * double(u) * factor);
}

void ieo_zigzag(int n, int* zz) {
    // sort (x, y) by (x+y, ((x-y) odd ? y : x))  -- algo.cpp:33-37,68-87
    std::vector<int> idx(n * n);
    for (int i = 0; i < n * n; i++) idx[i] = i;
    auto key = [n](int i) {
        const int x = i % n, y = i / n;
        return std::make_pair(x + y, ((x - y) & 1) ? y : x);
    };
    std::sort(idx.begin(), idx.end(), [&](int a, int b) { return key(a) < key(b); });
    for (int k = 0; k < n * n; k++) zz[k] = idx[k];
}

int ieo_bits_needed(int v) { return bits_needed_ref(int16_t(v)); }

int64_t ieo_write_header(uint8_t* out, size_t cap, int n, const uint16_t* q, int rle, int w, int h,
                         int huffman, int video, int frame_count, int gop, int merange) {
    BitWriter wr(out, cap, 0);
    if (!huffman) wr.put(1, 0);
    int qb = 0;
    for (int k = 0; k < n * n; k++) qb = std::max(qb, ffs_ref(q[k]));  // MatrixReader.cpp:182-190
    wr.put(5, uint32_t(qb));
    for (int k = 0; k < n * n; k++) wr.put(qb, q[k]);
    wr.put(1, uint32_t(rle != 0));
    wr.put(15, uint32_t(w));
    wr.put(15, uint32_t(h));
    if (video) {
        wr.put(15, uint32_t(frame_count));
        wr.put(15, uint32_t(gop));
        wr.put(15, uint32_t(merange));
    }
    if (wr.overflow) return -2;
    return int64_t(wr.pos);
}

int ieo_quantize(const uint8_t* y, int w, int h, size_t stride, int n, const uint16_t* q, int16_t* coef) {
    if ((n != 4 && n != 8) || w % n || h % n) return -1;
    Tables T(n);
    double qd[64];
    for (int k = 0; k < n * n; k++) qd[k] = double(q[k]);
    const int bx = w / n, by = h / n;
#pragma omp parallel for schedule(static)
    for (long b = 0; b < long(bx) * by; b++)
        quantize_block(T, y + size_t(b / bx) * n * stride + size_t(b % bx) * n, stride, qd, coef + size_t(b) * n * n);
    return 0;
}

int64_t ieo_encode_blocks(const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                          int n, const uint16_t* q, int rle, uint8_t* out, size_t cap, uint64_t start_bit,
                          uint64_t* frame_bits) {
    return encode_frames(y, w, h, stride, frame_pitch, nframes, n, q, rle, out, cap, start_bit, frame_bits);
}

static int64_t finish(std::vector<uint8_t>& buf, uint64_t end_bit, int huffman, uint8_t* out, size_t cap) {
    size_t bytes = size_t((end_bit + 7) / 8);
    if (huffman) {
        std::vector<uint8_t> h;
        const int64_t hl = huffman_encode(buf.data(), bytes, h);
        if (size_t(hl) > cap) return -2;
        std::memcpy(out, h.data(), size_t(hl));
        return hl;
    }
    if (bytes > cap) return -2;
    std::memcpy(out, buf.data(), bytes);
    return int64_t(bytes);
}

int64_t ieo_encode_image(const uint8_t* y, int w, int h, int n, const uint16_t* q, int rle, int huffman,
                         uint8_t* out, size_t cap) {
    if ((n != 4 && n != 8) || w % n || h % n || w > 32767 || h > 32767) return -1;
    const size_t bound = 64 + size_t(16 * 64 + 1) + size_t(w) * h * 17 / 8 + size_t(w) * h / (n * n);
    std::vector<uint8_t> buf(bound, 0);
    const int64_t hb = ieo_write_header(buf.data(), bound, n, q, rle, w, h, huffman, 0, 0, 0, 0);
    if (hb < 0) return hb;
    const int64_t end = encode_frames(y, w, h, size_t(w), 0, 1, n, q, rle, buf.data(), bound, uint64_t(hb), nullptr);
    if (end < 0) return end;
    return finish(buf, uint64_t(end), huffman, out, cap);
}

int64_t ieo_encode_video(const uint8_t* yuv, size_t yuv_len, int w, int h, int n, const uint16_t* q, int rle,
                         int huffman, int merange, uint8_t* out, size_t cap) {
    return ieo_encode_video_gop(yuv, yuv_len, w, h, n, q, rle, huffman, 1, merange, out, cap);
}

int64_t ieo_encode_video_gop(const uint8_t* yuv, size_t yuv_len, int w, int h, int n, const uint16_t* q, int rle,
                             int huffman, int gop, int merange, uint8_t* out, size_t cap) {
    if ((n != 4 && n != 8) || w % n || h % n) return -1;
    const size_t pitch = size_t(w) * h + size_t(w) * h / 2;  // Y + UV (VideoBase.cpp:8-9,39-40)
    const int frames = int(yuv_len / pitch);
    const size_t bound = 128 + 16 * 64 + (size_t(w) * h * 17 / 8 + size_t(w) * h / (n * n) + size_t(w) * h / 32) * size_t(frames);
    std::vector<uint8_t> buf(bound, 0);
    const int64_t hb = ieo_write_header(buf.data(), bound, n, q, rle, w, h, huffman, 1, frames, std::max(1, gop), merange);
    if (hb < 0) return hb;
    const int64_t end = encode_gop(yuv, w, h, size_t(w), pitch, frames, n, q, rle, gop, merange, buf.data(), bound,
                                   uint64_t(hb), nullptr);
    if (end < 0) return end;
    return finish(buf, uint64_t(end), huffman, out, cap);
}

int64_t ieo_encode_gop(const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes, int n,
                       const uint16_t* q, int rle, int gop, int merange, uint8_t* out, size_t cap, uint64_t start_bit,
                       uint64_t* frame_bits) {
    return encode_gop(y, w, h, stride, frame_pitch, nframes, n, q, rle, gop, merange, out, cap, start_bit, frame_bits);
}

// Huffman<uint8_t>::decode alone (Huffman.cpp:354-402): the decoded bytes (passthrough = 0) or,
// without a dictionary, nothing (passthrough = 1).  -3: a bit string no code prefixes.
int64_t ieo_huffman_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, int* passthrough) {
    std::vector<uint8_t> dec;
    uint64_t pos = 0;
    bool pass = false;
    if (!huffman_decode(in, n, dec, pos, pass)) return -3;
    if (passthrough) *passthrough = pass ? 1 : 0;
    if (dec.size() > cap) return -2;
    if (!dec.empty()) std::memcpy(out, dec.data(), dec.size());
    return int64_t(dec.size());
}

int64_t ieo_huffman_encode(const uint8_t* in, size_t n, uint8_t* out, size_t cap) {
    std::vector<uint8_t> h;
    const int64_t hl = huffman_encode(in, n, h);
    if (size_t(hl) > cap) return -2;
    std::memcpy(out, h.data(), size_t(hl));
    return hl;
}

void ieo_byte_histogram(const uint8_t* in, size_t n, uint32_t* hist, uint64_t* first_pos) {
    for (int b = 0; b < 256; b++) { hist[b] = 0; first_pos[b] = UINT64_MAX; }
    for (size_t i = 0; i < n; i++) {
        if (hist[in[i]]++ == 0) first_pos[in[i]] = i;
    }
}

int64_t ieo_decode_image(const uint8_t* enc, size_t len, int n, uint8_t* out, size_t cap, int* w_out, int* h_out) {
    if (n != 4 && n != 8) return -1;
    std::vector<uint8_t> dec;
    uint64_t pos = 0;
    bool pass = false;
    if (!huffman_decode(enc, len, dec, pos, pass)) return -3;
    const uint8_t* src = pass ? enc : dec.data();
    const size_t srclen = pass ? len : dec.size();
    BitReader rd(src, srclen);
    rd.pos = pos;
    Tables T(n);
    const int nn = n * n;
    const int qb = int(rd.get(5));
    double qd[64];
    for (int k = 0; k < nn; k++) qd[k] = double(rd.get(qb));   // MatrixReader.cpp:46-56
    const int rle = int(rd.get(1));
    const int w = int(rd.get(15)), h = int(rd.get(15));        // ImageBase.cpp:123-128
    if (w_out) *w_out = w;
    if (h_out) *h_out = h;
    if (w % n || h % n) return -1;
    if (size_t(w) * h > cap) return -2;
    const int bx = w / n, by = h / n;
    const size_t nb = size_t(bx) * by;
    std::vector<double> Y(nb * nn, 0.0);
    // serial parse (Block.cpp:442-472)
    for (size_t b = 0; b < nb; b++) {
        const int bl = int(rd.get(4));
        const int length = rle ? int(rd.get(bl)) : nn;
        if (length > nn) return -4;
        for (int k = 0; k < length; k++) Y[b * nn + T.zz[k]] = double(shift_signed16(rd.get(bl), bl));
    }
    // IDCT (Block.cpp:163-177, algo.cpp:343-363) and clamp-truncate (Block.cpp:100-107)
#pragma omp parallel for schedule(static)
    for (long b = 0; b < long(nb); b++) {
        double y[64], t[64];
        for (int k = 0; k < nn; k++) { y[k] = Y[size_t(b) * nn + k] * qd[k]; t[k] = 0.0; }
        for (int uv = 0; uv < nn; uv++) {
            const double* Ruv = &T.R[size_t(uv) * nn];
            for (int ij = 0; ij < nn; ij++) t[ij] = t[ij] + Ruv[ij] * y[uv];
        }
        uint8_t* o = out + size_t(b / bx) * n * w + size_t(b % bx) * n;
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++)
                o[size_t(i) * w + j] = uint8_t(std::clamp(t[i * n + j] + double(128), 0.0, 255.0));
    }
    return int64_t(w) * h;
}


// Video decode with I/P-frames (VideoDecoder.cpp:28-58, Frame.cpp:47-127): an I-frame is parsed and
// inverse-transformed as an image; a P-frame reads one motion vector per macroblock
// (Block.cpp:481-496: bits_needed(merange)-bit signed fields), copies the previous DECODED frame's
// block at the (clamped) vector into place, then reads a record for EVERY microblock and, with
// motion compensation on, adds the decoded error (IDCT + 128) to the copied pixels
// (Block.cpp:110-119).  P-frames need W and H multiples of 16 (otherwise the reference's macroblocks
// are misplaced and its uncovered microblocks read records the encoder never wrote): -1.
// out receives frames of Y + W*H/2 bytes of 0x80 (Frame.cpp:121-124).  Returns the byte count.
int64_t ieo_decode_video_gop(const uint8_t* enc, size_t len, int n, int motioncomp, uint8_t* out, size_t cap,
                             int* w_out, int* h_out, int* frames_out) {
    if (n != 4 && n != 8) return -1;
    std::vector<uint8_t> dec;
    uint64_t pos = 0;
    bool pass = false;
    if (!huffman_decode(enc, len, dec, pos, pass)) return -3;
    const uint8_t* src = pass ? enc : dec.data();
    BitReader rd(src, pass ? len : dec.size());
    rd.pos = pos;
    Tables T(n);
    const int nn = n * n;
    const int qb = int(rd.get(5));
    double qd[64];
    for (int k = 0; k < nn; k++) qd[k] = double(rd.get(qb));
    const int rle = int(rd.get(1));
    const int w = int(rd.get(15)), h = int(rd.get(15));
    const int frames = int(rd.get(15)), gop = std::max(1, int(rd.get(15))), merange = int(rd.get(15));
    if (w_out) *w_out = w;
    if (h_out) *h_out = h;
    if (frames_out) *frames_out = frames;
    if (w % n || h % n) return -1;
    if (gop > 1 && frames > 1 && (w % kMB || h % kMB)) return -1;
    const size_t fsz = size_t(w) * h, pitch = fsz + fsz / 2;
    if (pitch * size_t(frames) > cap) return -2;
    const int mv = bits_needed_ref(int16_t(merange));
    const int bx = w / n, by = h / n, mbx = w / kMB, mby = h / kMB;
    const size_t nb = size_t(bx) * by;
    std::vector<double> Y(nb * nn);
    for (int f = 0; f < frames; f++) {
        uint8_t* o = out + size_t(f) * pitch;
        const bool iframe = (f % gop) == 0;
        std::memset(o, 0, fsz);
        if (!iframe) {
            const uint8_t* ref = out + size_t(f - 1) * pitch;
            for (int mb = 0; mb < mbx * mby; mb++) {
                const int mx = (mb % mbx) * kMB, my = (mb / mbx) * kMB;
                const int vx = shift_signed16(rd.get(mv), mv), vy = shift_signed16(rd.get(mv), mv);
                const int cx = clamp_i16(int16_t(mx + vx), 0, w - kMB), cy = clamp_i16(int16_t(my + vy), 0, h - kMB);
                for (int y = 0; y < kMB; y++) std::memcpy(o + size_t(my + y) * w + mx, ref + size_t(cy + y) * w + cx, kMB);
            }
        }
        std::fill(Y.begin(), Y.end(), 0.0);
        for (size_t b = 0; b < nb; b++) {
            const int bl = int(rd.get(4));
            const int length = rle ? int(rd.get(bl)) : nn;
            if (length > nn) return -4;
            for (int k = 0; k < length; k++) Y[b * nn + T.zz[k]] = double(shift_signed16(rd.get(bl), bl));
        }
        if (iframe || motioncomp) {
            for (size_t b = 0; b < nb; b++) {
                double yq[64], t[64];
                for (int k = 0; k < nn; k++) { yq[k] = Y[b * nn + k] * qd[k]; t[k] = 0.0; }
                for (int uv = 0; uv < nn; uv++) {
                    const double* Ruv = &T.R[size_t(uv) * nn];
                    for (int ij = 0; ij < nn; ij++) t[ij] = t[ij] + Ruv[ij] * yq[uv];
                }
                uint8_t* ob = o + size_t(b / bx) * n * w + size_t(b % bx) * n;
                for (int i = 0; i < n; i++)
                    for (int j = 0; j < n; j++) {
                        const double e = t[i * n + j] + double(128);
                        uint8_t& px = ob[size_t(i) * w + j];
                        px = uint8_t(std::clamp(iframe ? e : double(px) + e, 0.0, 255.0));
                    }
            }
        }
        std::memset(o + fsz, 0x80, fsz / 2);
    }
    return int64_t(pitch * size_t(frames));
}

}  // extern "C"
