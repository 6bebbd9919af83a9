// imageencoder_amd/csrc/host/huffman.cpp -- the byte Huffman post-pass, algo::Huffman<uint8_t>
// (Huffman.cpp:233-402), with its O(bytes) stages on the GPU and only the 256-symbol tree here.
//
// Why the host replay is exact: the reference's output is a function of (a) the count of every
// byte value and (b) the order in which the values were first inserted into its
// std::unordered_map<uint8_t, uint32_t> (Huffman.cpp:237-243) -- that container's iteration
// order depends only on the insertion sequence, and it fixes the priority-queue push order, hence
// the tie-breaking of equal frequencies, the tree, the DFS dictionary order and (through the
// unstable std::sort of Huffman.cpp:287) the emitted dictionary order.  ie_huffman_hist returns
// both (a) and the first position of every value, so inserting the values in first-position
// order into the same libstdc++ containers reproduces every step.
#include <algorithm>
#include <omp.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <queue>
#include <stdexcept>
#include <thread>
#include <unordered_map>
#include <vector>

#include "ie_host.hpp"
#include "host_internal.hpp"

namespace algo {
namespace {

// Tree nodes live in one pool (no per-node allocation); children by pointer as in the reference.
struct Node {
    uint8_t data;
    size_t freq;
    Node* left = nullptr;
    Node* right = nullptr;
    bool leaf() const { return !left && !right; }
};
struct ByFreq {  // Node::comparator (Huffman.hpp:63-67): lower frequency = higher priority
    bool operator()(const Node* a, const Node* b) const { return a->freq > b->freq; }
};
struct Codeword {
    uint32_t word, len;
};

// Depth-first, left before right (Huffman.cpp:93-118): the order of the dictionary insertions.
// The path travels as (bits, depth); a depth past 32 is reported by the caller.
void walk(const Node* nd, uint64_t bits, uint32_t depth, std::unordered_map<uint8_t, Codeword>& dict) {
    if (!nd) return;
    if (nd->leaf()) {
        dict[nd->data] = Codeword{uint32_t(bits), depth};
        return;
    }
    walk(nd->left, bits << 1, depth + 1, dict);
    walk(nd->right, (bits << 1) | 1u, depth + 1, dict);
}

}  // namespace

// Dictionary + code table from the device histogram.  Returns the dictionary bit image in `hdr`.
bool build_code(const uint32_t* hist, const uint64_t* first, util::BitStreamWriter& hdr, uint32_t* code,
                uint8_t* len, uint64_t& data_bits, std::string& err) {
    std::vector<int> order;
    for (int b = 0; b < 256; b++)
        if (hist[b]) order.push_back(b);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return first[a] < first[b]; });
    std::unordered_map<uint8_t, uint32_t> freqs;
    for (int b : order) freqs[uint8_t(b)] = hist[b];

    std::vector<Node> pool;
    pool.reserve(2 * freqs.size());  // leaves + internal nodes: pointers stay valid
    std::vector<Node*> heap;
    heap.reserve(freqs.size());
    std::priority_queue<Node*, std::vector<Node*>, ByFreq> pq(ByFreq(), std::move(heap));
    for (const auto& pr : freqs) {
        pool.push_back(Node{pr.first, pr.second});
        pq.push(&pool.back());
    }
    while (pq.size() > 1) {
        Node* l = pq.top();
        pq.pop();
        Node* r = pq.top();
        pq.pop();
        pool.push_back(Node{uint8_t(-1), l->freq + r->freq, l, r});
        pq.push(&pool.back());
    }
    const Node* root = pq.top();
    std::unordered_map<uint8_t, Codeword> dict;
    walk(root, 0, 0, dict);

    std::vector<std::pair<uint8_t, Codeword>> sorted(dict.begin(), dict.end());
    std::sort(sorted.begin(), sorted.end(),
              [](const std::pair<uint8_t, Codeword>& a, const std::pair<uint8_t, Codeword>& b) {
                  return a.second.len > b.second.len;
              });
    std::unordered_map<uint32_t, uint32_t> group;
    for (const auto& e : sorted) group[e.second.len]++;

    // dictionary: groups of equal code length, {1, count:7, len:4} then {key:8, code:len}...
    uint32_t left = 0, bl = 0;
    for (const auto& e : sorted) {
        if (left == 0) {
            bl = e.second.len;
            left = group[bl];
            hdr.put(8, 0x80u | (left & 0x7Fu));  // Huffman.cpp:39-43 (7-bit count, 4-bit length)
            hdr.put(4, bl & 0xFu);
        }
        hdr.put(8, e.first);
        hdr.put(bl, e.second.word);
        left--;
    }
    hdr.put_bit(0);  // stop bit

    std::memset(code, 0, 256 * sizeof(uint32_t));
    std::memset(len, 0, 256);
    data_bits = 0;
    for (const auto& e : dict) {
        if (e.second.len > 32) {
            err = "Huffman code longer than 32 bits";
            return false;
        }
        code[e.first] = e.second.word;
        len[e.first] = uint8_t(e.second.len);
        data_bits += uint64_t(hist[e.first]) * e.second.len;
    }
    return true;
}

// Encode n device-resident bytes into the device buffer `out` (grown and zeroed as needed).
// Returns the output length in bytes or a negative error.
int64_t huffman_device(ie_ctx* c, const uint8_t* din, size_t n, dc::DeviceBuffer& out, std::string& err) {
    uint32_t hist[256];
    uint64_t first[256];
    int r;
    if ((r = ie_huffman_hist(c, din, n, hist, first))) return (err = ie_last_error(c), r);
    if (n == 0) {  // the reference pops an empty queue here; emit the bare stop bit
        if ((r = out.reserve(8)) || (r = ie_memset(c, out.p, 0, 8))) return (err = ie_last_error(c), r);
        return 1;
    }
    util::BitStreamWriter hdr(64);
    uint32_t code[256];
    uint8_t len[256];
    uint64_t data_bits = 0;
    if (!build_code(hist, first, hdr, code, len, data_bits, err)) return IE_EINVAL;
    const uint64_t dict_bits = hdr.get_position();
    const uint64_t total = (dict_bits + data_bits + 7) / 8;
    if (n < total) {
        // no gain: '0' + the input bytes, n + 1 bytes (Huffman.cpp:329-341)
        const size_t need = ie_stream_bound_bytes(1 + 8 * uint64_t(n));
        if ((r = out.reserve(need))) return (err = ie_last_error(c), r);
        if ((r = ie_memset(c, out.p, 0, 4))) return (err = ie_last_error(c), r);
        if ((r = ie_bitcopy(c, din, n, out.p, out.cap, 1))) return (err = ie_last_error(c), r);
        return int64_t(n + 1);
    }
    unsigned maxlen = 0;
    for (int b = 0; b < 256; b++) maxlen = std::max<unsigned>(maxlen, len[b]);
    const size_t need = ie_stream_bound_bytes(dict_bits + uint64_t(maxlen) * n);
    if ((r = out.reserve(need))) return (err = ie_last_error(c), r);
    // the packer completes the dictionary's last word from these bytes; later words it overwrites
    const size_t hb = size_t((dict_bits + 7) / 8);
    if ((r = ie_memset(c, out.p, 0, hb + 4))) return (err = ie_last_error(c), r);
    if ((r = ie_memcpy(c, out.p, hdr.get_buffer(), hb))) return (err = ie_last_error(c), r);
    uint64_t end = 0;
    if ((r = ie_huffman_pack(c, din, n, code, len, out.p, out.cap, dict_bits, &end))) return (err = ie_last_error(c), r);
    if (end != dict_bits + data_bits) return (err = "Huffman pack length mismatch", IE_EDEVICE);
    return int64_t(total);
}

// The host half of a batched pass, once the histograms are on the host: the tree builds on host
// threads, then one pack launch (asynchronous).  n[k] = string k's length.
static int trees_and_pack(ie_ctx* c, const uint8_t* din, size_t in_pitch, const uint64_t* n, int count,
                          const uint32_t* hist, const uint64_t* first, uint8_t* dout, size_t out_pitch, int64_t* bytes,
                          std::string& err) {
    const size_t K = size_t(count);
    std::vector<uint32_t> code(256 * K);
    std::vector<uint64_t> start(K);
    std::vector<uint8_t> len(256 * K);
    std::vector<std::vector<uint8_t>> dict(K);
    std::vector<std::string> errs(K);
    std::vector<char> ok(K, 1);
    auto build = [&](size_t k) {
        uint32_t* cd = &code[256 * k];
        uint8_t* ln = &len[256 * k];
        if (n[k] == 0) {  // the reference pops an empty queue: the bare stop bit
            dict[k].assign(1, 0);
            start[k] = 1;
            bytes[k] = 1;
            return;
        }
        util::BitStreamWriter hdr(64);
        uint64_t data_bits = 0;
        if (!build_code(&hist[256 * k], &first[256 * k], hdr, cd, ln, data_bits, errs[k])) {
            ok[k] = 0;
            return;
        }
        const uint64_t dict_bits = hdr.get_position();
        const uint64_t total = (dict_bits + data_bits + 7) / 8;
        if (n[k] < total) {  // no gain: '0' + the input bytes (Huffman.cpp:329-341)
            for (int b = 0; b < 256; b++) {
                cd[b] = uint32_t(b);
                ln[b] = 8;
            }
            dict[k].assign(1, 0);
            start[k] = 1;
            bytes[k] = int64_t(n[k] + 1);
            return;
        }
        const size_t hb = size_t((dict_bits + 7) / 8);
        dict[k].assign(hdr.get_buffer(), hdr.get_buffer() + hb);
        start[k] = dict_bits;
        bytes[k] = int64_t(total);
    };
    // one tree per string on OpenMP's persistent thread team (no thread start-up per call)
    const int T = int(std::min<size_t>(K, size_t(std::max(1, std::min(16, omp_get_max_threads())))));
#ifdef IE_HOST_PROFILE
    const auto b0 = std::chrono::steady_clock::now();
#endif
#pragma omp parallel for schedule(dynamic, 1) num_threads(T) if (T > 1)
    for (int k = 0; k < int(K); k++) build(size_t(k));
#ifdef IE_HOST_PROFILE
    fprintf(stderr, "[finish] %d trees on %d threads %.1f us\n", count, T,
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - b0).count());
#endif
    for (size_t k = 0; k < K; k++)
        if (!ok[k]) return (err = errs[k], IE_EINVAL);
    size_t pp = 4;
    for (const auto& d : dict) pp = std::max(pp, d.size());
    std::vector<uint8_t> prefix(pp * K, 0);
    for (size_t k = 0; k < K; k++) std::memcpy(&prefix[pp * k], dict[k].data(), dict[k].size());
    int r;
    if ((r = ie_huffman_pack_batch(c, din, in_pitch, n, count, code.data(), len.data(), prefix.data(), pp, dout,
                                   out_pitch, start.data(), nullptr)))
        return (err = ie_last_error(c), r);
    return IE_OK;
}

// A batch of device-resident strings (string k: n[k] bytes at din + k*in_pitch) into
// dout + k*out_pitch: one histogram launch, the tree builds on host threads, one pack launch.
// bytes[k] = output length of string k.  Asynchronous after the histogram read-back.
// d_end_bits (device, optional): the strings' end bits instead of host lengths n -- the encoder's
// own output (ie_last_end_bits): the lengths are then recovered from the histograms.
int huffman_device_batch(ie_ctx* c, const uint8_t* din, size_t in_pitch, const uint64_t* n_in, int count, uint8_t* dout,
                         size_t out_pitch, int64_t* bytes, std::string& err, const uint64_t* d_end_bits) {
    const size_t K = size_t(count);
    // IE_HTIME=1: per-stage host timing to stderr (profiling aid)
    static const bool htime = getenv("IE_HTIME") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    const auto t0 = now();
    std::vector<uint32_t> hist(256 * K);
    std::vector<uint64_t> first(256 * K);
    int r;
    std::vector<uint64_t> nv;
    const uint64_t* n = n_in;
    if (d_end_bits) {
        if ((r = ie_huffman_hist_batch_ends(c, din, in_pitch, d_end_bits, count, hist.data(), first.data())))
            return (err = ie_last_error(c), r);
        nv.assign(K, 0);
        for (size_t k = 0; k < K; k++)
            for (int b = 0; b < 256; b++) nv[k] += hist[256 * k + b];
        n = nv.data();
    } else if ((r = ie_huffman_hist_batch(c, din, in_pitch, n, count, hist.data(), first.data()))) {
        return (err = ie_last_error(c), r);
    }
    const auto t1 = now();
    r = trees_and_pack(c, din, in_pitch, n, count, hist.data(), first.data(), dout, out_pitch, bytes, err);
    if (htime) {
        const auto t2 = now();
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        fprintf(stderr, "[htime] hist+readback %.1f us, trees + pack submit %.1f us\n", us(t0, t1), us(t1, t2));
    }
    return r;
}

// Pipelined form of huffman_device_batch(d_end_bits): the second half, after
// ie_huffman_hist_batch_ends_async(slot) -- waits for that slot's histograms, then trees + pack.
int huffman_device_batch_finish(ie_ctx* c, const uint8_t* din, size_t in_pitch, int count, int slot, uint8_t* dout,
                                size_t out_pitch, int64_t* bytes, std::string& err) {
#ifdef IE_HOST_PROFILE  // (profiling builds: host time of the wait and of the trees + pack issue)
    const auto h0 = std::chrono::steady_clock::now();
#endif
    const size_t K = size_t(count);
    std::vector<uint32_t> hist(256 * K);
    std::vector<uint64_t> first(256 * K);
    int r;
    if ((r = ie_huffman_hist_batch_wait(c, slot, hist.data(), first.data()))) return (err = ie_last_error(c), r);
    std::vector<uint64_t> n(K, 0);
    for (size_t k = 0; k < K; k++)
        for (int b = 0; b < 256; b++) n[k] += hist[256 * k + b];
#ifdef IE_HOST_PROFILE
    const auto h1 = std::chrono::steady_clock::now();
    r = trees_and_pack(c, din, in_pitch, n.data(), count, hist.data(), first.data(), dout, out_pitch, bytes, err);
    const auto h2 = std::chrono::steady_clock::now();
    fprintf(stderr, "[finish] wait %.1f us, trees + pack %.1f us\n",
            std::chrono::duration<double, std::micro>(h1 - h0).count(), std::chrono::duration<double, std::micro>(h2 - h1).count());
    return r;
#else
    return trees_and_pack(c, din, in_pitch, n.data(), count, hist.data(), first.data(), dout, out_pitch, bytes, err);
#endif
}

int Huffman::encode(ie_ctx* c, const uint8_t* in, size_t n, std::vector<uint8_t>& out) {
    dc::DeviceBuffer src(c), dst(c);
    std::string err;
    int r;
    const uint8_t* din = in;
    if (!dc::is_device(c, in)) {
        if ((r = src.reserve(n + 4))) return r;
        if ((r = ie_memcpy(c, src.p, in, n))) return r;
        din = src.p;
    }
    const int64_t bytes = huffman_device(c, din, n, dst, err);
    if (bytes < 0) return int(bytes);
    out.resize(size_t(bytes));
    return ie_memcpy(c, out.data(), dst.p, size_t(bytes));
}

// ----------------------------------------------------------------------------------- decode
// Huffman<uint8_t>::decode (Huffman.cpp:120-204, 354-402): the dictionary rebuilds the tree leaf
// by leaf on the host (<= 256 leaves); no dictionary entry = passthrough (the stream continues
// after the stop bit).  The bit walk -- O(stream bits), serial in the reference -- runs on the
// device (ie_huffman_decode) over a 15-bit prefix table built from the tree.
int Huffman::decode_table(const uint8_t* in, size_t n, uint16_t* lut, bool& passthrough, size_t& start_bit) {
    uint64_t from = 0;
    const int r = ie_huffman_table(in, n, 0, lut, &from);  // the dictionary parse lives in the C ABI
    if (r < 0) return r;
    passthrough = r == 1;
    start_bit = size_t(from);
    return IE_OK;
}

int Huffman::decode(ie_ctx* ctx, const uint8_t* in, size_t n, std::vector<uint8_t>& out, bool& passthrough,
                    size_t& start_bit) {
    std::vector<uint16_t> lut(size_t(1) << 15);
    size_t from = 0;
    int r = decode_table(in, n, lut.data(), passthrough, from);
    if (r) return r;
    if (passthrough) {
        start_bit = from;
        return IE_OK;
    }
    start_bit = 0;
    // the symbol count first (the walk ends at the end of the buffer, padding bits included), then
    // the symbols into a buffer of exactly that size
    size_t got = 0;
    r = ie_huffman_decode(ctx, in, n, from, lut.data(), nullptr, 0, &got);
    if (r != IE_OK && r != IE_ECAP) return r;
    out.resize(got);
    if (!got) return IE_OK;
    r = ie_huffman_decode(ctx, in, n, from, lut.data(), out.data(), out.size(), &got);
    if (r) return r;
    out.resize(got);
    return IE_OK;
}

}  // namespace algo
