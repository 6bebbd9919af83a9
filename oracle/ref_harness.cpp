// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
//
// A driver around the *unmodified* reference sources, compiled in place from
// /root/reference by oracle/Makefile into oracle/_ref/ref_harness.  It exists for two reasons:
//
//   1. 8x8 golden vectors.  The reference fixes the block size at compile time
//      (Block.hpp:13, `BlockSize = 4u`), and the rules forbid editing or copying its sources.
//      This translation unit #includes Block.cpp and MatrixReader.cpp as they lie and adds the
//      implicit instantiations dc::Block<8> / dc::MatrixReader<8>, then drives them exactly the
//      way ImageEncoder::process drives Block<4> (ImageEncoder.cpp:52-175, serial branch
//      :140-145) and ImageDecoder::process drives the inverse (ImageDecoder.cpp:55-122).
//   2. The CPU baseline.  `time4` constructs the reference's own dc::ImageEncoder and times
//      only its process() call (block creation, DCT+quant, RLE build, serial bit emission and,
//      in the Huffman build, the Huffman pass) -- i.e. the hot path, without the file IO that
//      main.cpp:68,111 folds into its "Elapsed time".  The object is deliberately leaked: the
//      reference destructor frees an uninitialised pointer (ImageBase.cpp:78-88,161-165).
//      `time8` times the same work for 8x8 blocks: dc::ImageEncoder is hard-wired to Block<>
//      (BlockSize = 4), so it runs the body of ImageEncoder::process (ImageEncoder.cpp:52-147)
//      statement for statement over the unmodified dc::Block<8>: block creation as
//      ImageProcessor::process (ImageBase.cpp:175-206), the header, the OpenMP
//      `parallel for schedule(dynamic)` over processDCTDivQ + createRLESequence with its atomic
//      counter and critical progress call (:121-132), then the serial streamEncoded loop (:135-138).
//
// Usage (all files raw bytes):
//   ref_harness enc8  <raw> <w> <h> <rle> <matrix8.txt> <out> [huff]
//   ref_harness dec8  <enc> <out>
//   ref_harness time4 <raw> <w> <h> <rle> <matrix.txt> <iters> [out]
//   ref_harness time8 <raw> <w> <h> <rle> <matrix8.txt> <iters> [out]
//   ref_harness cos   <n>                      (prints the reference cos-product inputs as hex)
#include "Block.cpp"
#include "MatrixReader.cpp"

#include "ImageEncoder.hpp"
#include "Huffman.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <cmath>
#include <string>
#include <vector>

// dc::Block<8> / dc::MatrixReader<8> members are instantiated implicitly from the included
// definitions (an explicit instantiation would also instantiate MatrixReader<8>::fromBitstream,
// which only compiles for the default size).

static std::vector<uint8_t> read_file(const char* p) {
    FILE* f = std::fopen(p, "rb");
    if (!f) { std::perror(p); std::exit(2); }
    std::vector<uint8_t> v;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
    std::fclose(f);
    return v;
}

static void write_file(const char* p, const uint8_t* d, size_t n) {
    FILE* f = std::fopen(p, "wb");
    if (!f) { std::perror(p); std::exit(2); }
    std::fwrite(d, 1, n, f);
    std::fclose(f);
}

// 8x8 image encode through the reference Block<8> / MatrixReader<8> classes.
static int enc8(int argc, char** argv) {
    if (argc < 8) return 1;
    std::vector<uint8_t> raw = read_file(argv[2]);
    const uint16_t w = uint16_t(std::atoi(argv[3])), h = uint16_t(std::atoi(argv[4]));
    const bool rle = std::atoi(argv[5]) != 0;
    const bool huff = argc > 8 && std::string(argv[8]) == "huff";
    dc::MatrixReader<8> m;
    if (!m.read(argv[6])) return 4;
    if (raw.size() != size_t(w) * h || w % 8 || h % 8) return 3;

    std::vector<dc::Block<8>*> blocks;
    const size_t bx = w / 8, by = h / 8;
    uint8_t* rows[8];
    for (size_t y = 0; y < by; y++)
        for (size_t x = 0; x < bx; x++) {
            for (size_t r = 0; r < 8; r++) rows[r] = raw.data() + y * 64 * bx + x * 8 + r * w;
            blocks.push_back(new dc::Block<8>(rows));
        }
    dc::Block<8>::CreateZigZagLUT();

    const size_t hdr = 1 + 30 + 5 + size_t(m.getMaxBitLength()) * 64;
    size_t bytes = util::round_to_byte(hdr + blocks.size() * blocks.front()->streamSize() + 1);
    util::BitStreamWriter* wr = new util::BitStreamWriter(bytes);
    if (!huff) wr->put_bit(0);
    m.write(*wr);
    wr->put(1, uint32_t(rle));
    wr->put(15, w);
    wr->put(15, h);
    for (auto* b : blocks) {
        b->processDCTDivQ(m.getData());
        b->createRLESequence();
        b->streamEncoded(*wr, rle);
    }
    if (huff) {
        util::BitStreamReader in(wr->get_buffer(), wr->get_last_byte_position());
        algo::Huffman<> hm;
        util::BitStreamWriter* o = hm.encode(in);
        if (o) wr = o;
    }
    write_file(argv[7], wr->get_buffer(), wr->get_last_byte_position());
    return 0;
}

// 8x8 image decode (Huffman-aware), mirroring ImageProcessor(src,dst) + ImageDecoder::process.
static int dec8(int argc, char** argv) {
    if (argc < 4) return 1;
    std::vector<uint8_t> enc = read_file(argv[2]);
    util::BitStreamReader* rd = new util::BitStreamReader(enc.data(), enc.size());
    algo::Huffman<> hm;
    util::BitStreamReader* o = hm.decode(*rd);
    if (o) rd = o;
    const uint32_t qb = rd->get(5);
    double q[64];
    for (int k = 0; k < 64; k++) q[k] = double(rd->get(qb));
    const bool rle = rd->get(1) != 0;
    const uint16_t w = uint16_t(rd->get(15)), h = uint16_t(rd->get(15));
    std::vector<uint8_t> out(size_t(w) * h, 0);
    std::vector<dc::Block<8>*> blocks;
    const size_t bx = w / 8, by = h / 8;
    uint8_t* rows[8];
    for (size_t y = 0; y < by; y++)
        for (size_t x = 0; x < bx; x++) {
            for (size_t r = 0; r < 8; r++) rows[r] = out.data() + y * 64 * bx + x * 8 + r * w;
            blocks.push_back(new dc::Block<8>(rows));
        }
    dc::Block<8>::CreateZigZagLUT();
    for (auto* b : blocks) b->loadFromStream(*rd, rle);
    for (auto* b : blocks) {
        b->processIDCTMulQ(q);
        b->expand();
    }
    write_file(argv[3], out.data(), out.size());
    return 0;
}

// Time the reference's own ImageEncoder::process() (4x4, whatever OpenMP/Huffman flags this
// binary was built with).  Prints one JSON line.
static int time4(int argc, char** argv) {
    if (argc < 8) return 1;
    const std::string raw = argv[2], dst = argc > 8 ? argv[8] : "/dev/null";
    const uint16_t w = uint16_t(std::atoi(argv[3])), h = uint16_t(std::atoi(argv[4]));
    const bool rle = std::atoi(argv[5]) != 0;
    const int iters = std::atoi(argv[7]);
    dc::MatrixReader<> m;
    if (!m.read(argv[6])) return 4;
    util::Logger::Create("");
    double best = 1e30, total = 0;
    for (int it = 0; it < iters; it++) {
        // leaked on purpose: ~ImageProcessor frees an uninitialised pointer (ImageBase.cpp:161-165)
        dc::ImageEncoder* enc = new dc::ImageEncoder(raw, dst, w, h, rle, m);
        auto t0 = std::chrono::steady_clock::now();
        enc->process();
        auto t1 = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        best = ms < best ? ms : best;
        total += ms;
        if (it == iters - 1 && argc > 8) enc->saveResult();
    }
    std::fprintf(stderr, "{\"iters\": %d, \"best_ms\": %.3f, \"mean_ms\": %.3f, \"px\": %zu}\n",
                 iters, best, total / iters, size_t(w) * h);
    return 0;
}

// ImageEncoder::process (ImageEncoder.cpp:52-147) for Block<8>; see the header comment.
static double encode8_once(const std::vector<uint8_t>& raw, uint16_t w, uint16_t h, bool rle,
                           dc::MatrixReader<8>& m, std::vector<uint8_t>* out) {
    auto t0 = std::chrono::steady_clock::now();
    // ImageProcessor::process (ImageBase.cpp:175-206): one heap Block per 8x8 block
    std::vector<dc::Block<8>*>* blocks = new std::vector<dc::Block<8>*>();
    const size_t bx = w / 8, by = h / 8;
    uint8_t* rows[8];
    uint8_t* buf = const_cast<uint8_t*>(raw.data());
    for (size_t y = 0; y < by; y++)
        for (size_t x = 0; x < bx; x++) {
            for (size_t r = 0; r < 8; r++) rows[r] = buf + y * 64 * bx + x * 8 + r * w;
            blocks->push_back(new dc::Block<8>(rows));
        }
    size_t output_length = 1 + 30 + 5 + size_t(m.getMaxBitLength()) * 64;
    output_length += blocks->size() * blocks->front()->streamSize();
    output_length++;
    output_length = util::round_to_byte(output_length);
    util::BitStreamWriter* wr = new util::BitStreamWriter(output_length);
    wr->put_bit(0);
    m.write(*wr);
    wr->put(1, uint32_t(rle));
    wr->put(15, w);
    wr->put(15, h);
    const size_t block_count = blocks->size();
    size_t blockid = 0u;
    util::Logger::WriteProgress(0, block_count);
    #pragma omp parallel for shared(blockid) schedule(dynamic)
    for (auto it = blocks->begin(); it < blocks->end(); it++) {
        dc::Block<8>* b = *it;
        b->processDCTDivQ(m.getData());
        b->createRLESequence();
        #pragma omp atomic
        ++blockid;
        #pragma omp critical
        util::Logger::WriteProgress(blockid, block_count);
    }
    for (dc::Block<8>* b : *blocks) b->streamEncoded(*wr, rle);
    auto t1 = std::chrono::steady_clock::now();
    if (out) out->assign(wr->get_buffer(), wr->get_buffer() + wr->get_last_byte_position());
    // (blocks and writer leaked like the reference's own objects in time4)
    return std::chrono::duration<double, std::milli>(t1 - t0).count();
}

static int time8(int argc, char** argv) {
    if (argc < 8) return 1;
    std::vector<uint8_t> raw = read_file(argv[2]);
    const uint16_t w = uint16_t(std::atoi(argv[3])), h = uint16_t(std::atoi(argv[4]));
    const bool rle = std::atoi(argv[5]) != 0;
    const int iters = std::atoi(argv[7]);
    dc::MatrixReader<8> m;
    if (!m.read(argv[6])) return 4;
    if (raw.size() != size_t(w) * h || w % 8 || h % 8) return 3;
    util::Logger::Create("");
    dc::Block<8>::CreateZigZagLUT();
    double best = 1e30, total = 0;
    std::vector<uint8_t> out;
    for (int it = 0; it < iters; it++) {
        const double ms = encode8_once(raw, w, h, rle, m, (it == iters - 1 && argc > 8) ? &out : nullptr);
        best = ms < best ? ms : best;
        total += ms;
    }
    if (argc > 8) write_file(argv[8], out.data(), out.size());
    std::fprintf(stderr, "{\"iters\": %d, \"best_ms\": %.3f, \"mean_ms\": %.3f, \"px\": %zu}\n",
                 iters, best, total / iters, size_t(w) * h);
    return 0;
}

// The cos table the reference evaluates inside transformDCT (algo.cpp:312,318-319), printed
// as exact hex doubles so the repo can pin its own host table against it.
static int costab(int argc, char** argv) {
    const size_t n = argc > 2 ? size_t(std::atoi(argv[2])) : 4;
    const double factor = M_PI_2 / double(n);
    for (size_t u = 0; u < n; u++)
        for (size_t i = 0; i < n; i++)
            std::printf("%zu %zu %a\n", u, i, std::cos(double(2.0 * i + 1.0) * u * factor));
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) return 1;
    const std::string mode = argv[1];
    if (mode == "enc8") return enc8(argc, argv);
    if (mode == "dec8") return dec8(argc, argv);
    if (mode == "time4") return time4(argc, argv);
    if (mode == "time8") return time8(argc, argv);
    if (mode == "cos") return costab(argc, argv);
    return 1;
}
