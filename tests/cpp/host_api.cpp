// tests/cpp/host_api.cpp -- the host library's reference-shaped C++ surface (include/ie_host.hpp),
// used the way the reference's main.cpp uses its classes (main.cpp:68-131): a MatrixReader<N>
// read from the settings' quantfile, an encoder held through the dc::ImageProcessor base
// (virtual process / saveResult), a decoder built from (source, dest) only.
//
//   host_api matrix <matrix.txt> <n>                 -> header bits of MatrixReader<N>::write (CPU)
//   host_api encode <raw> <w> <h> <matrix> <n> <out> -> ImageEncoder via ImageProcessor* (GPU)
//   host_api decode <enc> <out> <n>                  -> ImageDecoder via ImageProcessor* (GPU)
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>

#include "ie_host.hpp"

template <size_t N>
static int matrix(const char* path) {
    dc::MatrixReader<N> m;
    if (!m.read(path)) return 4;
    util::BitStreamWriter w(1024);
    m.write(w);
    std::printf("%zu %u %.1f\n", w.get_position(), unsigned(m.getMaxBitLength()), m.getData()[N * N - 1]);
    for (size_t i = 0; i < w.get_last_byte_position(); i++) std::printf("%02x", w.get_buffer()[i]);
    std::printf("\n");
    // fromBitstream reads back what write wrote
    util::BitStreamReader r(w.get_buffer(), w.get_last_byte_position());
    const dc::MatrixReader<N> back = dc::MatrixReader<N>::fromBitstream(r);
    for (size_t k = 0; k < N * N; k++)
        if (back.data()[k] != m.data()[k]) return 6;
    return 0;
}

template <size_t N>
static int encode(char** a) {
    dc::MatrixReader<N> m;
    if (!m.read(a[5])) return 4;
    dc::EncodeOptions opt;
    opt.huffman = false;
    std::unique_ptr<dc::ImageProcessor> p(
        new dc::ImageEncoder(a[2], a[7], uint16_t(std::atoi(a[3])), uint16_t(std::atoi(a[4])), true, m, opt));
    if (!p->process()) {
        std::fprintf(stderr, "%s\n", p->error().c_str());
        return 7;
    }
    p->saveResult();
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) return 1;
    const std::string mode = argv[1];
    if (mode == "matrix" && argc >= 4) return std::atoi(argv[3]) == 8 ? matrix<8>(argv[2]) : matrix<4>(argv[2]);
    if (mode == "encode" && argc >= 8) return std::atoi(argv[6]) == 8 ? encode<8>(argv) : encode<4>(argv);
    if (mode == "decode" && argc >= 5) {
        std::unique_ptr<dc::ImageProcessor> p(new dc::ImageDecoder(argv[2], argv[3], std::atoi(argv[4])));
        if (!p->process()) {
            std::fprintf(stderr, "%s\n", p->error().c_str());
            return 7;
        }
        p->saveResult();
        return 0;
    }
    return 1;
}
