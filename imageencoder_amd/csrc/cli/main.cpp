// imageencoder_amd/csrc/cli/main.cpp -- the encoder / decoder command lines (built with
// -DENCODER or -DDECODER, like the reference's main.cpp), over the GPU host library.
//
// Same single argument (a settings file), same keys, same checks and exit codes
// (main.cpp:20-102): 1 wrong argument count, 2 unreadable settings, 3 inconsistent settings,
// 4 bad quantisation matrix, 5 a value that is not a uint16.  ENABLE_HUFFMAN selects the Huffman
// post-pass at build time as in the reference makefile (the default `encoder` has it; the
// `encoder_nohuff` build writes the leading '0' bit instead).  The reference's compile-time
// block size is the IE_BLOCKSIZE environment variable here (4 or 8, default 4).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <string>

#include "ie_host.hpp"

namespace {

bool to_u16(const std::string& s, uint16_t& out) {  // util::lexical_cast<uint16_t>
    std::stringstream ss;
    if (s.size() >= 2 && s[0] == '0' && (s[1] == 'x' || s[1] == 'X')) ss << std::hex;
    ss << s;
    return bool(ss >> out);
}

double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

void elapsed(std::chrono::steady_clock::time_point t) {
    char b[96];
    std::snprintf(b, sizeof(b), "Elapsed time: %f milliseconds", ms_since(t));
    util::Logger::WriteLn("");
    util::Logger::WriteLn(b);
    util::Logger::WriteLn("");
}

int block_size() {
    const char* e = std::getenv("IE_BLOCKSIZE");
    return (e && std::atoi(e) == 8) ? 8 : 4;
}

// The encoder half of main.cpp:68-131 for block size N (the reference's compile-time
// dc::BlockSize; dc::MatrixReader<N> reads the matrix).  Returns a non-zero exit code on error.
#ifdef ENCODER
template <size_t N>
int encode_with(const dc::ConfigReader& c, bool is_image, bool is_encvideo, std::chrono::steady_clock::time_point start,
                bool& success) {
    const std::string rawfile = c.getValue(dc::ImageSetting::rawfile);
    const std::string encfile = c.getValue(dc::ImageSetting::encfile);
    dc::MatrixReader<N> m;
    if (!m.read(c.getValue(dc::ImageSetting::quantfile))) return 4;
    util::Logger::WriteLn("Quantization matrix:");
    util::Logger::WriteLn("-------------------------");
    util::Logger::WriteLn(m.toString());

    uint16_t width = 0, height = 0, rle = 0, gop = 0, merange = 0;
    const char* bad = nullptr;
    std::string badv;
    auto cast = [&](const std::string& v, uint16_t& o) {
        if (!bad && !to_u16(v, o)) {
            bad = "uint16_t";
            badv = v;
        }
    };
    cast(c.getValue(dc::ImageSetting::width), width);
    cast(c.getValue(dc::ImageSetting::height), height);
    cast(c.getValue(dc::ImageSetting::rle), rle);
    if (is_encvideo) {
        cast(c.getValue(dc::VideoSetting::gop), gop);
        cast(c.getValue(dc::VideoSetting::merange), merange);
    }
    if (bad) {
        util::Logger::WriteLn("Could not cast '" + badv + "' to " + bad + ".");
        return 5;
    }
    dc::EncodeOptions opt;
#ifdef ENABLE_HUFFMAN
    opt.huffman = true;
#else
    opt.huffman = false;
#endif
    if (const char* e = std::getenv("IE_MODE")) opt.mode = (std::string(e) == "exact") ? IE_MODE_EXACT : IE_MODE_FAST;
    if (is_image) {
        dc::ImageEncoder enc(rawfile, encfile, width, height, rle != 0, m, opt);
        if ((success = enc.process())) {
            enc.saveResult();
            elapsed(start);
        } else {
            util::Logger::WriteLn("Error processing raw image for encoding! " + enc.error());
        }
    } else if (is_encvideo) {
        dc::VideoEncoder enc(rawfile, encfile, width, height, rle != 0, m, gop, merange, opt);
        if ((success = enc.process())) {
            enc.saveResult();
            elapsed(start);
        } else {
            util::Logger::WriteLn("Error processing raw video for encoding! " + enc.error());
        }
    }
    return 0;
}
#endif

}  // namespace

int main(int argc, char* argv[]) {
    if (argc != 2) {
        std::cerr << "One argument, the name of a settings file, expected!" << std::endl;
        return 1;
    }
    dc::ConfigReader c;
    if (!c.read(argv[1])) {
        std::cerr << "Error reading file '" << argv[1] << "'!" << std::endl;
        std::cerr << c.getErrorDescription() << std::endl;
        return 2;
    }
    const bool is_image = c.verifyForImage();
    const std::string ei = c.getErrorDescription();
    const bool is_encvideo = c.verifyForVideo(true);
    const std::string eev = c.getErrorDescription();
    const bool is_decvideo = c.verifyForVideo(false);
    const std::string edv = c.getErrorDescription();
    if (!((is_image && !(is_encvideo || is_decvideo)) || ((is_encvideo || is_decvideo) && !is_image))) {
        std::cerr << "Error in settings!" << std::endl;
        if (!ei.empty()) std::cerr << ei << std::endl;
        if (!eev.empty()) std::cerr << eev << std::endl;
        if (!edv.empty()) std::cerr << edv << std::endl;
        return 3;
    }
    util::Logger::Create(c.getValue(dc::ImageSetting::logfile));
    util::Logger::WriteLn("Input settings:");
    util::Logger::WriteLn("-------------------------");
    util::Logger::WriteLn(c.toString());

    const std::string encfile = c.getValue(dc::ImageSetting::encfile);
    const std::string decfile = c.getValue(dc::ImageSetting::decfile);
    const int n = block_size();
    bool success = true;
    auto start = std::chrono::steady_clock::now();
    (void)success;

#ifdef ENCODER
    const std::string rawfile = c.getValue(dc::ImageSetting::rawfile);
    if (rawfile == encfile) {
        std::cerr << "Error in settings! Encoded filename must be different from raw filename!" << std::endl;
        return 3;
    }
    const int rc = (n == 8) ? encode_with<8>(c, is_image, is_encvideo, start, success)
                            : encode_with<4>(c, is_image, is_encvideo, start, success);
    if (rc) return rc;
#endif

#ifdef DECODER
    if (encfile == decfile) {
        std::cerr << "Error in settings! Decoded filename must be different from encoded!" << std::endl;
        return 3;
    }
    if (success) {
        start = std::chrono::steady_clock::now();
        if (is_image) {
            dc::ImageDecoder dec(encfile, decfile, n);
            if (dec.process()) {
                dec.saveResult();
                elapsed(start);
            } else {
                util::Logger::WriteLn("Error processing raw image for decoding! " + dec.error());
            }
        } else if (is_decvideo) {
            uint16_t motioncomp = 0;
            if (!to_u16(c.getValue(dc::VideoSetting::motioncompensation), motioncomp)) {
                util::Logger::WriteLn("Could not cast '" + c.getValue(dc::VideoSetting::motioncompensation) +
                                      "' to uint16_t.");
                return 5;
            }
            dc::VideoDecoder dec(encfile, decfile, motioncomp != 0, n);
            if (dec.process()) {
                dec.saveResult();
                elapsed(start);
            } else {
                util::Logger::WriteLn("Error processing raw video for decoding! " + dec.error());
            }
        }
    }
#endif
    util::Logger::Destroy();
    return 0;
}
