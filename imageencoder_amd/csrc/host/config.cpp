// imageencoder_amd/csrc/host/config.cpp -- settings file and quantisation matrix readers with
// the reference's acceptance rules and messages:
//   dc::ConfigReader   ConfigReader.cpp:75-242 (key=value lines, CR/LF stripped, empty lines
//                      skipped; missing '=', empty key and duplicate key are errors)
//   dc::MatrixReader<N> MatrixReader.cpp:46-198 (rows split on single spaces after trimming and
//                      squeezing runs of spaces; exactly N rows of N values, each a uint16 as
//                      parsed by util::lexical_cast, utils.hpp:293-305)
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>

#include "ie_host.hpp"

namespace dc {
namespace {

const char* const kImageKeys[] = {"rawfile", "encfile", "decfile", "rle", "quantfile", "width", "height", "logfile"};
const char* const kVideoExtra[] = {"gop", "merange", "motioncompensation"};
// VideoEncoderSettings / VideoDecoderSettings (ConfigReader.hpp:41-53)
const VideoSetting kVideoEnc[] = {VideoSetting::rawfile, VideoSetting::encfile, VideoSetting::rle,
                                  VideoSetting::quantfile, VideoSetting::width, VideoSetting::height,
                                  VideoSetting::gop, VideoSetting::merange};
const VideoSetting kVideoDec[] = {VideoSetting::encfile, VideoSetting::decfile, VideoSetting::motioncompensation};

std::string key_of(ImageSetting s) { return kImageKeys[size_t(s)]; }
std::string key_of(VideoSetting s) {
    const size_t i = size_t(s), off = size_t(ImageSetting::AMOUNT);
    return i < off ? std::string(kImageKeys[i]) : std::string(kVideoExtra[i - off]);
}

// util::lexical_cast<uint16_t>: stream extraction, hex with a 0x prefix, trailing text ignored.
bool parse_u16(const std::string& s, uint16_t& out) {
    std::stringstream ss;
    std::string up = s.substr(0, 2);
    for (auto& ch : up) ch = char(std::toupper(static_cast<unsigned char>(ch)));
    if (up == "0X") ss << std::hex;
    ss << s;
    return bool(ss >> out);
}

}  // namespace

bool ConfigReader::read(const std::string& fileName) {
    kv_.clear();
    FILE* f = std::fopen(fileName.c_str(), "rt");
    if (!f) {
        err_ = "Can't open file";
        return false;
    }
    char line[16384];
    while (std::fgets(line, sizeof(line) - 1, f)) {
        size_t len = std::strlen(line);
        while (len && (line[len - 1] == '\r' || line[len - 1] == '\n')) line[--len] = '\0';
        if (!len) continue;
        const std::string s(line);
        const size_t eq = s.find('=');
        if (eq == std::string::npos) {
            err_ = "Can't find '=' in line";
            std::fclose(f);
            return false;
        }
        const std::string key = s.substr(0, eq), value = s.substr(eq + 1);
        if (key.empty()) {
            err_ = "Detected an empty key";
            std::fclose(f);
            return false;
        }
        if (kv_.count(key)) {
            err_ = "Key '" + key + "' was found more than once!";
            std::fclose(f);
            return false;
        }
        kv_[key] = value;
    }
    std::fclose(f);
    return true;
}

bool ConfigReader::verifyForImage() {
    const size_t amount = size_t(ImageSetting::AMOUNT);
    if (kv_.size() != amount) {
        err_ = "Too many or too few settings in file for image en/decoder!";
        return false;
    }
    std::string e;
    for (size_t s = 0; s < amount; s++)
        if (!kv_.count(key_of(ImageSetting(s)))) e += "Key not found: '" + key_of(ImageSetting(s)) + "'.\n";
    if (!e.empty()) {
        err_ = e;
        return false;
    }
    return true;
}

bool ConfigReader::verifyForVideo(bool encoder) {
    const VideoSetting* keys = encoder ? kVideoEnc : kVideoDec;
    const size_t n = encoder ? 8 : 3;
    if (kv_.size() < n) {
        err_ = encoder ? "Too many or too few settings in file for video encoder!"
                       : "Too many or too few settings in file for video decoder!";
        return false;
    }
    std::string e;
    for (size_t s = 0; s < n; s++)
        if (!kv_.count(key_of(keys[s]))) e += "Key not found: '" + key_of(keys[s]) + "'.\n";
    if (!e.empty()) {
        err_ = e;
        return false;
    }
    return true;
}

std::string ConfigReader::getValue(ImageSetting key) const {
    auto it = kv_.find(key_of(key));
    return it == kv_.end() ? "" : it->second;
}

std::string ConfigReader::getValue(VideoSetting key) const {
    auto it = kv_.find(key_of(key));
    return it == kv_.end() ? "" : it->second;
}

std::string ConfigReader::toString() const {
    std::ostringstream o;
    for (const auto& kv : kv_) o << std::setw(18) << kv.first << " = " << kv.second << '\n';
    return o.str();
}

// ---------------------------------------------------------------------------------- matrix
template <size_t size>
MatrixReader<size>::MatrixReader() {
    for (size_t k = 0; k < size * size; k++) {
        matrix_[k] = 0;
        expanded_[k] = 0.0;
    }
}

template <size_t size>
bool MatrixReader<size>::read(const std::string& fileName) {
    constexpr int n_ = int(size);
    std::ifstream f(fileName, std::ios::binary);
    if (!f) {
        std::cerr << "[MatrixReader] Could not read file '" << fileName << "'" << std::endl;
        return false;
    }
    std::stringstream all;
    all << f.rdbuf();
    std::vector<uint16_t> m(size_t(n_) * n_, 0);
    std::string line;
    int row = 0;
    while (std::getline(all, line)) {
        if (row >= n_) {
            std::cerr << "[MatrixReader] Too many rows in matrix! Expected " << n_ << " but got " << row
                      << " or more!" << std::endl;
            return false;
        }
        // trim, then squeeze runs of spaces (std::trim + strReplaceConsecutive)
        auto notsp = [](int ch) { return !std::isspace(ch); };
        line.erase(line.begin(), std::find_if(line.begin(), line.end(), notsp));
        line.erase(std::find_if(line.rbegin(), line.rend(), notsp).base(), line.end());
        line.erase(std::unique(line.begin(), line.end(), [](char a, char b) { return a == ' ' && b == ' '; }),
                   line.end());
        std::stringstream is(line);
        std::string item;
        int col = 0;
        while (std::getline(is, item, ' ')) {
            if (col >= n_) {
                std::cerr << "[MatrixReader] Too many cols in matrix! Expected " << n_ << " but got " << col
                          << " or more!" << std::endl;
                return false;
            }
            uint16_t v;
            if (!parse_u16(item, v)) {
                std::cerr << "[MatrixReader] Could not cast '" << item << "' to uint16_t" << std::endl;
                return false;
            }
            m[size_t(row) * n_ + col++] = v;
        }
        if (col < n_) {
            std::cerr << "[MatrixReader] Too little cols in matrix! Expected " << n_ << " but got " << col << "!"
                      << std::endl;
            return false;
        }
        row++;
    }
    if (row < n_) {
        std::cerr << "[MatrixReader] Too little rows in matrix! Expected " << n_ << " but got " << row << "!"
                  << std::endl;
        return false;
    }
    for (size_t k = 0; k < size * size; k++) {
        matrix_[k] = m[k];
        expanded_[k] = double(m[k]);  // MatrixReader.cpp:195-198 hands the doubles to the blocks
    }
    return true;
}

template <size_t size>
uint8_t MatrixReader<size>::getMaxBitLength() const {
    int len = 0;  // util::ffs = bit length (utils.hpp:210-216); ffs(0) = 1 as built
    for (uint16_t v : matrix_) len = std::max(len, v ? 32 - __builtin_clz(uint32_t(v)) : 1);
    return uint8_t(len);
}

template <size_t size>
void MatrixReader<size>::write(util::BitStreamWriter& w) const {
    const uint8_t qb = getMaxBitLength();
    w.put(SIZE_LEN_BITS, qb);
    for (uint16_t v : matrix_) w.put(qb, v);
}

template <size_t size>
MatrixReader<size> MatrixReader<size>::fromBitstream(util::BitStreamReader& r) {
    MatrixReader<size> m;
    const uint32_t qb = r.get(SIZE_LEN_BITS);
    for (size_t k = 0; k < size * size; k++) {
        m.matrix_[k] = uint16_t(r.get(qb));
        m.expanded_[k] = double(m.matrix_[k]);
    }
    return m;
}

template <size_t size>
const std::string MatrixReader<size>::toString() const {
    std::ostringstream o;
    for (size_t r = 0; r < size; r++) {
        for (size_t c = 0; c < size; c++) o << std::setw(4) << matrix_[r * size + c];
        o << '\n';
    }
    return o.str();
}

template class MatrixReader<4>;
template class MatrixReader<8>;

}  // namespace dc
