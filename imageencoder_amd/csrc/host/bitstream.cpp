// imageencoder_amd/csrc/host/bitstream.cpp -- MSB-first bit IO for headers and Huffman
// dictionaries (util::BitStreamWriter/Reader, BitStream.cpp:14-77) and the Logger
// (Logger.cpp).  Bulk payload bits never pass through here: the GPU writes them.
#include <algorithm>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <memory>

#include "ie_host.hpp"

namespace util {

void BitStreamWriter::put(size_t length, uint32_t value) {
    const size_t need = (pos_ + length + 7) / 8;
    if (need > buf_.size()) buf_.resize(std::max(need, buf_.size() * 2), 0);
    // OR in chunks that stay inside one byte, most significant bits first
    while (length) {
        const size_t room = 8 - (pos_ & 7);
        const size_t take = length < room ? length : room;
        const uint32_t bits = (value >> (length - take)) & ((1u << take) - 1u);
        buf_[pos_ >> 3] |= uint8_t(bits << (room - take));
        pos_ += take;
        length -= take;
    }
}

// Past the end a read yields 0 and the position stays put (BitStream.cpp:14-28).
uint32_t BitStreamReader::get_bit() {
    const size_t p = pos_;
    if ((p >> 3) >= size_) return 0;
    pos_++;
    return (buf_[p >> 3] >> (7 - (p & 7))) & 1u;
}

uint32_t BitStreamReader::get(size_t length) {
    uint32_t v = 0;
    while (length) {
        const size_t p = pos_;
        if ((p >> 3) >= size_) return v << length;
        const size_t room = 8 - (p & 7);
        const size_t take = length < room ? length : room;
        v = (v << take) | ((uint32_t(buf_[p >> 3]) >> (room - take)) & ((1u << take) - 1u));
        pos_ += take;
        length -= take;
    }
    return v;
}

namespace {
std::unique_ptr<std::ofstream> g_log;
}

void Logger::Create(const std::string& file) {
    g_log.reset();
    if (!file.empty()) g_log.reset(new std::ofstream(file, std::ios::app));
}

void Logger::Destroy() {
    if (g_log) g_log->flush();
    g_log.reset();
}

void Logger::WriteLn(const std::string& text) {
    std::cout << text << '\n';
    if (g_log && *g_log) *g_log << text << '\n';
}

}  // namespace util
