// integration/Huffman_decode_hip.cpp -- INTEGRATION.md §B, the Huffman decode, as a compiled translation unit.
//
// algo::Huffman<uint8_t>::decode(BitStreamReader&) (Huffman.cpp:354-402) rebuilds the code tree from
// the stream's dictionary and then walks it bit by bit over the whole payload (Huffman.cpp:190-204),
// one serial chain.  Its callers are the ImageProcessor / VideoProcessor decoding constructors
// (ImageBase.cpp:106-120, VideoBase.cpp:55-64).  The reference instantiates Huffman<uint8_t> once,
// in Huffman.o (`extern template`, Huffman.hpp:144-145), so those callers reach decode through an
// undefined symbol; oracle/Makefile links the decoder with
//     -Wl,--wrap=_ZN4algo7HuffmanIhE6decodeERN4util15BitStreamReaderE
// which routes every such call to the function below -- no reference source is touched.  It parses
// the dictionary (ie_huffman_table) and decodes the code stream on the device (ie_huffman_decode),
// then hands back a reader exactly as the reference's decode does: over the decoded bytes (owned
// by the reader), or -- without a dictionary -- the passthrough reader over the input buffer.
//
// Test infrastructure (tests/test_integration.py), never shipped.
#include <cstdint>
#include <string>
#include <vector>

#include "BitStream.hpp"
#include "Huffman.hpp"
#include "Logger.hpp"
#include "utils.hpp"

#include "ie_dropin.hpp"

extern "C" util::BitStreamReader* __wrap__ZN4algo7HuffmanIhE6decodeERN4util15BitStreamReaderE(
    algo::Huffman<uint8_t>* /*self: the dictionary is not kept, decoding needs the table only*/,
    util::BitStreamReader& reader) {
    const uint8_t* in = reader.get_buffer();
    const size_t len = reader.get_size();
    std::vector<uint16_t> lut(size_t(1) << 15);
    uint64_t code_start = 0;
    const int t = ie_huffman_table(in, len, reader.get_position(), lut.data(), &code_start);
    if (t < 0) {
        util::Logger::WriteLn("[Huffman] malformed dictionary");
        return nullptr;  // as if no Huffman pass: the caller keeps its reader
    }
    reader.set_position(size_t(code_start));
    const size_t raw_bits = reader.get_size_bits();
    const size_t data_bytes = util::round_to_byte(raw_bits - reader.get_position());
    if (t == 1) {
        // Huffman.cpp:361-371: no tree -- a reader over the same buffer, data_bytes long, at the
        // position after the dictionary's stop bit
        util::BitStreamReader* result = util::allocVar<util::BitStreamReader>(reader.get_buffer(), data_bytes);
        result->set_position(reader.get_position());
        util::Logger::WriteLn("[Huffman] No Huffman table present in file. Skipping decompression.");
        return result;
    }
    // Huffman.cpp:372-400: every code to the end of the buffer (the last byte's padding bits too);
    // first the symbol count, then the symbols into a buffer of exactly that size
    ie_ctx* c = ie_dropin::gpu();
    size_t n = 0;
    int r = c ? ie_huffman_decode(c, in, len, code_start, lut.data(), nullptr, 0, &n) : IE_EHIP;
    if (r != IE_OK && r != IE_ECAP) {
        util::Logger::WriteLn(std::string("[Huffman] ") + (c ? ie_last_error(c) : "no GPU context"));
        return nullptr;
    }
    uint8_t* out = util::allocArray<uint8_t>(n ? n : 1);
    if (n && (r = ie_huffman_decode(c, in, len, code_start, lut.data(), out, n, &n)) != IE_OK) {
        util::Logger::WriteLn(std::string("[Huffman] ") + ie_last_error(c));
        util::deallocArray(out);
        return nullptr;
    }
    reader.set_position(raw_bits);  // consumed, as the reference's walk leaves it
    util::BitStreamReader* result = util::allocVar<util::BitStreamReader>(out, n);
    result->set_managed(true);  // the reader owns the decoded bytes (Huffman.cpp:388-392)
    util::Logger::WriteLn(std::string_format("[Huffman]           Input file size: %8d bytes", len));
    util::Logger::WriteLn(std::string_format("[Huffman]         Decompressed size: %8d bytes  => Ratio: %.2f%%", n,
                                             float(n) / float(len) * 100.0f));
    return result;
}
