// integration/ImageDecoder_hip.cpp -- INTEGRATION.md §B, the decoder side, as a compiled translation unit.
//
// The reference's own dc::ImageDecoder (its unmodified ImageDecoder.hpp / ImageBase.hpp, found with
// -I<reference>) with the body of ImageDecoder::process (ImageDecoder.cpp:55-122: block creation,
// the serial Block<>::loadFromStream parse, then processIDCTMulQ + expand under OpenMP) replaced by
// ONE ie_decode_frames call.  Everything around it stays the reference's: the ImageProcessor(src, dst)
// constructor reads the file, runs the Huffman decode (routed to the device by
// Huffman_decode_hip.cpp) and parses the settings header (ImageBase.cpp:98-129); saveResult is
// ImageProcessor's.
//
// oracle/Makefile links it with the reference's objects (ImageDecoder.o left out) and the reference's
// unmodified main.cpp into oracle/_ref/decoder_hip -- test infrastructure (tests/test_integration.py):
// its files must equal the reference decoder's.  Nothing here is shipped.
#include "ImageDecoder.hpp"

#include <cassert>

#include "Logger.hpp"
#include "utils.hpp"

#include "ie_dropin.hpp"

dc::ImageDecoder::ImageDecoder(const std::string& source_file, const std::string& dest_file)
    : ImageProcessor(source_file, dest_file) {
    // ImageProcessor(src, dst) leaves `macroblocks` unset while its destructor frees it
    // (ImageBase.cpp:98-103,161-165): set it so the drop-in exits cleanly
    this->macroblocks = util::allocVar<std::vector<dc::MacroBlock*>>();
    assert(this->width % dc::BlockSize == 0);
    assert(this->height % dc::BlockSize == 0);
    const float hdrlen = float(this->reader->get_position()) / 8.0f;
    const float datlen = float(this->reader->get_size()) - hdrlen;
    util::Logger::WriteLn(std::string_format("[ImageDecoder] Loaded %dx%d image with "
                                             "%.1f bytes header and %.1f bytes data.",
                                             this->width, this->height, hdrlen, datlen));
    this->writer = util::allocVar<util::BitStreamWriter>(this->width * this->height);  // zeroed pixels
}

dc::ImageDecoder::~ImageDecoder(void) {}

bool dc::ImageDecoder::process(void) {
    util::Logger::WriteLn("[ImageDecoder] Processing image...");
    ie_ctx* c = ie_dropin::gpu();
    if (!c) {
        util::Logger::WriteLn("[ImageDecoder] no GPU context");
        return false;
    }
    // ImageDecoder.cpp:63-117, replaced: the exact parse of every block record from the reader's
    // position (Block.cpp:442-472), dequantise + FP64 inverse DCT in the reference's order
    // (Block.cpp:163-177, algo.cpp:343-363), +128, clamp and truncate (Block.cpp:100-107)
    if (ie_dropin::set_quant(c, this->quant_m) != IE_OK ||
        ie_decode_frames(c, this->reader->get_buffer(), this->reader->get_size(), this->reader->get_position(),
                         this->width, this->height, 1 /*nframes*/, this->use_rle ? 1 : 0,
                         this->writer->get_buffer(), this->width /*stride*/, 0 /*frame_pitch*/, nullptr) != IE_OK) {
        util::Logger::WriteLn(std::string("[ImageDecoder] ") + ie_last_error(c));
        return false;
    }
    this->writer->set_position(this->writer->get_size_bits());  // the buffer is written implicitly
    return true;
}

void dc::ImageDecoder::saveResult(void) const { ImageProcessor::saveResult(false); }
