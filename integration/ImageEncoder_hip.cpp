// integration/ImageEncoder_hip.cpp -- INTEGRATION.md §B as a compiled translation unit.
//
// This is the reference's own dc::ImageEncoder (its unmodified ImageEncoder.hpp / ImageBase.hpp /
// MatrixReader.hpp / BitStream.hpp, found with -I<reference>) with the block loop of
// ImageEncoder::process (ImageEncoder.cpp:96-147: Block<>::processDCTDivQ, createRLESequence and
// the serial streamEncoded, under OpenMP) replaced by ONE call into the MI355X library
// (include/ie_hip.h).  Everything around the loop stays the reference's: the ImageProcessor
// constructor reads the raw file, the settings header goes through the reference's own
// BitStreamWriter and MatrixReader<>::write (ImageEncoder.cpp:84-94), the Huffman pass is the
// reference's algo::Huffman<> (ImageEncoder.cpp:150-172), saveResult is ImageProcessor's.
//
// oracle/Makefile links it with the reference's other objects (compiled from /root/reference)
// in place of ImageEncoder.o -- test infrastructure (tests/test_integration.py): the resulting
// encoder must write files byte-identical to the reference's own.  Nothing here is shipped.
// With the decoder and video drop-ins beside it, the reference's unmodified main.cpp links into
// complete encoder / decoder command lines on the GPU library (oracle/_ref/{encoder,decoder}_hip).
#include "ImageEncoder.hpp"

#include "Huffman.hpp"
#include "Logger.hpp"
#include "utils.hpp"

#include "ie_dropin.hpp"

dc::ImageEncoder::ImageEncoder(const std::string& source_file, const std::string& dest_file, const uint16_t& width,
                               const uint16_t& height, const bool& use_rle, MatrixReader<>& quant_m)
    : ImageProcessor(source_file, dest_file, width, height, use_rle, quant_m) {
    // ImageProcessor's constructor leaves `macroblocks` and `writer` unset while its destructor frees
    // them (ImageBase.cpp:78-88,161-165: the reference crashes at exit after saving); set both here
    this->macroblocks = util::allocVar<std::vector<dc::MacroBlock*>>();
    this->writer = nullptr;
}

dc::ImageEncoder::~ImageEncoder(void) {}

bool dc::ImageEncoder::process(void) {
    util::Logger::WriteLn("[ImageEncoder] Processing image...");
    ie_ctx* c = ie_dropin::gpu();
    if (!c) {
        util::Logger::WriteLn("[ImageEncoder] no GPU context");
        return false;
    }
    // the settings header, as ImageEncoder.cpp:84-94 writes it
    size_t header_bits = dc::ImageProcessor::RLE_BITS + dc::ImageProcessor::DIM_BITS * 2u +
                         dc::MatrixReader<>::SIZE_LEN_BITS +
                         size_t(this->quant_m.getMaxBitLength()) * dc::BlockSize * dc::BlockSize;
#ifndef ENABLE_HUFFMAN
    header_bits++;
#endif
    // the writer's zeroed buffer holds the library's bound for the records after the header
    this->writer = util::allocVar<util::BitStreamWriter>(
        ie_stream_bound(this->width, this->height, dc::BlockSize, 1, header_bits));
#ifndef ENABLE_HUFFMAN
    this->writer->put_bit(0);  // '0': no Huffman sequence present
#endif
    this->quant_m.write(*this->writer);
    this->writer->put(dc::ImageProcessor::RLE_BITS, uint32_t(this->use_rle));
    this->writer->put(dc::ImageProcessor::DIM_BITS, this->width);
    this->writer->put(dc::ImageProcessor::DIM_BITS, this->height);

    // ImageEncoder.cpp:96-147, replaced: every block's DCT, quantisation, zig-zag RLE and bit
    // packing on the GPU, appended at the writer's bit position (earlier bits are never touched)
    uint64_t end_bit = 0;
    if (ie_dropin::set_quant(c, this->quant_m) != IE_OK ||
        ie_encode_frames(c, this->reader->get_buffer(), this->width, this->height, this->width /*stride*/,
                         0 /*frame_pitch*/, 1 /*nframes*/, this->use_rle ? 1 : 0, IE_MODE_FAST,
                         this->writer->get_buffer(), this->writer->get_size(), this->writer->get_position(),
                         nullptr, &end_bit) != IE_OK) {
        util::Logger::WriteLn(std::string("[ImageEncoder] ") + ie_last_error(c));
        return false;
    }
    this->writer->set_position(end_bit);

#ifdef ENABLE_HUFFMAN
    util::BitStreamReader hm_input(this->writer->get_buffer(), this->writer->get_last_byte_position());
    algo::Huffman<> hm;
    util::BitStreamWriter* hm_output = hm.encode(hm_input);
    if (hm_output != nullptr) {
        util::deallocVar(this->writer);
        this->writer = hm_output;
    }
#endif
    return true;
}

void dc::ImageEncoder::saveResult(void) const { ImageProcessor::saveResult(true); }
