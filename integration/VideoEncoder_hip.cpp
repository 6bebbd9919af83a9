// integration/VideoEncoder_hip.cpp -- INTEGRATION.md §B, the video encoder, as a compiled translation unit.
//
// The reference's own dc::VideoEncoder (unmodified VideoEncoder.hpp / VideoBase.hpp) with the frame
// loop of VideoEncoder::process (VideoEncoder.cpp:75-91: Frame objects per frame, then for every
// frame Frame::process -- an I-frame's block loop or a P-frame's macroblock motion search and coded
// prediction error -- and Frame::streamEncoded's bit-unaligned concatenation) replaced by ONE
// ie_encode_gop call over the YUV420 buffer.  The settings header goes through the reference's own
// BitStreamWriter and MatrixReader<>::write (VideoEncoder.cpp:56-73), the Huffman pass is the
// reference's algo::Huffman<> (:93-105), saveResult is VideoProcessor's.
//
// Linked by oracle/Makefile into oracle/_ref/encoder_hip{,_huff} with the reference's unmodified
// main.cpp -- test infrastructure (tests/test_integration.py).  Nothing here is shipped.
#include "VideoEncoder.hpp"

#include <cassert>

#include "Huffman.hpp"
#include "Logger.hpp"
#include "utils.hpp"

#include "ie_dropin.hpp"

dc::VideoEncoder::VideoEncoder(const std::string& source_file, const std::string& dest_file, const uint16_t& width,
                               const uint16_t& height, const bool& use_rle, MatrixReader<>& m, const uint16_t& gop,
                               const uint16_t& merange)
    : VideoProcessor(source_file, dest_file, width, height, use_rle, m, gop, merange) {
    assert(this->width % dc::BlockSize == 0);
    assert(this->height % dc::BlockSize == 0);
    assert(this->reader->get_size() % size_t(this->frame_buffer_size + this->frame_garbage_size) == 0);
    this->writer = nullptr;  // VideoProcessor's destructor frees it
}

// the reference's destructor releases the motion-search pattern LUT (VideoEncoder.cpp:18-20); the
// device search walks the pattern tree without one
dc::VideoEncoder::~VideoEncoder(void) {}

bool dc::VideoEncoder::process(void) {
    util::Logger::WriteLn("[VideoEncoder] Processing video...");
    ie_ctx* c = ie_dropin::gpu();
    if (!c) {
        util::Logger::WriteLn("[VideoEncoder] no GPU context");
        return false;
    }
    // the settings header, as VideoEncoder.cpp:36-73 writes it
    size_t header_bits = dc::ImageProcessor::RLE_BITS + dc::ImageProcessor::DIM_BITS * 2u +
                         dc::MatrixReader<>::SIZE_LEN_BITS +
                         size_t(this->quant_m.getMaxBitLength()) * dc::BlockSize * dc::BlockSize +
                         dc::ImageProcessor::DIM_BITS * 3u;  // frame count, gop, merange
#ifndef ENABLE_HUFFMAN
    header_bits++;
#endif
    const int frames = int(this->frame_count);
    this->writer = util::allocVar<util::BitStreamWriter>(
        ie_gop_stream_bound(this->width, this->height, int(dc::BlockSize), frames, this->merange, header_bits));
#ifndef ENABLE_HUFFMAN
    this->writer->put_bit(0);  // '0': no Huffman sequence present
#endif
    this->quant_m.write(*this->writer);
    this->writer->put(dc::ImageProcessor::RLE_BITS, uint32_t(this->use_rle));
    this->writer->put(dc::ImageProcessor::DIM_BITS, this->width);
    this->writer->put(dc::ImageProcessor::DIM_BITS, this->height);
    this->writer->put(dc::ImageProcessor::DIM_BITS, uint32_t(this->frame_count));
    this->writer->put(dc::ImageProcessor::DIM_BITS, uint32_t(this->gop));
    this->writer->put(dc::ImageProcessor::DIM_BITS, uint32_t(this->merange));

    // VideoEncoder.cpp:75-91, replaced: frame f is an I-frame when f % gop == 0 (VideoBase.hpp:32),
    // every frame's records follow the previous frame's at bit granularity (Frame.cpp:31-45); the
    // Y plane of frame f starts at f * 1.5 * W * H (VideoBase.cpp:96-122)
    uint64_t end_bit = 0;
    const size_t pitch = size_t(this->frame_buffer_size) + size_t(this->frame_garbage_size);
    if (frames > 0 &&
        (ie_dropin::set_quant(c, this->quant_m) != IE_OK ||
         ie_encode_gop(c, this->reader->get_buffer(), this->width, this->height, this->width /*stride*/, pitch,
                       frames, this->gop, this->merange, this->use_rle ? 1 : 0, IE_MODE_FAST,
                       this->writer->get_buffer(), this->writer->get_size(), this->writer->get_position(), nullptr,
                       &end_bit) != IE_OK)) {
        util::Logger::WriteLn(std::string("[VideoEncoder] ") + ie_last_error(c));
        return false;
    }
    if (frames > 0) this->writer->set_position(end_bit);

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

void dc::VideoEncoder::saveResult(void) const { VideoProcessor::saveResult(true); }
