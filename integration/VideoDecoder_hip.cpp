// integration/VideoDecoder_hip.cpp -- INTEGRATION.md §B, the video decoder, as a compiled translation unit.
//
// The reference's own dc::VideoDecoder (unmodified VideoDecoder.hpp / VideoBase.hpp) with the frame
// loop of VideoDecoder::process (VideoDecoder.cpp:33-58: Frame objects per frame, then for every frame
// Frame::loadFromStream -- an I-frame's record parse + inverse DCT, or a P-frame's motion vectors,
// reference-block copies and decoded error -- and Frame::streamEncoded) replaced by ONE ie_decode_gop
// call.  The VideoProcessor(src, dst, motioncomp) constructor reads the file, runs the Huffman decode
// (Huffman_decode_hip.cpp) and parses the settings (VideoBase.cpp:50-88); saveResult is
// VideoProcessor's.
//
// Linked by oracle/Makefile into oracle/_ref/decoder_hip with the reference's unmodified main.cpp --
// test infrastructure (tests/test_integration.py).  Nothing here is shipped.
#include "VideoDecoder.hpp"

#include <cassert>
#include <cstring>

#include "Logger.hpp"
#include "utils.hpp"

#include "ie_dropin.hpp"

dc::VideoDecoder::VideoDecoder(const std::string& source_file, const std::string& dest_file, const bool& motioncomp)
    : VideoProcessor(source_file, dest_file, motioncomp) {
    assert(this->width % dc::BlockSize == 0);
    assert(this->height % dc::BlockSize == 0);
    const float hdrlen = float(this->reader->get_position()) / 8.0f;
    const float datlen = float(this->reader->get_size()) - hdrlen;
    util::Logger::WriteLn(std::string_format("[VideoDecoder] Loaded %dx%d video with "
                                             "%.1f bytes header and %.1f bytes data.",
                                             this->width, this->height, hdrlen, datlen));
    const size_t total_frame_size = this->frame_buffer_size + this->frame_garbage_size;
    this->writer = util::allocVar<util::BitStreamWriter>(total_frame_size * this->frame_count);
}

dc::VideoDecoder::~VideoDecoder(void) {}

bool dc::VideoDecoder::process(void) {
    util::Logger::WriteLn("[VideoDecoder] Processing video...");
    ie_ctx* c = ie_dropin::gpu();
    if (!c) {
        util::Logger::WriteLn("[VideoDecoder] no GPU context");
        return false;
    }
    const size_t pitch = size_t(this->frame_buffer_size) + size_t(this->frame_garbage_size);
    const int frames = int(this->frame_count);
    // every decoded frame is its Y plane followed by W*H/2 bytes of VIDEO_UV_FILL (Frame.cpp:121-124)
    std::memset(this->writer->get_buffer(), int(dc::VIDEO_UV_FILL), pitch * size_t(frames));
    // VideoDecoder.cpp:41-56, replaced: frame f an I-frame when f % gop == 0, otherwise a P-frame
    // decoded against the previous decoded frame (motion compensation on / off as configured)
    if (frames > 0 &&
        (ie_dropin::set_quant(c, this->quant_m) != IE_OK ||
         ie_decode_gop(c, this->reader->get_buffer(), this->reader->get_size(), this->reader->get_position(),
                       this->width, this->height, frames, this->gop, this->merange, this->use_rle ? 1 : 0,
                       this->motioncomp ? 1 : 0, this->writer->get_buffer(), this->width /*stride*/, pitch,
                       nullptr) != IE_OK)) {
        util::Logger::WriteLn(std::string("[VideoDecoder] ") + ie_last_error(c));
        return false;
    }
    this->writer->set_position(this->writer->get_size_bits());  // the buffer is written implicitly
    return true;
}

void dc::VideoDecoder::saveResult(void) const { VideoProcessor::saveResult(false); }
