// include/ie_host.hpp -- the host-side mirror of the reference's encoder/decoder interface,
// running its block hot path on MI355X through the C-ABI of include/ie_hip.h.
//
// Same class names, constructor arguments, settings keys, bitstream layout and error
// behaviour as the reference (cited per class), so the encoder/decoder CLIs drop onto it:
//   util::BitStreamWriter/Reader  BitStream.hpp:91-171      MSB-first bit IO (header, Huffman dict)
//   dc::ConfigReader              ConfigReader.hpp:41-75    key=value settings file
//   dc::MatrixReader<N>           MatrixReader.hpp:15-37    N x N quantisation matrix (N = 4 or 8)
//   dc::ImageProcessor            ImageBase.hpp:35-77       base of the image encoder / decoder
//   dc::VideoProcessor            VideoBase.hpp:17-48       base of the video encoder / decoder
//   algo::Huffman                 Huffman.hpp:109-142       byte Huffman post-pass (tree on the host)
//   dc::ImageEncoder/ImageDecoder ImageEncoder.hpp, ImageDecoder.hpp
//   dc::VideoEncoder/VideoDecoder VideoEncoder.hpp, VideoDecoder.hpp (any gop: I-frames and
//                                 P-frames with motion compensation on / off, ie_decode_gop)
// Every block-level operation (DCT, quantisation, RLE, bit packing, the inverse) runs on the
// GPU; there is no CPU fallback.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "ie_hip.h"

namespace util {

class BitStreamWriter {
public:
    explicit BitStreamWriter(size_t bytes = 0) : buf_(bytes, 0), pos_(0) {}
    void put_bit(int v) { put(1, v ? 1u : 0u); }
    void put(size_t length, uint32_t value);           // low `length` bits, MSB first
    void flush() { pos_ = (pos_ + 7) & ~size_t(7); }  // byte-align (BitStream.cpp:54-59)
    size_t get_position() const { return pos_; }
    size_t get_last_byte_position() const { return (pos_ + 7) / 8; }
    uint8_t* get_buffer() { return buf_.data(); }
    const uint8_t* get_buffer() const { return buf_.data(); }
    std::vector<uint8_t>& bytes() { return buf_; }
    void set_position(size_t p) { pos_ = p; }

private:
    std::vector<uint8_t> buf_;
    size_t pos_;
};

class BitStreamReader {
public:
    BitStreamReader(const uint8_t* b, size_t size) : buf_(b), size_(size), pos_(0) {}
    uint32_t get_bit();                                // 0 past the end (BitStream.cpp:14-28)
    uint32_t get(size_t length);
    size_t get_position() const { return pos_; }
    void set_position(size_t p) { pos_ = p; }
    size_t get_size() const { return size_; }
    size_t get_size_bits() const { return size_ * 8; }
    const uint8_t* get_buffer() const { return buf_; }

private:
    const uint8_t* buf_;
    size_t size_;
    size_t pos_;
};

// Logger (Logger.hpp:12-40): stdout + an append-mode file; "" disables it.
class Logger {
public:
    static void Create(const std::string& file);
    static void Destroy();
    static void WriteLn(const std::string& text);
};

}  // namespace util

namespace dc {

enum class ImageSetting : uint8_t { rawfile = 0, encfile, decfile, rle, quantfile, width, height, logfile, AMOUNT };
enum class VideoSetting : uint8_t {
    rawfile = 0, encfile, decfile, rle, quantfile, width, height, logfile, gop, merange, motioncompensation, AMOUNT
};

// ConfigReader.cpp:75-242 semantics: duplicate keys, missing '=', empty keys are errors; an image
// file has exactly the 8 image keys; a video encoder file has at least the 8 encoder keys.
class ConfigReader {
public:
    bool read(const std::string& fileName);
    bool verifyForImage();
    bool verifyForVideo(bool encoder);
    std::string getValue(ImageSetting key) const;
    std::string getValue(VideoSetting key) const;
    std::string getErrorDescription() const { return err_; }
    std::string toString() const;

private:
    std::map<std::string, std::string> kv_;
    std::string err_;
};

// The reference's default block size (Block.hpp:13); the GPU library takes 4 or 8 at run time.
static constexpr uint16_t BlockSize = 4u;

// dc::MatrixReader<size> (MatrixReader.hpp:15-37, MatrixReader.cpp:46-198): a size x size
// quantisation matrix read from whitespace-separated text (the reference's acceptance rules and
// messages), written to the stream as a 5-bit width followed by size*size values of that width.
// getData() is the matrix as doubles, as the reference hands it to Block<>::processDCTDivQ;
// data() the uint16 values for ie_set_quant.  Instantiated for 4 and 8 (config.cpp).
template <size_t size = BlockSize>
class MatrixReader {
public:
    MatrixReader();
    static MatrixReader<size> fromBitstream(util::BitStreamReader& reader);
    bool read(const std::string& fileName);
    void write(util::BitStreamWriter& writer) const;
    const std::string toString() const;
    uint8_t getMaxBitLength() const;
    const double* getData() const { return expanded_; }
    const uint16_t* data() const { return matrix_; }
    static constexpr size_t SIZE_LEN_BITS = 5;

private:
    uint16_t matrix_[size * size];
    double expanded_[size * size];
};

// What an encoder keeps of its MatrixReader<N>: the block size (a run-time parameter of the GPU
// library) and the matrix values.
struct QuantSpec {
    int n = 0;
    std::vector<uint16_t> q;
    template <size_t N>
    static QuantSpec from(const MatrixReader<N>& m) {
        QuantSpec s;
        s.n = int(N);
        s.q.assign(m.data(), m.data() + N * N);
        return s;
    }
};

}  // namespace dc

namespace algo {

// Huffman<uint8_t> (Huffman.cpp:233-402).  encode(): device histogram + first occurrence, the
// tree / dictionary replayed on the host with the reference's own libstdc++ containers, device
// re-encode.  decode(): dictionary and tree on the host, the bit walk on the device.
class Huffman {
public:
    // Encode `n` bytes at `in` (host or device).  Returns the output bytes (host).  `ctx` runs
    // the device stages.
    static int encode(ie_ctx* ctx, const uint8_t* in, size_t n, std::vector<uint8_t>& out);
    // Decode a stream that starts with the Huffman flag bit.  passthrough = true: no table, the
    // payload starts at *start_bit of `in` itself; else `out` receives the decoded bytes (the bit
    // walk runs on ctx's device, ie_huffman_decode).  Returns IE_OK or an ie_hip.h error code.
    // The dictionary part alone: the 15-bit prefix table ie_huffman_decode walks with (lut: 32768
    // entries), and where the code stream starts; passthrough when the stream holds no dictionary.
    static int decode_table(const uint8_t* in, size_t n, uint16_t* lut, bool& passthrough, size_t& start_bit);
    static int decode(ie_ctx* ctx, const uint8_t* in, size_t n, std::vector<uint8_t>& out, bool& passthrough,
                      size_t& start_bit);
};

}  // namespace algo

namespace dc {

// Owns one device context; one per process is enough for the CLIs.
class Device {
public:
    static ie_ctx* get();
};

// dc::ImageProcessor (ImageBase.hpp:35-77): the image encoder / decoder base.  The encoder
// constructor takes (source, dest, width, height, use_rle, quant matrix) and reads the raw file
// (ImageBase.cpp:19-30, 78-88); the decoder constructor takes (source, dest) and learns every
// setting from the stream (ImageBase.cpp:98-129).  process() / saveResult() are the reference's
// virtual pair.  Where the reference builds one heap Block<> per block (ImageBase.cpp:175-206)
// and loops over them, process() here hands the whole frame to the GPU library: dc::Block<N>
// has no counterpart -- see DESIGN.md §1.
class ImageProcessor {
public:
    ImageProcessor(const std::string& source_file, const std::string& dest_file, const uint16_t& width,
                   const uint16_t& height, const bool& use_rle, MatrixReader<>& quant_m)
        : ImageProcessor(source_file, dest_file, width, height, use_rle, QuantSpec::from(quant_m)) {}
    template <size_t N>
    ImageProcessor(const std::string& source_file, const std::string& dest_file, const uint16_t& width,
                   const uint16_t& height, const bool& use_rle, MatrixReader<N>& quant_m)
        : ImageProcessor(source_file, dest_file, width, height, use_rle, QuantSpec::from(quant_m)) {}
    ImageProcessor(const std::string& source_file, const std::string& dest_file);
    virtual ~ImageProcessor() = default;

    virtual bool process() = 0;
    virtual void saveResult() const {}

    const std::vector<uint8_t>& result() const { return result_; }  // encoded file / decoded pixels
    std::string error() const { return err_; }
    uint16_t getWidth() const { return width; }
    uint16_t getHeight() const { return height; }

    static constexpr size_t RLE_BITS = 1u;   // ImageBase.hpp:75
    static constexpr size_t DIM_BITS = 15u;  // ImageBase.hpp:76

protected:
    ImageProcessor(const std::string& source_file, const std::string& dest_file, uint16_t width, uint16_t height,
                   bool use_rle, QuantSpec quant);
    void saveResult(bool encoded) const;  // ImageBase.cpp:309-330: the file and the size report

    uint16_t width = 0, height = 0;
    bool use_rle = true;
    QuantSpec quant_m;
    std::string source_file, dest_file;
    std::vector<uint8_t> raw;      // the input file (ImageBase::raw)
    std::vector<uint8_t> result_;  // what saveResult writes
    std::string err_;
};

struct EncodeOptions {
    bool huffman = true;   // the reference's ENABLE_HUFFMAN (makefile:13)
    int mode = IE_MODE_FAST;
};

// dc::ImageEncoder (ImageEncoder.hpp:12-23, ImageEncoder.cpp:19-180).
class ImageEncoder : public ImageProcessor {
public:
    ImageEncoder(const std::string& source_file, const std::string& dest_file, const uint16_t& width,
                 const uint16_t& height, const bool& use_rle, MatrixReader<>& m, EncodeOptions opt = EncodeOptions())
        : ImageProcessor(source_file, dest_file, width, height, use_rle, m), opt_(opt) {}
    template <size_t N>
    ImageEncoder(const std::string& source_file, const std::string& dest_file, const uint16_t& width,
                 const uint16_t& height, const bool& use_rle, MatrixReader<N>& m, EncodeOptions opt = EncodeOptions())
        : ImageProcessor(source_file, dest_file, width, height, use_rle, m), opt_(opt) {}
    bool process() override;
    void saveResult() const override { ImageProcessor::saveResult(true); }

private:
    EncodeOptions opt_;
};

// dc::ImageDecoder (ImageDecoder.hpp:11-21, ImageDecoder.cpp:17-129).  The block size of the
// stream is the reference's compile-time BlockSize; here block_size (0: IE_BLOCKSIZE, default 4).
class ImageDecoder : public ImageProcessor {
public:
    ImageDecoder(const std::string& source_file, const std::string& dest_file, int block_size = 0);
    bool process() override;
    void saveResult() const override { ImageProcessor::saveResult(false); }
    uint16_t width_px() const { return width; }

private:
    int n_;
};

// dc::VideoProcessor (VideoBase.hpp:17-48): the video encoder / decoder base; frames are YUV420
// (Y + W*H/2 bytes, VideoBase.cpp:6-19).  gop = 1 only: every frame an I-frame, payloads
// concatenated bit-contiguously after a 210-bit header (VideoEncoder.cpp:22-107, Frame.cpp:31-45).
// gop > 1 needs motion estimation (P-frames), outside this library's scope: process() then fails
// with an explanatory error.
class VideoProcessor {
public:
    VideoProcessor(const std::string& source_file, const std::string& dest_file, const uint16_t& width,
                   const uint16_t& height, const bool& use_rle, MatrixReader<>& quant_m, const uint16_t& gop,
                   const uint16_t& merange)
        : VideoProcessor(source_file, dest_file, width, height, use_rle, QuantSpec::from(quant_m), gop, merange) {}
    template <size_t N>
    VideoProcessor(const std::string& source_file, const std::string& dest_file, const uint16_t& width,
                   const uint16_t& height, const bool& use_rle, MatrixReader<N>& quant_m, const uint16_t& gop,
                   const uint16_t& merange)
        : VideoProcessor(source_file, dest_file, width, height, use_rle, QuantSpec::from(quant_m), gop, merange) {}
    VideoProcessor(const std::string& source_file, const std::string& dest_file, const bool& motioncomp);
    virtual ~VideoProcessor() = default;

    virtual bool process() = 0;
    virtual void saveResult() const {}

    const std::vector<uint8_t>& result() const { return result_; }
    std::string error() const { return err_; }

protected:
    VideoProcessor(const std::string& source_file, const std::string& dest_file, uint16_t width, uint16_t height,
                   bool use_rle, QuantSpec quant, uint16_t gop, uint16_t merange);
    void saveResult(bool encoded) const;

    uint16_t width = 0, height = 0, gop = 1, merange = 0;
    bool use_rle = true, motioncomp = false;
    QuantSpec quant_m;
    std::string source_file, dest_file;
    // the decoder reads its (encoded) input whole; the encoder STREAMS its .raw/YUV420 input
    // (VideoEncoder::process reads it frame chunk by frame chunk), so raw stays empty there
    std::vector<uint8_t> raw, result_;
    size_t raw_size = 0;  // input file size
    std::string err_;
};

// dc::VideoEncoder (VideoEncoder.hpp:11-21).
class VideoEncoder : public VideoProcessor {
public:
    VideoEncoder(const std::string& source_file, const std::string& dest_file, const uint16_t& width,
                 const uint16_t& height, const bool& use_rle, MatrixReader<>& m, const uint16_t& gop,
                 const uint16_t& merange, EncodeOptions opt = EncodeOptions())
        : VideoProcessor(source_file, dest_file, width, height, use_rle, m, gop, merange), opt_(opt) {}
    template <size_t N>
    VideoEncoder(const std::string& source_file, const std::string& dest_file, const uint16_t& width,
                 const uint16_t& height, const bool& use_rle, MatrixReader<N>& m, const uint16_t& gop,
                 const uint16_t& merange, EncodeOptions opt = EncodeOptions())
        : VideoProcessor(source_file, dest_file, width, height, use_rle, m, gop, merange), opt_(opt) {}
    bool process() override;
    void saveResult() const override { VideoProcessor::saveResult(true); }

private:
    EncodeOptions opt_;
};

// dc::VideoDecoder (VideoDecoder.hpp): frames of Y + W*H/2 bytes of 0x80 (Frame.cpp:121-124).
class VideoDecoder : public VideoProcessor {
public:
    VideoDecoder(const std::string& source_file, const std::string& dest_file, const bool& motioncomp,
                 int block_size = 0);
    bool process() override;
    void saveResult() const override { VideoProcessor::saveResult(false); }

private:
    int n_;
};

}  // namespace dc

// C entry points of the host library (Python bindings, tests, bench).
extern "C" {
// The settings header alone (ImageEncoder.cpp:84-94; video adds frame_count, gop, merange,
// VideoEncoder.cpp:60-73) into out (host, zeroed by this call).  Returns its length in BITS.
int64_t ieh_write_header(uint8_t* out, size_t cap, int n, const uint16_t* q, int rle, int w, int h, int huffman,
                         int video, int frames, int gop, int merange);
// Whole image file as the reference encoder writes it (header + blocks [+ Huffman pass]).
// y: host or device; out: host.  Returns bytes written, < 0 on error.
int64_t ieh_encode_image(ie_ctx* ctx, const uint8_t* y, int w, int h, const uint16_t* q, int n, int rle,
                         int huffman, int mode, uint8_t* out, size_t cap);
// gop=1 video file from a YUV420 buffer (frame_count = len / (1.5 w h)).
int64_t ieh_encode_video(ie_ctx* ctx, const uint8_t* yuv, size_t len, int w, int h, const uint16_t* q, int n,
                         int rle, int huffman, int merange, int mode, uint8_t* out, size_t cap);
// Video file with I/P-frames: frame f is an I-frame when f % gop == 0 (VideoEncoder.cpp:22-107; the
// P-frames' motion search + coded error through ie_encode_gop).  gop = 1: ieh_encode_video.
int64_t ieh_encode_video_gop(ie_ctx* ctx, const uint8_t* yuv, size_t len, int w, int h, const uint16_t* q, int n,
                             int rle, int huffman, int gop, int merange, int mode, uint8_t* out, size_t cap);
// Decode an image file (host buffer) with block size n: pixels into out (w*h bytes).  A cap
// below w*h returns IE_ECAP with *w / *h set, right after the header (the payload is not decoded):
// call with cap = 0 to size the buffer.
int64_t ieh_decode_image(ie_ctx* ctx, const uint8_t* enc, size_t len, int n, uint8_t* out, size_t cap, int* w,
                         int* h);
// Decode a gop=1 video file: frames of Y + w*h/2 bytes of 0x80 (Frame.cpp:121-124).  A cap
// below the frames' size returns IE_ECAP after the header, as ieh_decode_image.
int64_t ieh_decode_video(ie_ctx* ctx, const uint8_t* enc, size_t len, int n, uint8_t* out, size_t cap, int* w,
                         int* h, int* frames);
// Huffman post-pass entirely between device buffers (in, out device memory; out needs
// ~n + 4 KiB).  Returns output bytes; only the 256-entry histogram and code table cross PCIe.
int64_t ieh_huffman_encode_device(ie_ctx* ctx, const uint8_t* din, size_t n, uint8_t* dout, size_t cap);
/* Batched device Huffman pass: string k = n[k] bytes at din + k*in_pitch -> dout + k*out_pitch
 * (device memory; out_pitch 4-byte aligned and >= the loose bound (dict + max_len * n[k]) / 8).
 * bytes[k] receives each output length.  The outputs are complete when the context's stream is. */
int ieh_huffman_encode_device_batch(ie_ctx* ctx, const uint8_t* din, size_t in_pitch, const uint64_t* n, int count,
                                    uint8_t* dout, size_t out_pitch, int64_t* bytes);
// Free the host library's device scratch for ctx (call before ie_destroy).
void ieh_release(ie_ctx* ctx);
// Huffman post-pass of n bytes (host or device) into out (host).  Returns output bytes.
int64_t ieh_huffman_encode(ie_ctx* ctx, const uint8_t* in, size_t n, uint8_t* out, size_t cap);
// Batched Huffman pass over the images of the last ie_encode_images launch on ctx (device output
// at din + k*in_pitch), lengths from the encoder's end bits on the device; bytes[k] = output size.
int ieh_huffman_encode_after_encode(ie_ctx* ctx, const uint8_t* din, size_t in_pitch, int count, uint8_t* dout,
                                    size_t out_pitch, int64_t* bytes);
// The same in two halves for pipelining batches (slot 0 / 1 alternating): _begin launches the
// histogram and returns; _finish waits for it, builds the trees and launches the pack.
int ieh_huffman_begin_after_encode(ie_ctx* ctx, const uint8_t* din, size_t in_pitch, int count, int slot);
int ieh_huffman_finish_after_encode(ie_ctx* ctx, const uint8_t* din, size_t in_pitch, int count, int slot,
                                    uint8_t* dout, size_t out_pitch, int64_t* bytes);
// Huffman<uint8_t>::decode alone (Huffman.cpp:354-402; the bit walk on the device): decoded byte
// count, or 0 with *passthrough = 1 when the stream has no dictionary.
int64_t ieh_huffman_decode(ie_ctx* ctx, const uint8_t* in, size_t n, uint8_t* out, size_t cap, int* passthrough);
// The dictionary of a Huffman-coded stream (host bytes) as ie_huffman_decode's 15-bit prefix table
// (lut: 32768 entries) and the code stream's first bit: a caller with the stream in device memory
// then decodes it device-resident.  Returns 1 when there is no dictionary (passthrough), 0, or < 0.
int ieh_huffman_table(const uint8_t* in, size_t n, uint16_t* lut, uint64_t* start_bit);
}
