// imageencoder_amd/csrc/host/host_internal.hpp -- helpers shared by the host library sources.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "ie_host.hpp"

// Bytes of a word-granular device stream holding `bits` bits (the kernels store 32-bit words).
inline size_t ie_stream_bound_bytes(uint64_t bits) { return size_t((bits + 31) / 32) * 4 + 4; }

namespace dc {

bool is_device(ie_ctx* c, const void* p);

// A growable device allocation owned through the C-ABI allocator.
struct DeviceBuffer {
    ie_ctx* c;
    uint8_t* p = nullptr;
    size_t cap = 0;
    bool owned = true;
    explicit DeviceBuffer(ie_ctx* ctx) : c(ctx) {}
    // a caller's device buffer: never reallocated or freed
    DeviceBuffer(ie_ctx* ctx, uint8_t* ext, size_t n) : c(ctx), p(ext), cap(n), owned(false) {}
    DeviceBuffer(const DeviceBuffer&) = delete;
    DeviceBuffer& operator=(const DeviceBuffer&) = delete;
    ~DeviceBuffer() {
        if (p && owned) ie_free(c, p);
    }
    int reserve(size_t n) {
        if (n <= cap && p) return IE_OK;
        if (!owned) return IE_ECAP;
        if (p) ie_free(c, p);
        p = nullptr;
        cap = 0;
        void* q = nullptr;
        const int r = ie_malloc(c, n, &q);
        if (r) return r;
        p = static_cast<uint8_t*>(q);
        cap = n;
        return IE_OK;
    }
};

}  // namespace dc

namespace algo {
bool build_code(const uint32_t* hist, const uint64_t* first, util::BitStreamWriter& hdr, uint32_t* code,
                uint8_t* len, uint64_t& data_bits, std::string& err);
int64_t huffman_device(ie_ctx* c, const uint8_t* din, size_t n, dc::DeviceBuffer& out, std::string& err);
int huffman_device_batch(ie_ctx* c, const uint8_t* din, size_t in_pitch, const uint64_t* n, int count, uint8_t* dout,
                         size_t out_pitch, int64_t* bytes, std::string& err, const uint64_t* d_end_bits = nullptr);
int huffman_device_batch_finish(ie_ctx* c, const uint8_t* din, size_t in_pitch, int count, int slot, uint8_t* dout,
                                size_t out_pitch, int64_t* bytes, std::string& err);
}  // namespace algo

namespace dc {

// Whole-file encoder shared by ImageEncoder, VideoEncoder and the C entry points.
struct FileParams {
    int w = 0, h = 0, n = 4;
    const uint16_t* q = nullptr;
    bool rle = true, huffman = true;
    int mode = IE_MODE_FAST;
    bool video = false;
    int frames = 1, gop = 1, merange = 0;
    size_t frame_pitch = 0;
};
void write_header(util::BitStreamWriter& hdr, const FileParams& p);
// Encode into `out` (host).  y may be host or device memory.  Returns IE_OK or an IE_E* code
// with the reason in `err`.
int encode_file(ie_ctx* c, const uint8_t* y, const FileParams& p, std::vector<uint8_t>& out, std::string& err);
// A video file encoded while it is read from `path` (ie_vstream; see codec.cpp).
int encode_video_streamed(ie_ctx* c, const std::string& path, const FileParams& p, std::vector<uint8_t>& out,
                          std::string& err);

}  // namespace dc
