/* oracle/ie_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement of the ThenTech/ImageEncoder hot path, used only as the checker by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing on the product path
 * links or loads it.  Parity of this restatement with the reference is pinned by the golden
 * vectors under tests/golden/ that oracle/_ref (the reference compiled from its own sources)
 * produced; see tests/golden/make_golden.py.
 *
 * Every entry point returns >= 0 on success, < 0 on error.
 */
#ifndef IE_ORACLE_H
#define IE_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* c[u*n+i] = std::cos(((2i+1)*u) * (M_PI_2/n))  -- algo.cpp:312,318-319 */
void ieo_cos_table(int n, double* c);

/* Zig-zag order: zz[k] = row-major index of the k-th coefficient  -- algo.cpp:68-87 */
void ieo_zigzag(int n, int* zz);

/* minimal two's-complement width -- utils.hpp:226-243 */
int ieo_bits_needed(int v);

/* Write the image (video=0) or video (video=1) settings header at bit 0 of out (zeroed by
 * caller).  huffman=1 omits the leading '0' flag bit (ImageEncoder.cpp:84-94,
 * VideoEncoder.cpp:60-73, MatrixReader.cpp:145-158).  Returns the header length in bits. */
int64_t ieo_write_header(uint8_t* out, size_t cap, int n, const uint16_t* q, int rle, int w, int h,
                         int huffman, int video, int frame_count, int gop, int merange);

/* Quantised coefficients of every block of one frame, block raster order, natural (row-major)
 * coefficient order: coef[b*n*n + k]  -- Block.cpp:139-153 + algo.cpp:309-331. */
int ieo_quantize(const uint8_t* y, int w, int h, size_t stride, int n, const uint16_t* q,
                 int16_t* coef);

/* Encode nframes frames (frame f's Y plane at y + f*frame_pitch, rows `stride` apart) as block
 * records appended at bit start_bit of out (bits from start_bit on must be zero).
 * frame_bits[f] receives each frame's payload length.  Returns the end bit position.
 * -- Block.cpp:186-232 (RLE list), :372-413 (emission), Frame.cpp:31-45 (bit-unaligned concat) */
int64_t ieo_encode_blocks(const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch,
                          int nframes, int n, const uint16_t* q, int rle, uint8_t* out, size_t cap,
                          uint64_t start_bit, uint64_t* frame_bits);

/* Complete image file as the reference encoder saves it (header + blocks [+ Huffman]).
 * Returns the file size in bytes (ImageBase.cpp:315-323). */
int64_t ieo_encode_image(const uint8_t* y, int w, int h, int n, const uint16_t* q, int rle,
                         int huffman, uint8_t* out, size_t cap);

/* Complete gop=1 video file (VideoEncoder.cpp:22-107 with every frame an I-frame). */
int64_t ieo_encode_video(const uint8_t* yuv, size_t yuv_len, int w, int h, int n, const uint16_t* q,
                         int rle, int huffman, int merange, uint8_t* out, size_t cap);

/* Complete video file with I/P-frames: frame f is an I-frame when f % gop == 0, every other frame
 * a P-frame -- macroblock motion search + coded prediction error (VideoEncoder.cpp:22-107,
 * VideoBase.cpp:96-122, Frame.cpp:129-247, Block.cpp:241-339, ImageBase.cpp:208-306). */
int64_t ieo_encode_video_gop(const uint8_t* yuv, size_t yuv_len, int w, int h, int n, const uint16_t* q,
                             int rle, int huffman, int gop, int merange, uint8_t* out, size_t cap);

/* The payload alone (ieo_encode_blocks with gop / merange): frames at y + f*frame_pitch. */
int64_t ieo_encode_gop(const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes, int n,
                       const uint16_t* q, int rle, int gop, int merange, uint8_t* out, size_t cap,
                       uint64_t start_bit, uint64_t* frame_bits);

/* Huffman post-pass over whole bytes (Huffman.cpp:233-344).  Returns output bytes. */
int64_t ieo_huffman_encode(const uint8_t* in, size_t n, uint8_t* out, size_t cap);
/* Huffman<uint8_t>::decode (Huffman.cpp:354-402): decoded bytes, or 0 with *passthrough = 1 when
 * the stream carries no dictionary. */
int64_t ieo_huffman_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, int* passthrough);

/* Histogram + first occurrence of each byte value (the inputs the host tree build needs). */
void ieo_byte_histogram(const uint8_t* in, size_t n, uint32_t* hist, uint64_t* first_pos);

/* Huffman-aware image decode (ImageBase.cpp:98-129 + ImageDecoder.cpp:55-122 + Block.cpp:
 * 100-107,163-177,442-472).  Block size n must be given (the format does not carry it).
 * Writes w*h pixels, returns w*h; *w_out/*h_out receive the dimensions. */
int64_t ieo_decode_image(const uint8_t* enc, size_t len, int n, uint8_t* out, size_t cap,
                         int* w_out, int* h_out);

/* Video decode with I/P-frames (VideoDecoder.cpp:28-58, Frame.cpp:47-127, Block.cpp:441-496):
 * frames of Y + W*H/2 bytes of 0x80.  motioncomp 0: P-frames are the copied blocks only. */
int64_t ieo_decode_video_gop(const uint8_t* enc, size_t len, int n, int motioncomp, uint8_t* out, size_t cap,
                             int* w_out, int* h_out, int* frames_out);

#ifdef __cplusplus
}
#endif
#endif
