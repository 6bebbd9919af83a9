/* include/ie_hip.h -- the drop-in boundary: a C-ABI over the MI355X (gfx950) block codec.
 *
 * libie_hip.so replaces the LOOP BODY of the reference's frame encoders, i.e. everything between
 * "blocks exist" and "payload bits are in the writer":
 *
 *   dc::ImageEncoder::process      ImageEncoder.cpp:96-147  (DCT+quant, RLE build, serial emission)
 *   dc::Frame::process (I-frame)   Frame.cpp:129-159 + Frame::streamEncoded Frame.cpp:31-45
 *   algo::Huffman<>::encode        Huffman.cpp:233-344      (histogram + re-encode; the tree build
 *                                                            stays on the host, see ie_huffman_*)
 *   dc::ImageDecoder::process      ImageDecoder.cpp:55-122  (parse + IDCT + clamp; ie_decode_*)
 *
 * A per-block C call would cross the host/device boundary 518 400 times per 4K frame, so the
 * boundary is frame-batch level.  dc::Block<> has no counterpart here or in the host library
 * (include/ie_host.hpp, which mirrors ImageProcessor / MatrixReader / the encoders and decoders):
 * only the reference's own Block.o, linked into the drop-in builds of integration/, keeps that API
 * ("Why there is no dc::Block<N>").
 *
 * Conventions
 *   - Every function returns IE_OK (0) or a negative IE_E* code; ie_last_error() describes it.
 *     No C++ exception crosses this boundary.
 *   - Pixel and stream pointers may be host or device (hipMalloc) memory; the library detects
 *     which (hipPointerGetAttributes).  With device pointers and NULL result pointers every call is
 *     asynchronous on the context's stream.
 *   - Streams are MSB-first (bit k = bit 7-k%8 of byte k/8, BitStream.cpp:61-77).  The library
 *     only ORs bits in from `start_bit` on and never changes earlier bits, so a caller can write
 *     the settings header with its own BitStreamWriter and hand over start_bit = header length.
 *     Bits from start_bit on must be zero (the reference's writer buffer is zero-initialised,
 *     utils.hpp:443-446).  Device output buffers are written in whole 32-bit words: size them
 *     with ie_stream_bound().
 *   - One context per device, not internally locked; one stream per context.
 */
#ifndef IE_HIP_H
#define IE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ie_ctx ie_ctx;

enum {
    IE_OK = 0,
    IE_EINVAL = -1,    /* bad argument: N not 4|8, W%N or H%N != 0, W/H > 32767 (15-bit DIM_BITS) */
    IE_ECAP = -2,      /* output capacity too small */
    IE_EHIP = -3,      /* HIP runtime error */
    IE_ENOQUANT = -4,  /* ie_set_quant not called */
    IE_EFORMAT = -5,   /* malformed encoded stream */
    IE_EDEVICE = -6,   /* device-side protocol error (look-back timeout) */
};

enum {
    IE_MODE_FAST = 0,  /* separable FP32 DCT + exact FP64 re-evaluation of near-tie coefficients */
    IE_MODE_EXACT = 1, /* every coefficient in the reference's FP64 operation order */
};

/* Context lifetime.  device = HIP device ordinal. */
int ie_create(int device, ie_ctx** out);
int ie_destroy(ie_ctx* ctx);
const char* ie_last_error(const ie_ctx* ctx);
/* Run on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL restores
 * the context's own stream. */
int ie_set_stream(ie_ctx* ctx, void* hip_stream);
/* Wait for the context's stream, then check the device error counters: IE_EDEVICE if a tile
 * look-back timed out in any launch that returned without a read-back (asynchronous encodes,
 * packs, bit copies) since the last check -- that launch's output is invalid.  Later launches
 * then order their tiles by an atomic ticket.  Call it after a pipeline of asynchronous calls. */
int ie_sync(ie_ctx* ctx);

/* Quantisation matrix, n x n row-major uint16 (MatrixReader<N>::read, MatrixReader.cpp:65-134;
 * used as double[] via getData, :195-198).  n = 4 or 8 (the reference's compile-time
 * dc::BlockSize, Block.hpp:13, becomes a runtime parameter).  The host builds the DCT cos table
 * with std::cos in the reference's exact expression (algo.cpp:312,318-319).  q[k] must be > 0. */
int ie_set_quant(ie_ctx* ctx, const uint16_t* q, int n);

/* The cos table of the current quant matrix as the kernels use it, read back from the device:
 * out[u*n + i] = std::cos(((2.0*i + 1.0) * u) * (M_PI_2 / n)) evaluated by THIS host's libm when
 * ie_set_quant ran (algo.cpp:312,318-319), n*n doubles.  Lets a caller pin the machine's libm
 * against the reference's values (tests/golden/cos_table.json). */
int ie_cos_table(ie_ctx* ctx, double* out);

/* Upper bound in bytes of an output buffer for nframes frames of w x h encoded from start_bit
 * (4 + 17*16 bits per 4x4 block, 4 + 65*16 per 8x8 block, rounded up to whole 32-bit words). */
size_t ie_stream_bound(int w, int h, int n, int nframes, uint64_t start_bit);

/* Encode nframes frames as ONE bit-contiguous stream of block records (the gop=1 video payload
 * of Frame.cpp:31-45 / VideoEncoder.cpp:83-91; nframes = 1 is ImageEncoder's payload).
 *   y            frame f row r starts at y + f*frame_pitch + r*stride
 *   use_rle      Block::streamEncoded's use_rle (Block.cpp:372-413)
 *   mode         IE_MODE_FAST or IE_MODE_EXACT (identical output)
 *   out          stream buffer; records are appended from bit start_bit
 *   frame_bits   optional [nframes]: payload bits of each frame
 *   end_bit      optional: bit position after the last record
 * Replaces ImageEncoder.cpp:96-147 and the frame loop of VideoEncoder.cpp:83-91. */
int ie_encode_frames(ie_ctx* ctx, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch,
                     int nframes, int use_rle, int mode, uint8_t* out, size_t out_cap,
                     uint64_t start_bit, uint64_t* frame_bits, uint64_t* end_bit);

/* Videos with P-frames (gop > 1; VideoEncoder.cpp:22-107, VideoBase.cpp:96-122, Frame.cpp:129-247):
 * frame f is an I-frame when f % gop == 0 (its payload = ie_encode_frames'), every other frame a
 * P-frame against the previous frame as the reference leaves it: per 16x16 macroblock a SAD pattern
 * search within merange (Block.cpp:267-339, algo.cpp:90-139), its motion vector (bits_needed(merange)
 * bits per component, Block.cpp:415-423), then the records of the 4x4 microblocks' coded prediction
 * error (ImageBase.cpp:266-306) -- 8x8 blocks carry the vectors only (the reference's
 * micro_per_macro_row is 0 there, ImageBase.cpp:271).  Replaces the frame loop of
 * VideoEncoder.cpp:83-91 for any gop; gop = 1 equals ie_encode_frames.  Arguments as
 * ie_encode_frames; out holds ie_gop_stream_bound() bytes.  IE_EINVAL for P-frames with W % 16 != 0
 * and H >= 32 (the reference reads misplaced, overlapping macroblocks there, ImageBase.cpp:223-227). */
size_t ie_gop_stream_bound(int w, int h, int n, int nframes, int merange, uint64_t start_bit);
int ie_encode_gop(ie_ctx* ctx, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch, int nframes,
                  int gop, int merange, int use_rle, int mode, uint8_t* out, size_t out_cap, uint64_t start_bit,
                  uint64_t* frame_bits, uint64_t* end_bit);

/* Encode nframes INDEPENDENT images in one launch (an image-server batch): image f's records
 * go to out + f*out_pitch from bit start_bit (each image carries its own header region).
 * end_bits optional [nframes].  out_pitch must be a multiple of 4 bytes. */
int ie_encode_images(ie_ctx* ctx, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch,
                     int nframes, int use_rle, int mode, uint8_t* out, size_t out_pitch,
                     uint64_t start_bit, uint64_t* end_bits);

/* ie_encode_images (device output) that also counts the bytes of every image's stream -- the
 * caller's header words included, bytes [0, ceil(end_bit / 8)) -- while storing them: the counts
 * stay on the device for the next ie_huffman_hist_batch_ends_async over the same batch, which
 * then skips its own histogram pass (Huffman.cpp:237-243 without re-reading the stream).  MODE_EXACT,
 * 8x8 blocks or host output: a plain ie_encode_images (the histogram pass counts later).  No end bits are
 * returned (ie_last_end_bits holds them on the device). */
int ie_encode_images_counted(ie_ctx* ctx, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch,
                             int nframes, int use_rle, int mode, uint8_t* out, size_t out_pitch, uint64_t start_bit);

/* Quantised DCT coefficients only (Block::processDCTDivQ, Block.cpp:139-153): coef receives
 * nframes * (w/n) * (h/n) blocks of n*n int16 in natural (row-major) order, block raster order.
 * coef may be host or device memory.  Diagnostic / analysis entry point. */
int ie_quantize_frames(ie_ctx* ctx, const uint8_t* y, int w, int h, size_t stride, size_t frame_pitch,
                       int nframes, int mode, int16_t* coef);

/* Fallback statistics of the last FAST-mode encode launch: FP64 re-evaluation requests (one per
 * structural coefficient at a tie, one per block with another coefficient near a tie). */
int ie_last_fallbacks(ie_ctx* ctx, uint64_t* count);

/* ---- Device memory on the context's stream (for hosts that keep streams device-resident
 * between stages, e.g. the host library's encode -> Huffman pipeline).  ie_memcpy infers the
 * direction of each pointer and is asynchronous only when both are device memory. */
int ie_malloc(ie_ctx* ctx, size_t bytes, void** out);
int ie_free(ie_ctx* ctx, void* p);
int ie_memcpy(ie_ctx* ctx, void* dst, const void* src, size_t bytes);
int ie_memset(ie_ctx* ctx, void* dst, int value, size_t bytes);
/* 1 if p is device (hipMalloc) memory, 0 otherwise. */
int ie_is_device_ptr(const void* p);

/* ---- Streamed host path (the reference reads / writes whole files: utils.hpp:352-402,
 * VideoBase.cpp:6-19) -------------------------------------------------------------------------
 * ie_encode_images / ie_encode_frames with host frames AND a host stream buffer and nframes > 1
 * stream the batch through the device in chunks of a few frames: the H2D of chunk k+1, the encode
 * of chunk k and the D2H of chunk k-1 run concurrently on three HIP streams (PCIe full duplex),
 * through two device and two pinned host slots per direction.  Pinned caller buffers are DMA'd
 * directly, pageable ones through the pinned slots.  Page-locked host memory for such buffers: */
int ie_host_alloc(ie_ctx* ctx, size_t bytes, void** out);
int ie_host_free(ie_ctx* ctx, void* p);

/* Streamed gop=1 video payload (Frame.cpp:31-45 / VideoEncoder.cpp:83-91 for frames that arrive
 * over time, e.g. read from a .raw/YUV420 file chunk by chunk): ONE bit-contiguous stream grown on
 * the device.  open: `head` holds the caller's bytes [0, ceil(start_bit/8)) (the settings header;
 * bits from start_bit on are ignored), max_frames bounds the device stream.  push: host frames
 * (frame f row r at frames + f*frame_pitch + r*stride), copied and encoded asynchronously, each
 * chunk continuing the chain from the previous chunk's end ON THE DEVICE (no host round trip);
 * pageable frames may be reused when push returns, pinned ones are DMA'd asynchronously and may
 * be reused once the NEXT push (or finish) returns (double-buffered readers alternate two).
 * pull: the whole bytes finished so far that were not pulled yet (from byte 0, the head included)
 * into dst (*nbytes of them), while later chunks still encode.  finish: waits, checks the device
 * error counters, copies the remaining bytes (last byte zero-padded) to dst when dst != NULL, and
 * returns the end bit and optionally each frame's payload bits.  ie_vstream_device: the device
 * stream (valid until close; complete after finish), e.g. for the device Huffman pass.  One open
 * stream per context at a time; other calls on the context between pushes are allowed. */
typedef struct ie_vstream ie_vstream;
int ie_vstream_open(ie_ctx* ctx, int w, int h, size_t stride, size_t frame_pitch, int use_rle, int mode,
                    const uint8_t* head, uint64_t start_bit, int max_frames, ie_vstream** out);
int ie_vstream_push(ie_vstream* v, const uint8_t* frames, int nframes);
int ie_vstream_pull(ie_vstream* v, uint8_t* dst, size_t cap, size_t* nbytes);
int ie_vstream_finish(ie_vstream* v, uint8_t* dst, size_t cap, size_t* nbytes, uint64_t* end_bit,
                      uint64_t* frame_bits);
const uint8_t* ie_vstream_device(const ie_vstream* v);
int ie_vstream_close(ie_vstream* v);

/* ---- Huffman post-pass (config 5; Huffman.cpp:233-344) ----------------------------------
 * hist[b] = occurrences of byte value b; first_pos[b] = index of its first occurrence
 * (UINT64_MAX if absent).  The first-occurrence order is the insertion order of the reference's
 * std::unordered_map (Huffman.cpp:237-243), which the host needs to replay the tree build. */
int ie_huffman_hist(ie_ctx* ctx, const uint8_t* bytes, size_t n, uint32_t* hist, uint64_t* first_pos);

/* Re-encode n bytes with a code table (code[b] right-aligned in len[b] bits, len <= 32),
 * appending from start_bit of out (Huffman.cpp:314-319).  end_bit optional. */
int ie_huffman_pack(ie_ctx* ctx, const uint8_t* bytes, size_t n, const uint32_t* code, const uint8_t* len,
                    uint8_t* out, size_t out_cap, uint64_t start_bit, uint64_t* end_bit);

/* Batched Huffman post-pass over `count` device-resident byte strings (one encoded image each):
 * string k is n[k] bytes at in + k*in_pitch (n: host array).  Replaces the per-image
 * Huffman.cpp:237-243 histogram loop; hist/first_pos hold count*256 entries (string k at 256*k),
 * host or device memory.  One launch for the whole batch. */
int ie_huffman_hist_batch(ie_ctx* ctx, const uint8_t* in, size_t in_pitch, const uint64_t* n, int count,
                          uint32_t* hist, uint64_t* first_pos);

/* The device array of per-image end bits of the last ie_encode_images launch (valid until the
 * next encode or Huffman call on the context; stream-ordered). */
const uint64_t* ie_last_end_bits(ie_ctx* ctx);

/* ie_huffman_hist_batch with the string lengths taken on the device from stream end bits
 * (n[k] = ceil(end_bits[k] / 8), e.g. ie_last_end_bits): the encoder -> Huffman pipeline needs no
 * host round trip for the sizes.  The host can recover n[k] as the sum of string k's histogram. */
int ie_huffman_hist_batch_ends(ie_ctx* ctx, const uint8_t* in, size_t in_pitch, const uint64_t* end_bits,
                               int count, uint32_t* hist, uint64_t* first_pos);

/* The same, split for pipelining batches: _async launches the histogram and its read-back into
 * pinned slot `slot` (0 or 1) and returns at once; _wait blocks until that slot's read-back is
 * complete and copies out count*256 counts and first positions.  While the host builds the trees
 * of batch i (between _wait and ie_huffman_pack_batch), the device runs batch i+1's encode and
 * histogram.  Same reference interface as ie_huffman_hist_batch (Huffman.cpp:237-243). */
/* After ie_encode_images_counted over the same batch, _async is ONE launch that takes the
 * encoder's counts (and clears them for the next counted encode) and writes counts and first
 * positions straight into the pinned slot; a string with a value first seen past its first
 * 256 KiB is finished by _wait, so `in` must stay unchanged until _wait returns (the pack that
 * follows reads it anyway). */
int ie_huffman_hist_batch_ends_async(ie_ctx* ctx, const uint8_t* in, size_t in_pitch, const uint64_t* end_bits,
                                     int count, int slot);
int ie_huffman_hist_batch_wait(ie_ctx* ctx, int slot, uint32_t* hist, uint64_t* first_pos);

/* Batched re-encode (Huffman.cpp:314-319 for every string of the batch in one launch): string k
 * with the code table code/len[256*k ...] into out + k*out_pitch from bit start_bit[k].  The
 * bits before start_bit[k] (the dictionary, Huffman.cpp:283-311, or the '0' bit of the "no gain"
 * copy) come from prefix + k*prefix_pitch, so `out` needs no preparation; bits of the prefix
 * from start_bit[k] on are ignored.  in/out: device memory, out and out_pitch 4-byte aligned,
 * out_pitch >= (start_bit[k] + max_len_k * n[k] + 31) / 32 * 4.  Host arrays n, code, len,
 * prefix, start_bit are copied before the call returns.  end_bit (host, count entries) optional:
 * asking for it synchronises; without it the call is asynchronous on the context's stream. */
int ie_huffman_pack_batch(ie_ctx* ctx, const uint8_t* in, size_t in_pitch, const uint64_t* n, int count,
                          const uint32_t* code, const uint8_t* len, const uint8_t* prefix, size_t prefix_pitch,
                          uint8_t* out, size_t out_pitch, const uint64_t* start_bit, uint64_t* end_bit);

/* Device time of the last batched Huffman stage on the context's stream (HIP events around its
 * launches): stage 0 = the histogram / first-occurrence kernels of ie_huffman_hist_batch_ends_async,
 * stage 1 = the pack kernel of ie_huffman_pack_batch.  Only those two batched calls record the
 * events (two hipEventRecord each), and only while ie_set_stage_timing(ctx, 1) is in effect (off by
 * default: the timing events cost the pipelined C5 step about 15 us of device idle time); the
 * single-string ie_huffman_hist / ie_huffman_pack never do.  Waits for the stage to finish. */
int ie_last_stage_ms(ie_ctx* ctx, int stage, float* ms);
int ie_set_stage_timing(ie_ctx* ctx, int on);

/* Copy n bytes into out starting at bit start_bit, i.e. shifted by start_bit % 8 (the "no gain"
 * path of Huffman.cpp:329-341 writes '0' + the input: start_bit = 1).  Device input and output:
 * asynchronous on the context's stream, like an encode without sizes (checked at ie_sync). */
int ie_bitcopy(ie_ctx* ctx, const uint8_t* bytes, size_t n, uint8_t* out, size_t out_cap, uint64_t start_bit);

/* Huffman decode on the device (algo::Huffman<uint8_t>::decode, Huffman.cpp:354-402, replacing the
 * per-bit tree walk of Huffman.cpp:190-204): the symbols of the code stream `in` (len bytes, host or
 * device) from start_bit (just past the dictionary) to the END OF THE BUFFER -- the reference also
 * decodes the padding bits of the last byte, a code running past the end reads zero bits.  lut
 * (host or device): 32768 uint16 entries, lut[p] = sym | len << 8 for the code that prefixes the
 * 15-bit string p (len 0: none; codes are <= 15 bits, Huffman.cpp:41-42), built by the caller from
 * the dictionary.  out (host or device, out_cap bytes) receives the symbols; *nout their count
 * (also when IE_ECAP is returned).  IE_EFORMAT: a bit string that no code prefixes.  A device
 * stream (4-byte aligned) and a device lut are read in place, not copied; with a device out the
 * symbols are written as they are decoded, never past out_cap (on IE_ECAP the first out_cap
 * symbols are there), and the call synchronises once. */
/* The dictionary half of Huffman<uint8_t>::decode (buildTree, Huffman.cpp:120-173): parse the
 * dictionary of a Huffman-coded stream from bit start_bit of `in` (host memory, len bytes) into
 * ie_huffman_decode's prefix table lut (32768 entries); *code_start = the bit after its stop bit.
 * Returns 0, 1 when the stream has no dictionary (the data follows uncompressed from *code_start,
 * Huffman.cpp:361-371), or IE_EFORMAT when the dictionary runs past the buffer. */
int ie_huffman_table(const uint8_t* in, size_t len, uint64_t start_bit, uint16_t* lut, uint64_t* code_start);

int ie_huffman_decode(ie_ctx* ctx, const uint8_t* in, size_t len, uint64_t start_bit, const uint16_t* lut,
                      uint8_t* out, size_t out_cap, size_t* nout);

/* ---- Inverse path (ImageDecoder.cpp:55-122, Block.cpp:100-107,163-177,442-472) ------------
 * Decode nframes frames of block records starting at bit start_bit of `in` (len bytes) into
 * pixels (frame f row r at out + f*frame_pitch + r*stride).  Uses the quant matrix of
 * ie_set_quant.  end_bit optional. */
int ie_decode_frames(ie_ctx* ctx, const uint8_t* in, size_t len, uint64_t start_bit, int w, int h,
                     int nframes, int use_rle, uint8_t* out, size_t stride, size_t frame_pitch,
                     uint64_t* end_bit);

/* Video payload with P-frames (VideoDecoder.cpp:28-58, Frame.cpp:47-127, Block.cpp:441-496): frame f
 * an I-frame when f % gop == 0 (decoded as ie_decode_frames), otherwise a P-frame: its motion vectors
 * (bits_needed(merange) bits each), the previous decoded frame's blocks at the clamped vectors copied
 * into place, then a record for every microblock whose decoded error (IDCT + 128) is added to the
 * copied pixels (motioncomp != 0) or read and dropped (motioncomp == 0).  W and H multiples of 16
 * when P-frames exist (IE_EINVAL otherwise).  end_bit optional. */
int ie_decode_gop(ie_ctx* ctx, const uint8_t* in, size_t len, uint64_t start_bit, int w, int h, int nframes,
                  int gop, int merange, int use_rle, int motioncomp, uint8_t* out, size_t stride,
                  size_t frame_pitch, uint64_t* end_bit);

/* Chunks and composition levels of the last ie_decode_frames call's exact parse (diagnostics: the
 * stream is cut into chunks of about 32 (4x4) / 16 (8x8) records, each tabulated over every entry
 * offset; the tables are composed G at a time, level after level). */
int ie_last_decode_info(ie_ctx* ctx, int* chunks, int* levels);

/* Record-parse mode of ie_decode_frames / ie_decode_gop.  By default (exact != 0, any nonzero
 * value) the exact parse over composed transfer tables.  exact = 0: a call first parses
 * speculatively -- every chunk's entry is where a walk from its predecessor's first bit left it,
 * and the counting walks, each from its predecessor's speculative exit, verify every exit; on any
 * mismatch (periodic content, e.g. gradients) nothing is written and the exact parse runs.  Faster
 * only on flat content.
 * ie_set_spec_warm: the speculative parse's warm-up chunks (clamped to [0, 8], default 0) -- a
 * chunk's walk starts that many chunks earlier (the count pass's LDS bounds it further for long
 * chunks).  (Round 4 briefly encoded the warm-up as a negative `exact`; that meaning is gone: a
 * negative `exact` is nonzero, i.e. the exact parse, as before it.)
 * ie_last_decode_spec returns 1 when the last record decode was completed by the speculative
 * parse, 0 when by the exact one. */
int ie_set_exact_parse(ie_ctx* ctx, int exact);
int ie_set_spec_warm(ie_ctx* ctx, int warm);
int ie_last_decode_spec(ie_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
