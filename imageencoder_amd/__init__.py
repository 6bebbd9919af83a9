"""imageencoder_amd -- MI355X-native (gfx950) implementation of ImageEncoder's block hot path.

The product is the C-ABI library ``lib/libie_hip.so`` (include/ie_hip.h); this module is a thin
ctypes binding over it for tests, the bench and Python callers.  It mirrors the reference's
encoder surface: a quantisation matrix (``MatrixReader``), block size N, ``use_rle``, and frame
encodes that append block records to a bit stream after a settings header
(``ImageEncoder::process``, ImageEncoder.cpp:52-175).

There is no CPU fallback: importing succeeds without the library, but constructing a
:class:`Codec` raises if ``libie_hip.so`` is missing or no HIP device is present.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIBDIR, "libie_hip.so")
HOST_LIB_PATH = os.path.join(LIBDIR, "libie_host.so")

IE_OK, IE_EINVAL, IE_ECAP, IE_EHIP, IE_ENOQUANT, IE_EFORMAT, IE_EDEVICE = 0, -1, -2, -3, -4, -5, -6
MODE_FAST, MODE_EXACT = 0, 1

_lib = None
_host = None


class IEError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ie error {code}: {msg}")
        self.code = code


def load_library(path: str | None = None) -> C.CDLL:
    """Load libie_hip.so (raises if absent: the HIP path is the only path).  IE_LIB overrides
    the path (kernel variants built by tools/variants.sh)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("IE_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise IEError(IE_EHIP, f"{path} not built -- run `make lib` (or __graft_entry__.build())")
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so (same SONAME as
    # /opt/rocm's).  Loading torch first makes our DT_NEEDED resolve to the copy torch already
    # mapped, so device pointers and streams from torch are valid in this library.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    vp, u8p, u16p, u32p, u64p = C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)
    L.ie_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.ie_destroy.argtypes = [vp]
    L.ie_last_error.argtypes = [vp]
    L.ie_last_error.restype = C.c_char_p
    L.ie_set_stream.argtypes = [vp, vp]
    L.ie_sync.argtypes = [vp]
    L.ie_set_quant.argtypes = [vp, u16p, C.c_int]
    L.ie_cos_table.argtypes = [vp, vp]
    L.ie_last_stage_ms.argtypes = [vp, C.c_int, C.POINTER(C.c_float)]
    L.ie_set_stage_timing.argtypes = [vp, C.c_int]
    L.ie_stream_bound.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64]
    L.ie_stream_bound.restype = C.c_size_t
    L.ie_encode_frames.argtypes = [vp, u8p, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                   u8p, C.c_size_t, C.c_uint64, u64p, u64p]
    L.ie_decode_gop.argtypes = [vp, u8p, C.c_size_t, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                C.c_int, u8p, C.c_size_t, C.c_size_t, u64p]
    L.ie_gop_stream_bound.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64]
    L.ie_gop_stream_bound.restype = C.c_size_t
    L.ie_encode_gop.argtypes = [vp, u8p, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                C.c_int, C.c_int, u8p, C.c_size_t, C.c_uint64, u64p, u64p]
    L.ie_encode_images.argtypes = [vp, u8p, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                   u8p, C.c_size_t, C.c_uint64, u64p]
    L.ie_encode_images_counted.argtypes = [vp, u8p, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int,
                                           C.c_int, u8p, C.c_size_t, C.c_uint64]
    L.ie_huffman_hist_batch_ends_async.argtypes = [vp, u8p, C.c_size_t, u64p, C.c_int, C.c_int]
    L.ie_huffman_hist_batch_wait.argtypes = [vp, C.c_int, vp, vp]
    L.ie_last_end_bits.argtypes = [vp]
    L.ie_last_end_bits.restype = C.c_void_p
    L.ie_last_fallbacks.argtypes = [vp, u64p]
    L.ie_quantize_frames.argtypes = [vp, u8p, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int, vp]
    for name in ("ie_huffman_hist", "ie_huffman_pack", "ie_bitcopy", "ie_decode_frames"):
        if hasattr(L, name):
            getattr(L, name).restype = C.c_int
    if hasattr(L, "ie_huffman_hist"):
        L.ie_huffman_hist.argtypes = [vp, u8p, C.c_size_t, u32p, u64p]
        L.ie_huffman_pack.argtypes = [vp, u8p, C.c_size_t, u32p, u8p, u8p, C.c_size_t, C.c_uint64, u64p]
        L.ie_bitcopy.argtypes = [vp, u8p, C.c_size_t, u8p, C.c_size_t, C.c_uint64]
    if hasattr(L, "ie_huffman_hist_batch"):
        L.ie_huffman_hist_batch.restype = C.c_int
        L.ie_huffman_hist_batch.argtypes = [vp, u8p, C.c_size_t, u64p, C.c_int, u32p, u64p]
        L.ie_huffman_pack_batch.restype = C.c_int
        L.ie_huffman_pack_batch.argtypes = [vp, u8p, C.c_size_t, u64p, C.c_int, u32p, u8p, u8p, C.c_size_t, u8p,
                                            C.c_size_t, u64p, u64p]
    if hasattr(L, "ie_decode_frames"):
        L.ie_decode_frames.argtypes = [vp, u8p, C.c_size_t, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int,
                                       u8p, C.c_size_t, C.c_size_t, u64p]
    L.ie_host_alloc.argtypes = [vp, C.c_size_t, C.POINTER(C.c_void_p)]
    L.ie_host_free.argtypes = [vp, vp]
    L.ie_vstream_open.argtypes = [vp, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int, u8p, C.c_uint64,
                                  C.c_int, C.POINTER(C.c_void_p)]
    L.ie_vstream_push.argtypes = [vp, u8p, C.c_int]
    L.ie_vstream_pull.argtypes = [vp, u8p, C.c_size_t, C.POINTER(C.c_size_t)]
    L.ie_vstream_finish.argtypes = [vp, u8p, C.c_size_t, C.POINTER(C.c_size_t), u64p, u64p]
    L.ie_vstream_device.argtypes = [vp]
    L.ie_vstream_device.restype = C.c_void_p
    L.ie_vstream_close.argtypes = [vp]
    L.ie_huffman_decode.argtypes = [vp, u8p, C.c_size_t, C.c_uint64, vp, u8p, C.c_size_t, C.POINTER(C.c_size_t)]
    L.ie_last_decode_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.ie_set_exact_parse.argtypes = [vp, C.c_int]
    L.ie_set_spec_warm.argtypes = [vp, C.c_int]
    L.ie_last_decode_spec.argtypes = [vp]
    L.ie_malloc.argtypes = [vp, C.c_size_t, C.POINTER(C.c_void_p)]
    L.ie_free.argtypes = [vp, vp]
    L.ie_memcpy.argtypes = [vp, vp, vp, C.c_size_t]
    L.ie_memset.argtypes = [vp, vp, C.c_int, C.c_size_t]
    L.ie_is_device_ptr.argtypes = [vp]
    _lib = L
    return L


def load_host_library(path: str | None = None) -> C.CDLL:
    """Load libie_host.so: the file-level encoders/decoders (include/ie_host.hpp).  With IE_LIB set
    (an A/B build of libie_hip.so) the libie_host.so beside it is used, so that both libraries
    are the same build."""
    global _host
    if _host is not None:
        return _host
    load_library()
    if path is None:
        alt = os.environ.get("IE_LIB")
        path = os.path.join(os.path.dirname(alt), "libie_host.so") if alt else HOST_LIB_PATH
    if not os.path.exists(path):
        raise IEError(IE_EHIP, f"{path} not built -- run `make host` (or __graft_entry__.build())")
    H = C.CDLL(path)
    vp, ip = C.c_void_p, C.POINTER(C.c_int)
    H.ieh_encode_image.argtypes = [vp, vp, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp,
                                   C.c_size_t]
    H.ieh_encode_video.argtypes = [vp, vp, C.c_size_t, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_int, vp, C.c_size_t]
    H.ieh_encode_video_gop.argtypes = [vp, vp, C.c_size_t, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_int, C.c_int, vp, C.c_size_t]
    H.ieh_decode_image.argtypes = [vp, vp, C.c_size_t, C.c_int, vp, C.c_size_t, ip, ip]
    H.ieh_decode_video.argtypes = [vp, vp, C.c_size_t, C.c_int, vp, C.c_size_t, ip, ip, ip]
    H.ieh_huffman_encode.argtypes = [vp, vp, C.c_size_t, vp, C.c_size_t]
    H.ieh_huffman_decode.argtypes = [vp, vp, C.c_size_t, vp, C.c_size_t, ip]
    H.ieh_huffman_table.argtypes = [vp, C.c_size_t, vp, C.POINTER(C.c_uint64)]
    H.ieh_huffman_table.restype = C.c_int
    H.ieh_huffman_encode_after_encode.argtypes = [vp, vp, C.c_size_t, C.c_int, vp, C.c_size_t, vp]
    H.ieh_huffman_encode_after_encode.restype = C.c_int
    H.ieh_huffman_begin_after_encode.argtypes = [vp, vp, C.c_size_t, C.c_int, C.c_int]
    H.ieh_huffman_begin_after_encode.restype = C.c_int
    H.ieh_huffman_finish_after_encode.argtypes = [vp, vp, C.c_size_t, C.c_int, C.c_int, vp, C.c_size_t, vp]
    H.ieh_huffman_finish_after_encode.restype = C.c_int
    H.ieh_write_header.argtypes = [vp, C.c_size_t, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_int, C.c_int, C.c_int]
    H.ieh_write_header.restype = C.c_int64
    H.ieh_huffman_encode_device.argtypes = [vp, vp, C.c_size_t, vp, C.c_size_t]
    H.ieh_huffman_encode_device.restype = C.c_int64
    H.ieh_huffman_encode_device_batch.argtypes = [vp, vp, C.c_size_t, vp, C.c_int, vp, C.c_size_t, vp]
    H.ieh_huffman_encode_device_batch.restype = C.c_int
    H.ieh_release.argtypes = [vp]
    H.ieh_release.restype = None
    for f in ("ieh_encode_image", "ieh_encode_video", "ieh_encode_video_gop", "ieh_decode_image", "ieh_decode_video", "ieh_huffman_encode",
              "ieh_huffman_decode"):
        getattr(H, f).restype = C.c_int64
    _host = H
    return H


def _ptr(a):
    """Address of a numpy array or a torch tensor (host or device)."""
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    raise TypeError(type(a))


def _nbytes(a) -> int:
    if isinstance(a, np.ndarray):
        return a.nbytes
    return a.numel() * a.element_size()


def write_header(n: int, q, rle: bool, w: int, h: int, huffman: bool = False, video: bool = False,
                 frames: int = 0, gop: int = 1, merange: int = 0):
    """Settings header bytes + bit length (host library; ImageEncoder.cpp:84-94, VideoEncoder.cpp:60-73)."""
    H = load_host_library()
    q = np.ascontiguousarray(np.asarray(q, dtype=np.uint16).ravel())
    out = np.zeros(256, dtype=np.uint8)
    bits = H.ieh_write_header(out.ctypes.data, out.size, n, q.ctypes.data, int(rle), w, h, int(huffman),
                              int(video), frames, gop, merange)
    if bits < 0:
        raise IEError(int(bits), "ieh_write_header")
    return out[: (bits + 7) // 8].copy(), int(bits)


def read_matrix(path: str, n: int) -> np.ndarray:
    """A quantisation matrix file: n*n whitespace-separated unsigned values, row-major
    (dc::MatrixReader<N>::read, MatrixReader.cpp:65-134).  Raises ValueError on a malformed file."""
    with open(path) as f:
        vals = [int(t) for t in f.read().split()]
    if len(vals) != n * n or any(v <= 0 or v > 0xFFFF for v in vals):
        raise ValueError(f"{path}: expected {n * n} values in 1..65535, got {len(vals)}")
    return np.array(vals, dtype=np.uint16)


def stream_bound(w: int, h: int, n: int, nframes: int = 1, start_bit: int = 0) -> int:
    return int(load_library().ie_stream_bound(w, h, n, nframes, start_bit))


class _PinnedOwner:
    """Frees an ie_host_alloc block when the numpy array viewing it is collected."""
    _live = {}

    @classmethod
    def attach(cls, arr, codec, addr):
        import weakref
        key = id(arr)
        cls._live[key] = weakref.finalize(arr, cls._free, codec, addr, key)

    @classmethod
    def _free(cls, codec, addr, key):
        cls._live.pop(key, None)
        if getattr(codec, "h", None):
            codec.L.ie_host_free(codec.h, C.c_void_p(addr))


class VideoStream:
    """ie_vstream_*: push host frames, pull finished stream bytes, finish (see include/ie_hip.h)."""

    def __init__(self, codec, w, h, head, start_bit, max_frames, stride, frame_pitch, rle, mode):
        self.c = codec
        self.w, self.h = w, h
        self.stride = w if stride is None else stride
        self.frame_pitch = self.stride * h if frame_pitch is None else frame_pitch
        head = np.zeros(1, dtype=np.uint8) if head is None else np.ascontiguousarray(head, dtype=np.uint8)
        self._head = head
        v = C.c_void_p()
        codec._chk(codec.L.ie_vstream_open(codec.h, w, h, self.stride, self.frame_pitch, int(rle), mode,
                                           head.ctypes.data, start_bit, max_frames, C.byref(v)))
        self.v = v
        self.max_frames = max_frames
        self.pushed = 0
        self.cap = stream_bound(w, h, codec.n, max_frames, start_bit)

    def push(self, frames, nframes: int):
        self.c._chk(self.c.L.ie_vstream_push(self.v, _ptr(frames), nframes))
        self.pushed += nframes

    def pull(self, dst: np.ndarray, offset: int) -> int:
        """Finished bytes into dst[offset:]; returns how many."""
        n = C.c_size_t(0)
        self.c._chk(self.c.L.ie_vstream_pull(self.v, dst.ctypes.data + offset, dst.size - offset, C.byref(n)))
        return int(n.value)

    def finish(self, dst: np.ndarray | None = None, offset: int = 0):
        """Remaining bytes into dst[offset:] (if given); returns (nbytes, end_bit, frame_bits)."""
        n, end = C.c_size_t(0), C.c_uint64(0)
        fb = np.zeros(max(self.pushed, 1), dtype=np.uint64)
        dp = dst.ctypes.data + offset if dst is not None else None
        cap = dst.size - offset if dst is not None else 0
        self.c._chk(self.c.L.ie_vstream_finish(self.v, dp, cap, C.byref(n), C.byref(end),
                                               fb.ctypes.data_as(C.POINTER(C.c_uint64))))
        return int(n.value), int(end.value), fb[: self.pushed]

    def device_ptr(self) -> int:
        return int(self.c.L.ie_vstream_device(self.v) or 0)

    def close(self):
        if getattr(self, "v", None):
            self.c.L.ie_vstream_close(self.v)
            self.v = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Codec:
    """One device context (``ie_ctx``) with its quantisation tables."""

    def __init__(self, device: int = 0, quant=None, n: int | None = None):
        self.L = load_library()
        h = C.c_void_p()
        r = self.L.ie_create(device, C.byref(h))
        if r != IE_OK:
            raise IEError(r, "ie_create failed (no HIP device?)")
        self.h = h
        self.n = None
        if quant is not None:
            self.set_quant(quant, n)

    def close(self):
        if getattr(self, "h", None):
            if _host is not None:
                _host.ieh_release(self.h)
            self.L.ie_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, r: int):
        if r != IE_OK:
            raise IEError(r, self.L.ie_last_error(self.h).decode())

    def set_stream(self, stream_handle: int | None):
        self._chk(self.L.ie_set_stream(self.h, stream_handle))

    def sync(self):
        self._chk(self.L.ie_sync(self.h))

    def set_quant(self, q, n: int | None = None):
        q = np.ascontiguousarray(np.asarray(q, dtype=np.uint16).ravel())
        if n is None:
            n = int(round(q.size ** 0.5))
        assert q.size == n * n
        self._chk(self.L.ie_set_quant(self.h, q.ctypes.data, n))
        self.n = n

    def set_stage_timing(self, on: bool) -> None:
        """Record HIP events around the batched Huffman stages (for :meth:`last_stage_ms`; off by
        default, the events delay the pipelined launches)."""
        self._chk(self.L.ie_set_stage_timing(self.h, int(bool(on))))

    def last_stage_ms(self, stage: int) -> float:
        """Device time (ms) of the last batched Huffman histogram (0) or pack (1) (ie_last_stage_ms)."""
        v = C.c_float()
        self._chk(self.L.ie_last_stage_ms(self.h, stage, C.byref(v)))
        return float(v.value)

    def cos_table(self) -> np.ndarray:
        """The cos table the kernels use (read back from the device; ie_cos_table), n x n doubles."""
        out = np.zeros(self.n * self.n, np.float64)
        self._chk(self.L.ie_cos_table(self.h, out.ctypes.data))
        return out.reshape(self.n, self.n)

    def encode_frames(self, y, w: int, h: int, out, start_bit: int = 0, stride: int | None = None,
                      frame_pitch: int | None = None, nframes: int = 1, rle: bool = True,
                      mode: int = MODE_FAST, want_sizes: bool = True):
        """Append the block records of ``nframes`` frames to ``out`` from ``start_bit``.
        ``y``/``out``: numpy arrays (host) or torch tensors (device).  Returns
        ``(frame_bits, end_bit)`` or ``None`` when ``want_sizes`` is False (async)."""
        stride = w if stride is None else stride
        frame_pitch = stride * h if frame_pitch is None else frame_pitch
        fb = np.zeros(nframes, dtype=np.uint64)
        end = C.c_uint64(0)
        fbp = fb.ctypes.data_as(C.POINTER(C.c_uint64)) if want_sizes else None
        endp = C.pointer(end) if want_sizes else None
        self._chk(self.L.ie_encode_frames(self.h, _ptr(y), w, h, stride, frame_pitch, nframes, int(rle), mode,
                                          _ptr(out), _nbytes(out), start_bit, fbp, endp))
        if not want_sizes:
            return None
        return fb, int(end.value)

    def gop_stream_bound(self, w: int, h: int, nframes: int, merange: int, start_bit: int = 0) -> int:
        return int(self.L.ie_gop_stream_bound(w, h, self.n, nframes, merange, start_bit))

    def encode_gop(self, y, w: int, h: int, out, gop: int, merange: int, start_bit: int = 0,
                   stride: int | None = None, frame_pitch: int | None = None, nframes: int = 1, rle: bool = True,
                   mode: int = MODE_FAST):
        """The payload of a video with I- and P-frames (frame f is an I-frame when f % gop == 0;
        VideoEncoder.cpp:83-91, Frame.cpp:129-247) appended to ``out`` from ``start_bit``; ``out``
        holds :meth:`gop_stream_bound` bytes.  Returns ``(frame_bits, end_bit)``."""
        stride = w if stride is None else stride
        frame_pitch = stride * h if frame_pitch is None else frame_pitch
        fb = np.zeros(nframes, dtype=np.uint64)
        end = C.c_uint64(0)
        self._chk(self.L.ie_encode_gop(self.h, _ptr(y), w, h, stride, frame_pitch, nframes, gop, merange, int(rle),
                                       mode, _ptr(out), _nbytes(out), start_bit,
                                       fb.ctypes.data_as(C.POINTER(C.c_uint64)), C.pointer(end)))
        return fb, int(end.value)

    def decode_gop(self, stream, w: int, h: int, out, gop: int, merange: int, nframes: int, start_bit: int = 0,
                   length: int | None = None, stride: int | None = None, frame_pitch: int | None = None,
                   rle: bool = True, motioncomp: bool = True) -> int:
        """Decode an I/P-frame payload (VideoDecoder / Frame::loadFromStream) into ``out``; the end bit."""
        stride = w if stride is None else stride
        frame_pitch = stride * h if frame_pitch is None else frame_pitch
        end = C.c_uint64(0)
        self._chk(self.L.ie_decode_gop(self.h, _ptr(stream), _nbytes(stream) if length is None else length, start_bit,
                                       w, h, nframes, gop, merange, int(rle), int(motioncomp), _ptr(out), stride,
                                       frame_pitch, C.pointer(end)))
        return int(end.value)

    def encode_images(self, y, w: int, h: int, out, out_pitch: int, nframes: int, start_bit: int = 0,
                      stride: int | None = None, frame_pitch: int | None = None, rle: bool = True,
                      mode: int = MODE_FAST, want_sizes: bool = True, count_bytes: bool = False):
        """count_bytes (device ``out``): also count every image's stream bytes for the following
        Huffman pass (:meth:`huffman_begin_after_encode` then skips its histogram kernel);
        implies want_sizes=False."""
        stride = w if stride is None else stride
        frame_pitch = stride * h if frame_pitch is None else frame_pitch
        if count_bytes:
            self._chk(self.L.ie_encode_images_counted(self.h, _ptr(y), w, h, stride, frame_pitch, nframes, int(rle),
                                                      mode, _ptr(out), out_pitch, start_bit))
            return None
        eb = np.zeros(nframes, dtype=np.uint64)
        ebp = eb.ctypes.data_as(C.POINTER(C.c_uint64)) if want_sizes else None
        self._chk(self.L.ie_encode_images(self.h, _ptr(y), w, h, stride, frame_pitch, nframes, int(rle), mode,
                                          _ptr(out), out_pitch, start_bit, ebp))
        return eb if want_sizes else None

    def quantize_frames(self, y, w: int, h: int, nframes: int = 1, stride: int | None = None,
                        frame_pitch: int | None = None, mode: int = MODE_FAST) -> np.ndarray:
        """Quantised coefficients (natural order) of every block: shape (blocks, n*n) int16."""
        stride = w if stride is None else stride
        frame_pitch = stride * h if frame_pitch is None else frame_pitch
        n = self.n
        coef = np.zeros((nframes * (w // n) * (h // n), n * n), dtype=np.int16)
        self._chk(self.L.ie_quantize_frames(self.h, _ptr(y), w, h, stride, frame_pitch, nframes, mode,
                                            coef.ctypes.data))
        return coef

    def host_array(self, nbytes: int) -> np.ndarray:
        """A uint8 numpy array in page-locked host memory (ie_host_alloc): host buffers the
        streamed path DMAs directly.  Freed when the array (and the codec) are gone."""
        p = C.c_void_p()
        self._chk(self.L.ie_host_alloc(self.h, nbytes, C.byref(p)))
        buf = (C.c_uint8 * nbytes).from_address(p.value)
        arr = np.frombuffer(buf, dtype=np.uint8)
        _PinnedOwner.attach(arr, self, p.value)
        return arr

    def open_video_stream(self, w: int, h: int, head=None, start_bit: int = 0, max_frames: int = 1,
                          stride: int | None = None, frame_pitch: int | None = None, rle: bool = True,
                          mode: int = MODE_FAST) -> "VideoStream":
        """ie_vstream_open: a gop=1 video payload grown on the device from host frames pushed over
        time (Frame.cpp:31-45 / VideoEncoder.cpp:83-91)."""
        return VideoStream(self, w, h, head, start_bit, max_frames, stride, frame_pitch, rle, mode)

    def end_bits_into(self, dst, count: int = 1):
        """Stream-ordered device copy of the last encode's end bit(s) (one per chain) into the
        device tensor ``dst`` (uint64/int64): no host read-back."""
        src = self.L.ie_last_end_bits(self.h)
        self._chk(self.L.ie_memcpy(self.h, C.c_void_p(_ptr(dst)), C.c_void_p(src), 8 * count))

    def last_decode_info(self) -> tuple[int, int]:
        """(chunks, composition levels) of the last record decode's exact parse (ie_last_decode_info)."""
        f, r = C.c_int(0), C.c_int(0)
        self._chk(self.L.ie_last_decode_info(self.h, C.byref(f), C.byref(r)))
        return int(f.value), int(r.value)

    def set_exact_parse(self, exact: bool, warm: int = 0) -> None:
        """Record decodes parse exactly (composed transfer tables) instead of speculatively first
        (ie_set_exact_parse); a speculative parse may start each chunk's walk ``warm`` (<= 8)
        chunks early."""
        self._chk(self.L.ie_set_spec_warm(self.h, int(warm)))
        self._chk(self.L.ie_set_exact_parse(self.h, 1 if exact else 0))

    def last_decode_spec(self) -> bool:
        """True when the last record decode was completed by the speculative parse."""
        return bool(self.L.ie_last_decode_spec(self.h))

    def last_fallbacks(self) -> int:
        v = C.c_uint64(0)
        self._chk(self.L.ie_last_fallbacks(self.h, C.byref(v)))
        return int(v.value)

    # ---- Huffman post-pass (Huffman.cpp:233-344) and the inverse path
    def huffman_hist(self, data):
        """(hist[256] uint32, first_pos[256] uint64) of the bytes in ``data`` (host or device)."""
        hist = np.zeros(256, dtype=np.uint32)
        first = np.zeros(256, dtype=np.uint64)
        self._chk(self.L.ie_huffman_hist(self.h, _ptr(data), _nbytes(data), hist.ctypes.data,
                                         first.ctypes.data_as(C.POINTER(C.c_uint64))))
        return hist, first

    def huffman_pack(self, data, code, length, out, start_bit: int = 0) -> int:
        code = np.ascontiguousarray(code, dtype=np.uint32)
        length = np.ascontiguousarray(length, dtype=np.uint8)
        end = C.c_uint64(0)
        self._chk(self.L.ie_huffman_pack(self.h, _ptr(data), _nbytes(data), code.ctypes.data, length.ctypes.data,
                                         _ptr(out), _nbytes(out), start_bit, C.byref(end)))
        return int(end.value)

    def bitcopy(self, data, out, start_bit: int):
        self._chk(self.L.ie_bitcopy(self.h, _ptr(data), _nbytes(data), _ptr(out), _nbytes(out), start_bit))

    def decode_frames(self, stream, w: int, h: int, out, start_bit: int = 0, nframes: int = 1, rle: bool = True,
                      stride: int | None = None, frame_pitch: int | None = None, length: int | None = None) -> int:
        """Decode ``nframes`` frames of block records from bit ``start_bit``; returns the end bit."""
        stride = w if stride is None else stride
        frame_pitch = stride * h if frame_pitch is None else frame_pitch
        end = C.c_uint64(0)
        n = _nbytes(stream) if length is None else length
        self._chk(self.L.ie_decode_frames(self.h, _ptr(stream), n, start_bit, w, h, nframes, int(rle), _ptr(out),
                                          stride, frame_pitch, C.byref(end)))
        return int(end.value)

    # ---- whole files (libie_host.so, include/ie_host.hpp)
    def _host_chk(self, r: int) -> int:
        if r < 0:
            raise IEError(int(r), self.L.ie_last_error(self.h).decode())
        return int(r)

    def encode_image_file(self, y, w: int, h: int, q, n: int, rle: bool = True, huffman: bool = True,
                          mode: int = MODE_FAST) -> bytes:
        H = load_host_library()
        q = np.ascontiguousarray(np.asarray(q, dtype=np.uint16).ravel())
        cap = stream_bound(w, h, n, 1, 2048) + 64
        out = np.zeros(cap, dtype=np.uint8)
        r = self._host_chk(H.ieh_encode_image(self.h, _ptr(y), w, h, q.ctypes.data, n, int(rle), int(huffman), mode,
                                              out.ctypes.data, cap))
        return out[:r].tobytes()

    def encode_video_file(self, yuv, w: int, h: int, q, n: int, rle: bool = True, huffman: bool = True,
                          merange: int = 0, mode: int = MODE_FAST, gop: int = 1) -> bytes:
        """A video file as VideoEncoder writes it; gop > 1 adds P-frames (motion search + coded
        prediction error, Frame.cpp:160-243)."""
        H = load_host_library()
        q = np.ascontiguousarray(np.asarray(q, dtype=np.uint16).ravel())
        frames = _nbytes(yuv) // (w * h + w * h // 2)
        cap = stream_bound(w, h, n, max(frames, 1), 2048) + (w // 16) * (h // 16) * 4 * max(frames, 1) + 64
        out = np.zeros(cap, dtype=np.uint8)
        r = self._host_chk(H.ieh_encode_video_gop(self.h, _ptr(yuv), _nbytes(yuv), w, h, q.ctypes.data, n, int(rle),
                                                  int(huffman), gop, merange, mode, out.ctypes.data, cap))
        return out[:r].tobytes()

    def decode_image_file(self, data: bytes, n: int):
        """Pixels (h, w) uint8 of an encoded image file (ImageDecoder)."""
        H = load_host_library()
        src = np.frombuffer(data, dtype=np.uint8).copy()
        w, h = C.c_int(0), C.c_int(0)
        cap = 32767 * 32767
        # size from the header first: decode into a small buffer to learn w, h
        r = H.ieh_decode_image(self.h, src.ctypes.data, src.size, n, src.ctypes.data, 0, C.byref(w), C.byref(h))
        if r != IE_ECAP:
            self._host_chk(r)
        cap = w.value * h.value
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        r = self._host_chk(H.ieh_decode_image(self.h, src.ctypes.data, src.size, n, out.ctypes.data, cap, C.byref(w),
                                              C.byref(h)))
        return out[:r].reshape(h.value, w.value)

    def decode_video_file(self, data: bytes, n: int):
        """Decoded YUV420 frames (Y + 0x80 UV fill), flat uint8, plus (w, h, frames)."""
        H = load_host_library()
        src = np.frombuffer(data, dtype=np.uint8).copy()
        w, h, f = C.c_int(0), C.c_int(0), C.c_int(0)
        r = H.ieh_decode_video(self.h, src.ctypes.data, src.size, n, src.ctypes.data, 0, C.byref(w), C.byref(h),
                               C.byref(f))
        if r != IE_ECAP:
            self._host_chk(r)
        cap = (w.value * h.value + w.value * h.value // 2) * f.value
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        r = self._host_chk(H.ieh_decode_video(self.h, src.ctypes.data, src.size, n, out.ctypes.data, cap, C.byref(w),
                                              C.byref(h), C.byref(f)))
        return out[:r], (w.value, h.value, f.value)

    def huffman_encode_device(self, data, nbytes: int, out) -> int:
        """Huffman pass from device ``data[:nbytes]`` into device ``out``; returns output bytes."""
        H = load_host_library()
        return self._host_chk(H.ieh_huffman_encode_device(self.h, _ptr(data), nbytes, _ptr(out), _nbytes(out)))

    def huffman_encode_batch(self, data, in_pitch: int, sizes, out, out_pitch: int) -> list[int]:
        """Huffman pass over a batch of device strings (string k: ``sizes[k]`` bytes at
        ``data + k*in_pitch``) into device ``out + k*out_pitch``: one histogram launch, host tree
        builds, one pack launch (asynchronous on the context's stream).  Returns output bytes."""
        H = load_host_library()
        k = len(sizes)
        n = np.asarray(sizes, dtype=np.uint64)
        nb = np.zeros(k, dtype=np.int64)
        self._host_chk(H.ieh_huffman_encode_device_batch(self.h, _ptr(data), in_pitch, n.ctypes.data, k, _ptr(out),
                                                         out_pitch, nb.ctypes.data))
        return [int(v) for v in nb]

    def huffman_encode_after_encode(self, out, out_pitch: int, count: int, hout, hpitch: int) -> list[int]:
        """The batched Huffman pass over the ``count`` images the last :meth:`encode_images` call
        wrote to device ``out`` (lengths from the encoder's end bits, on the device: no size
        read-back).  Returns the Huffman output bytes per image."""
        H = load_host_library()
        nb = np.zeros(count, dtype=np.int64)
        self._host_chk(H.ieh_huffman_encode_after_encode(self.h, _ptr(out), out_pitch, count, _ptr(hout), hpitch,
                                                         nb.ctypes.data))
        return [int(v) for v in nb]

    def huffman_begin_after_encode(self, out, out_pitch: int, count: int, slot: int) -> None:
        """First half of :meth:`huffman_encode_after_encode` for pipelining batches: launches the
        histogram of the last :meth:`encode_images` output and returns (read-back into ``slot``,
        0 or 1).  Finish it with :meth:`huffman_finish_after_encode` on the same arguments after
        issuing the next batch's encode and begin."""
        H = load_host_library()
        self._host_chk(H.ieh_huffman_begin_after_encode(self.h, _ptr(out), out_pitch, count, slot))

    def huffman_finish_after_encode(self, out, out_pitch: int, count: int, slot: int, hout, hpitch: int) -> list[int]:
        """Second half: trees for the batch begun in ``slot``, then the pack launch into ``hout``.
        Returns the Huffman output bytes per image (``out`` must still hold that batch)."""
        H = load_host_library()
        nb = np.zeros(count, dtype=np.int64)
        self._host_chk(H.ieh_huffman_finish_after_encode(self.h, _ptr(out), out_pitch, count, slot, _ptr(hout), hpitch,
                                                         nb.ctypes.data))
        return [int(v) for v in nb]

    def huffman_hist_after_encode(self, out, out_pitch: int, count: int):
        """(hist [count, 256] uint32, first [count, 256] uint64) of the images the last encode
        wrote (counts fused into the encoder when it ran with count_bytes=True)."""
        u64p = C.POINTER(C.c_uint64)
        ends = C.cast(C.c_void_p(self.L.ie_last_end_bits(self.h)), u64p)
        self._chk(self.L.ie_huffman_hist_batch_ends_async(self.h, _ptr(out), out_pitch, ends, count, 0))
        hist = np.zeros((count, 256), dtype=np.uint32)
        first = np.zeros((count, 256), dtype=np.uint64)
        self._chk(self.L.ie_huffman_hist_batch_wait(self.h, 0, hist.ctypes.data, first.ctypes.data))
        return hist, first

    def huffman_table(self, data: bytes):
        """(lut uint16[32768], start_bit) of a Huffman-coded stream's dictionary, or None when the
        stream has none (passthrough)."""
        H = load_host_library()
        src = np.frombuffer(data, dtype=np.uint8)
        lut = np.zeros(32768, dtype=np.uint16)
        sb = C.c_uint64(0)
        r = H.ieh_huffman_table(src.ctypes.data, src.size, lut.ctypes.data, C.byref(sb))
        if r < 0:
            raise IEError(r, "ieh_huffman_table")
        return None if r == 1 else (lut, int(sb.value))

    def huffman_decode_device(self, stream, nbytes: int, lut, start_bit: int, out) -> int:
        """ie_huffman_decode with device-resident stream / table / output (torch tensors): the
        symbol count (raises on IE_ECAP / malformed streams)."""
        n = C.c_size_t(0)
        self._chk(self.L.ie_huffman_decode(self.h, _ptr(stream), nbytes, start_bit, _ptr(lut), _ptr(out),
                                           _nbytes(out), C.byref(n)))
        return int(n.value)

    def huffman_decode(self, data: bytes):
        """The Huffman decode alone (device bit walk): (decoded bytes, passthrough)."""
        H = load_host_library()
        src = np.frombuffer(bytes(data), dtype=np.uint8).copy()
        cap = 8 * src.size + 16
        out = np.zeros(cap, dtype=np.uint8)
        pt = C.c_int(0)
        r = self._host_chk(H.ieh_huffman_decode(self.h, src.ctypes.data, src.size, out.ctypes.data, cap, C.byref(pt)))
        return out[:r].tobytes(), bool(pt.value)

    def huffman_encode(self, data) -> bytes:
        """The Huffman post-pass alone (host or device input)."""
        H = load_host_library()
        n = _nbytes(data)
        cap = 4 * n + 4096
        out = np.zeros(cap, dtype=np.uint8)
        r = self._host_chk(H.ieh_huffman_encode(self.h, _ptr(data), n, out.ctypes.data, cap))
        return out[:r].tobytes()
