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

IE_OK, IE_EINVAL, IE_ECAP, IE_EHIP, IE_ENOQUANT, IE_EFORMAT, IE_EDEVICE = 0, -1, -2, -3, -4, -5, -6
MODE_FAST, MODE_EXACT = 0, 1

_lib = None


class IEError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ie error {code}: {msg}")
        self.code = code


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load libie_hip.so (raises if absent: the HIP path is the only path)."""
    global _lib
    if _lib is not None:
        return _lib
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
    L.ie_stream_bound.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64]
    L.ie_stream_bound.restype = C.c_size_t
    L.ie_encode_frames.argtypes = [vp, u8p, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                   u8p, C.c_size_t, C.c_uint64, u64p, u64p]
    L.ie_encode_images.argtypes = [vp, u8p, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                   u8p, C.c_size_t, C.c_uint64, u64p]
    L.ie_last_fallbacks.argtypes = [vp, u64p]
    L.ie_quantize_frames.argtypes = [vp, u8p, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int, vp]
    for name in ("ie_huffman_hist", "ie_huffman_pack", "ie_bitcopy", "ie_decode_frames"):
        if hasattr(L, name):
            getattr(L, name).restype = C.c_int
    if hasattr(L, "ie_huffman_hist"):
        L.ie_huffman_hist.argtypes = [vp, u8p, C.c_size_t, u32p, u64p]
        L.ie_huffman_pack.argtypes = [vp, u8p, C.c_size_t, u32p, u8p, u8p, C.c_size_t, C.c_uint64, u64p]
        L.ie_bitcopy.argtypes = [vp, u8p, C.c_size_t, u8p, C.c_size_t, C.c_uint64]
    if hasattr(L, "ie_decode_frames"):
        L.ie_decode_frames.argtypes = [vp, u8p, C.c_size_t, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int,
                                       u8p, C.c_size_t, C.c_size_t, u64p]
    _lib = L
    return L


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


def stream_bound(w: int, h: int, n: int, nframes: int = 1, start_bit: int = 0) -> int:
    return int(load_library().ie_stream_bound(w, h, n, nframes, start_bit))


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

    def encode_images(self, y, w: int, h: int, out, out_pitch: int, nframes: int, start_bit: int = 0,
                      stride: int | None = None, frame_pitch: int | None = None, rle: bool = True,
                      mode: int = MODE_FAST, want_sizes: bool = True):
        stride = w if stride is None else stride
        frame_pitch = stride * h if frame_pitch is None else frame_pitch
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

    def last_fallbacks(self) -> int:
        v = C.c_uint64(0)
        self._chk(self.L.ie_last_fallbacks(self.h, C.byref(v)))
        return int(v.value)
