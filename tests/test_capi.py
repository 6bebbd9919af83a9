"""CPU checks of the C-ABI boundary: the library loads and exports every symbol the header
declares (no compute call -- there may be no GPU here)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "ie_hip.h")).read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(ie_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_api():
    names = _declared()
    for must in ("ie_create", "ie_destroy", "ie_set_quant", "ie_encode_frames", "ie_encode_images",
                 "ie_stream_bound", "ie_last_error", "ie_huffman_hist", "ie_huffman_pack", "ie_decode_frames"):
        assert must in names


def test_library_exports_every_declared_symbol():
    import ctypes
    from imageencoder_amd import LIB_PATH
    assert os.path.exists(LIB_PATH), "libie_hip.so not built"
    lib = ctypes.CDLL(LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_stream_bound_cpu():
    from imageencoder_amd import stream_bound
    # 4 + 17*16 bits per 4x4 block, whole 32-bit words
    assert stream_bound(8, 8, 4, 1, 0) == ((4 * 276 + 31) // 32) * 4
    assert stream_bound(8, 8, 8, 1, 165) == ((165 + 1044 + 31) // 32) * 4
    assert stream_bound(8, 8, 5, 1, 0) == 0
