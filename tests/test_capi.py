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


def _declared_host():
    src = open(os.path.join(ROOT, "include", "ie_host.hpp")).read()
    body = src[src.index('extern "C"'):]
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(ieh_\w+)\s*\(", body, flags=re.M)))


def test_host_library_exports_every_declared_symbol():
    import ctypes
    from imageencoder_amd import HOST_LIB_PATH, load_library
    assert os.path.exists(HOST_LIB_PATH), "libie_host.so not built"
    load_library()
    lib = ctypes.CDLL(HOST_LIB_PATH)
    names = _declared_host()
    assert {"ieh_encode_image", "ieh_encode_video", "ieh_decode_image", "ieh_huffman_encode"} <= set(names)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_no_oracle_in_product_libraries():
    """The product libraries must not link or embed the CPU oracle."""
    import subprocess
    from imageencoder_amd import HOST_LIB_PATH, LIB_PATH
    for p in (LIB_PATH, HOST_LIB_PATH):
        syms = subprocess.run(["nm", "-D", p], capture_output=True, text=True).stdout
        assert "ieo_" not in syms, p
        deps = subprocess.run(["ldd", p], capture_output=True, text=True).stdout
        assert "oracle" not in deps, p
