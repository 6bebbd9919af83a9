"""Videos with P-frames (gop > 1): the oracle against the reference's own outputs (CPU), and the
HIP path through the C ABI against the goldens and the oracle (GPU).

Reference: VideoEncoder.cpp:22-107, VideoBase.cpp:96-122 (I-frame every gop frames),
Frame.cpp:129-247 (P-frame), Block.cpp:241-339 (SAD pattern search), algo.cpp:90-139 (pattern
tree), ImageBase.cpp:208-306 (macroblocks, prediction error per microblock).  8x8 P-frames have no
reference output (the reference's video path is hard-wired to Block<4>): they are checked against
the oracle only (parity unpinned by the reference).
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from tests import oracle_lib as O

CASES = O.manifest_gop()
SMALL = [c for c in CASES if c["size"] <= 64 * 1024]


def _frames(c):
    raw = np.frombuffer(O.case_input(c), dtype=np.uint8)
    w, h = c["w"], c["h"]
    pitch = w * h * 3 // 2
    f = raw.size // pitch
    return raw.reshape(f, pitch)[:, : w * h].reshape(f, h, w)


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_gop(c):
    o = O.load()
    q = O.read_matrix(c["matrix"], 4)
    enc = o.encode_video_gop(O.case_input(c), c["w"], c["h"], 4, q, rle=c["rle"], gop=c["gop"],
                             merange=c["merange"])
    assert len(enc) == c["size"]
    assert hashlib.md5(enc).hexdigest() == c["md5"]
    exp = O.case_expected(c)
    if exp is not None:
        assert enc == exp


def test_oracle_gop_payload_matches_file():
    """The payload entry (ieo_encode_gop) continues the header exactly as the file writer does."""
    o = O.load()
    c = next(c for c in CASES if c["name"] == "gopP64x48x5_g3_m8")
    q = O.read_matrix(c["matrix"], 4)
    y = _frames(c)
    hdr, hb = o.header(4, q, c["rle"], c["w"], c["h"], video=True, frames=y.shape[0], gop=c["gop"],
                       merange=c["merange"])
    buf, end, fb = o.encode_gop(y, 4, q, c["gop"], c["merange"], rle=c["rle"], start_bit=hb)
    # the file = header (its leading '0': no Huffman) + payload, whole bytes
    bits = np.concatenate([np.unpackbits(hdr)[:hb], np.unpackbits(buf)[hb:end]]).astype(np.uint8)
    data = np.packbits(bits).tobytes()
    assert data == O.case_expected(c)
    assert int(fb.sum()) == end - hb


def test_oracle_rejects_misplaced_macroblocks():
    """W % 16 != 0 with >= 2 macroblock rows: the reference's macroblocks overlap (rejected)."""
    o = O.load()
    q = O.read_matrix("matrix.txt", 4)
    y = np.zeros((2, 40, 72), dtype=np.uint8)
    with pytest.raises(AssertionError):
        o.encode_gop(y, 4, q, 2, 8)
