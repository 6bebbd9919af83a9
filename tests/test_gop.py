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


DEC = [c for c in CASES if "dec1_md5" in c]


@pytest.mark.parametrize("c", DEC, ids=[c["name"] for c in DEC])
@pytest.mark.parametrize("mc", [1, 0])
def test_oracle_video_decode_matches_reference(c, mc):
    """The reference's VideoDecoder (Frame::loadFromStream, motion compensation on / off)."""
    dec = O.load().decode_video_gop(O.case_expected(c), 4, bool(mc))
    assert len(dec) == c[f"dec{mc}_size"]
    assert hashlib.md5(dec).hexdigest() == c[f"dec{mc}_md5"]


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


# ------------------------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def codec():
    from imageencoder_amd import Codec
    return Codec(0)


@pytest.mark.gpu
@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_gpu_gop_file_matches_reference(codec, c):
    """Whole video files (header + I/P payload) through libie_host.so -> ie_encode_gop."""
    from imageencoder_amd import MODE_FAST
    q = O.read_matrix(c["matrix"], 4)
    y = np.frombuffer(O.case_input(c), dtype=np.uint8)
    got = codec.encode_video_file(y, c["w"], c["h"], q, 4, rle=bool(c["rle"]), huffman=c["huffman"],
                                  merange=c["merange"], mode=MODE_FAST, gop=c["gop"])
    assert len(got) == c["size"], (len(got), c["size"])
    assert hashlib.md5(got).hexdigest() == c["md5"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["gopP64x48x5_g3_m8", "gopM64x48x5_g2_m0", "gopP64x40x4_g4_m8"])
def test_gpu_gop_exact_mode_and_huffman(codec, name):
    """EXACT mode gives the same file; the Huffman pass over a P-frame payload equals the
    oracle's (the reference's Huffman build aborts on P-frame videos, see make_golden_gop.py)."""
    from imageencoder_amd import MODE_EXACT
    c = next(c for c in CASES if c["name"] == name)
    q = O.read_matrix(c["matrix"], 4)
    raw = O.case_input(c)
    y = np.frombuffer(raw, dtype=np.uint8)
    got = codec.encode_video_file(y, c["w"], c["h"], q, 4, rle=bool(c["rle"]), huffman=False,
                                  merange=c["merange"], mode=MODE_EXACT, gop=c["gop"])
    assert hashlib.md5(got).hexdigest() == c["md5"]
    gh = codec.encode_video_file(y, c["w"], c["h"], q, 4, rle=bool(c["rle"]), huffman=True,
                                 merange=c["merange"], gop=c["gop"])
    assert gh == O.load().encode_video_gop(raw, c["w"], c["h"], 4, q, rle=c["rle"], huffman=True, gop=c["gop"],
                                           merange=c["merange"])


@pytest.mark.gpu
@pytest.mark.parametrize("n,gen,w,h,frames,gop,merange,start", [
    (8, "P", 64, 48, 5, 3, 8, 0),       # 8x8: motion vectors only (parity pinned by the oracle)
    (8, "M", 72, 24, 4, 4, 16, 7),
    (4, "P", 128, 96, 7, 4, 32, 13),    # odd start bit, device-resident frames and stream
    (4, "U", 48, 32, 6, 2, 6, 31),
    (4, "P", 256, 144, 9, 9, 64, 1),
])
def test_gpu_gop_payload_vs_oracle(codec, n, gen, w, h, frames, gop, merange, start):
    import torch
    from imageencoder_amd import synth
    q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
    y = synth.frames(gen, w, h, frames, synth.DEFAULT_SEED + 31 * w + h)
    exp, exp_end, exp_fb = O.load().encode_gop(y, n, q, gop, merange, start_bit=start)
    codec.set_quant(q, n)
    cap = codec.gop_stream_bound(w, h, frames, merange, start)
    dy = torch.from_numpy(y).cuda()
    out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    fb, end = codec.encode_gop(dy, w, h, out, gop, merange, start_bit=start, nframes=frames)
    assert end == exp_end
    assert list(fb) == list(exp_fb)
    nb = (end + 7) // 8
    assert out.cpu().numpy()[:nb].tobytes() == exp[:nb].tobytes()


@pytest.mark.gpu
def test_gpu_gop_rejects_misplaced_macroblocks(codec):
    from imageencoder_amd import IEError
    q = O.read_matrix("matrix.txt", 4)
    codec.set_quant(q, 4)
    y = np.zeros((2, 40, 72), dtype=np.uint8)
    out = np.zeros(codec.gop_stream_bound(72, 40, 2, 8), dtype=np.uint8)
    with pytest.raises(IEError):
        codec.encode_gop(y, 72, 40, out, 2, 8, nframes=2)
    # gop = 1 (no P-frame) stays valid at that size
    codec.encode_gop(y, 72, 40, out, 1, 8, nframes=2)


@pytest.mark.gpu
@pytest.mark.parametrize("c", DEC, ids=[c["name"] for c in DEC])
def test_gpu_video_decode_matches_reference(codec, c):
    """P-frame video files decoded through libie_host.so -> ie_decode_gop == the reference decoder."""
    dec, (w, h, f) = codec.decode_video_file(O.case_expected(c), 4)
    assert (w, h) == (c["w"], c["h"])
    assert len(dec) == c["dec1_size"]
    assert hashlib.md5(dec.tobytes()).hexdigest() == c["dec1_md5"]


@pytest.mark.gpu
@pytest.mark.parametrize("mc", [1, 0])
@pytest.mark.parametrize("name", ["gopP64x48x5_g3_m8", "gopM64x48x5_g2_m0", "gopM64x48x5_g3_m8_norle"])
def test_gpu_decode_gop_payload(codec, name, mc):
    """ie_decode_gop on a device-resident payload (motion compensation on / off) == the reference."""
    import torch
    c = next(c for c in DEC if c["name"] == name)
    q = O.read_matrix(c["matrix"], 4)
    codec.set_quant(q, 4)
    w, h = c["w"], c["h"]
    f = c["dec1_size"] // (w * h * 3 // 2)
    _, hb = O.load().header(4, q, c["rle"], w, h, video=True, frames=f, gop=c["gop"], merange=c["merange"])
    enc = np.frombuffer(O.case_expected(c), dtype=np.uint8)
    pitch = w * h * 3 // 2
    out = torch.full((f * pitch,), 0x80, dtype=torch.uint8, device="cuda")
    end = codec.decode_gop(torch.from_numpy(enc.copy()).cuda(), w, h, out, c["gop"], c["merange"], f, start_bit=hb,
                           frame_pitch=pitch, rle=bool(c["rle"]), motioncomp=bool(mc))
    assert (end + 7) // 8 == enc.size
    assert hashlib.md5(out.cpu().numpy().tobytes()).hexdigest() == c[f"dec{mc}_md5"]


@pytest.mark.gpu
@pytest.mark.parametrize("keep", [0.2, 0.5, 0.9, 0.999])
def test_gpu_decode_gop_truncated(codec, keep):
    """A truncated video payload fails with IE_EFORMAT (device-chained decode: the frames after the
    cut read an end bit no frame wrote and stay within the stream), and the context decodes the
    whole payload correctly afterwards."""
    import torch
    from imageencoder_amd import IEError
    c = next(c for c in DEC if c["name"] == "gopP64x48x5_g3_m8")
    q = O.read_matrix(c["matrix"], 4)
    codec.set_quant(q, 4)
    w, h = c["w"], c["h"]
    f = c["dec1_size"] // (w * h * 3 // 2)
    _, hb = O.load().header(4, q, c["rle"], w, h, video=True, frames=f, gop=c["gop"], merange=c["merange"])
    enc = np.frombuffer(O.case_expected(c), dtype=np.uint8)
    pitch = w * h * 3 // 2
    cut = hb // 8 + int((enc.size - hb // 8) * keep)
    out = torch.full((f * pitch,), 0x80, dtype=torch.uint8, device="cuda")
    with pytest.raises(IEError, match="stream ends"):
        codec.decode_gop(torch.from_numpy(enc[:cut].copy()).cuda(), w, h, out, c["gop"], c["merange"], f,
                         start_bit=hb, frame_pitch=pitch, rle=bool(c["rle"]), motioncomp=True)
    out.fill_(0x80)
    end = codec.decode_gop(torch.from_numpy(enc.copy()).cuda(), w, h, out, c["gop"], c["merange"], f, start_bit=hb,
                           frame_pitch=pitch, rle=bool(c["rle"]), motioncomp=True)
    assert (end + 7) // 8 == enc.size
    assert hashlib.md5(out.cpu().numpy().tobytes()).hexdigest() == c["dec1_md5"]


@pytest.mark.gpu
def test_gpu_gop_roundtrip_1080_multiple_of_16(codec):
    """Encode a 1920x1088 panning video with P-frames on the GPU, decode it on the GPU: the oracle's
    decode of the same file (parity pinned by the goldens above at small sizes)."""
    from imageencoder_amd import synth
    q = O.read_matrix("matrix.txt", 4)
    w, h, f = 1920, 1088, 4
    y = synth.frames("P", w, h, f, synth.DEFAULT_SEED + 99)
    enc = codec.encode_video_file(np.frombuffer(synth.yuv420(y), dtype=np.uint8), w, h, q, 4, huffman=False,
                                  merange=16, gop=4)
    assert enc == O.load().encode_video_gop(synth.yuv420(y), w, h, 4, q, gop=4, merange=16)
    dec, _ = codec.decode_video_file(enc, 4)
    assert dec.tobytes() == O.load().decode_video_gop(enc, 4)


@pytest.mark.gpu
@pytest.mark.parametrize("fake", [1, 2])
def test_gpu_gop_timeout_redo_clears_stream(fake, monkeypatch):
    """The look-back timeout recovery of ie_encode_gop (IE_FAKE_TIMEOUTS reports k timeouts): one
    timeout redoes the video in ticket mode on a device-resident stream whose first attempt already
    ORed vectors and records in -- the redo clears it from start_bit on and the result equals the
    reference's payload, the caller's bits before start_bit kept; a second timeout in ticket mode
    fails with IE_EDEVICE instead of recursing."""
    import torch
    from imageencoder_amd import Codec, IEError
    c = next(c for c in CASES if c["name"] == "gopP64x48x5_g3_m8")
    q = O.read_matrix(c["matrix"], 4)
    y = _frames(c)
    f = y.shape[0]
    hdr, hb = O.load().header(4, q, c["rle"], c["w"], c["h"], video=True, frames=f, gop=c["gop"],
                              merange=c["merange"])
    monkeypatch.setenv("IE_FAKE_TIMEOUTS", str(fake))
    codec = Codec(0, q, 4)
    try:
        cap = codec.gop_stream_bound(c["w"], c["h"], f, c["merange"], hb)
        head = np.zeros(cap, np.uint8)
        head[: len(hdr)] = hdr[:cap]
        out = torch.from_numpy(head).cuda()
        dy = torch.from_numpy(np.ascontiguousarray(y)).cuda()
        if fake == 2:
            with pytest.raises(IEError):
                codec.encode_gop(dy, c["w"], c["h"], out, c["gop"], c["merange"], start_bit=hb, nframes=f)
            return
        _, end = codec.encode_gop(dy, c["w"], c["h"], out, c["gop"], c["merange"], start_bit=hb, nframes=f)
        got = out.cpu().numpy()[: (end + 7) // 8].tobytes()
        assert got == O.case_expected(c)
    finally:
        codec.close()
