"""GPU parity of the streamed host path (include/ie_hip.h "Streamed host path"): host frames in and
host streams out through pinned double-buffered staging on three HIP streams, and the ie_vstream
video stream that continues one chain across launches on the device.  Bit-exact against the
reference's golden files, the oracle and the device-resident path.
"""
import hashlib

import numpy as np
import pytest

from imageencoder_amd import IE_ECAP, IEError, stream_bound, synth
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    from imageencoder_amd import Codec
    return Codec(0)


@pytest.fixture(scope="module")
def oracle():
    return O.load()


def _md5(b) -> str:
    return hashlib.md5(bytes(b)).hexdigest()


VIDEO = [c for c in O.manifest() if c["video"] and not c["huffman"] and c["n"] == 4]


@pytest.mark.parametrize("pattern", [[1], [2, 1], [3, 5]], ids=["by1", "by2-1", "by3-5"])
@pytest.mark.parametrize("c", VIDEO, ids=[c["name"] for c in VIDEO])
def test_vstream_pushes_build_the_reference_file(codec, oracle, c, pattern):
    """Frames pushed a few at a time (every push its own launch, chained on the device), bytes
    pulled between pushes: the concatenation is the reference encoder's file."""
    n, w, h = c["n"], c["w"], c["h"]
    q = O.read_matrix(c["matrix"], n)
    codec.set_quant(q, n)
    raw = O.case_input(c)
    pitch = w * h * 3 // 2
    frames = len(raw) // pitch
    hdr, hb = oracle.header(n, q, c["rle"], w, h, video=True, frames=frames, gop=1, merange=16)
    y = np.frombuffer(raw, dtype=np.uint8)
    vs = codec.open_video_stream(w, h, head=hdr, start_bit=hb, max_frames=frames, frame_pitch=pitch)
    out = np.zeros(stream_bound(w, h, n, frames, hb), dtype=np.uint8)
    got, f, i = 0, 0, 0
    while f < frames:
        k = min(pattern[i % len(pattern)], frames - f)
        vs.push(y[f * pitch:], k)
        f += k
        i += 1
        got += vs.pull(out, got)
    nb, end, fb = vs.finish(out, got)
    vs.close()
    got += nb
    assert got == (end + 7) // 8 and int(fb.sum()) == end - hb
    assert _md5(out[:got]) == c["md5"] and got == c["size"]


def test_vstream_rejects_frames_beyond_capacity(codec):
    codec.set_quant(O.read_matrix("matrix.txt", 4), 4)
    vs = codec.open_video_stream(64, 48, max_frames=2)
    y = np.zeros(64 * 48 * 3, dtype=np.uint8)
    with pytest.raises(IEError) as e:
        vs.push(y, 3)
    assert e.value.code == IE_ECAP
    vs.close()


@pytest.mark.parametrize("pinned", [False, True], ids=["pageable", "pinned"])
def test_streamed_frames_equal_the_oracle_stream(codec, oracle, pinned):
    """ie_encode_frames with host buffers and enough frames for several chunks (the video
    pipeline under the classic call) == the oracle's stream, from an odd start bit."""
    w, h, nf, start = 64, 48, 150, 165
    q = O.read_matrix("matrix.txt", 4)
    codec.set_quant(q, 4)
    frames = synth.frames("M", w, h, nf, seed=11)
    cap = stream_bound(w, h, 4, nf, start)
    head = np.random.default_rng(5).integers(0, 256, (start + 7) // 8, dtype=np.uint8)
    head[-1] &= np.uint8((0xFF00 >> (start % 8)) & 0xFF)
    if pinned:
        y = codec.host_array(frames.size)
        y[:] = frames.ravel()
        out = codec.host_array(cap)
        out[:] = 0
    else:
        y, out = frames.ravel(), np.zeros(cap, dtype=np.uint8)
    out[: head.size] = head
    fb, end = codec.encode_frames(y, w, h, out, start_bit=start, nframes=nf)
    ref = np.zeros(cap + 64, dtype=np.uint8)
    ref[: head.size] = head
    ref, ref_end, ref_fb = oracle.encode_blocks(frames.reshape(nf, h, w), 4, q, start_bit=start, out=ref)
    assert end == ref_end and list(fb) == list(ref_fb)
    assert _md5(out[: (end + 7) // 8]) == _md5(ref[: (end + 7) // 8])


@pytest.mark.parametrize("pinned", [False, True], ids=["pageable", "pinned"])
def test_streamed_images_equal_the_device_path(codec, pinned):
    """ie_encode_images with host buffers (chunks through the pinned slots, H2D / encode / D2H on
    three streams) == the same batch encoded device-resident, byte for byte, header bytes kept."""
    import torch
    w, h, nf, start = 640, 360, 19, 165
    codec.set_quant(O.read_matrix("matrix.txt", 4), 4)
    frames = synth.frames("U", w, h, nf, seed=7)
    pitch = (stream_bound(w, h, 4, 1, start) + 255) // 256 * 256
    rng = np.random.default_rng(3)
    heads = rng.integers(0, 256, (nf, (start + 7) // 8), dtype=np.uint8)
    heads[:, -1] &= np.uint8((0xFF00 >> (start % 8)) & 0xFF)
    if pinned:
        y = codec.host_array(frames.size)
        y[:] = frames.ravel()
        out = codec.host_array(pitch * nf)
        out[:] = 0
    else:
        y, out = frames.ravel(), np.zeros(pitch * nf, dtype=np.uint8)
    for f in range(nf):
        out[f * pitch: f * pitch + heads.shape[1]] = heads[f]
    ends = codec.encode_images(y, w, h, out, pitch, nf, start_bit=start)
    dout = torch.zeros(pitch * nf, dtype=torch.uint8, device="cuda")
    for f in range(nf):
        dout[f * pitch: f * pitch + heads.shape[1]] = torch.from_numpy(heads[f]).cuda()
    dends = codec.encode_images(torch.from_numpy(frames.ravel()).cuda(), w, h, dout, pitch, nf, start_bit=start)
    assert list(ends) == list(dends)
    d = dout.cpu().numpy()
    for f in range(nf):
        b = (int(ends[f]) + 7) // 8
        assert _md5(out[f * pitch: f * pitch + b]) == _md5(d[f * pitch: f * pitch + b]), f
