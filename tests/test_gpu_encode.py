"""GPU parity: the HIP encoder (through the C-ABI) against the reference's golden streams and the
CPU oracle.  Bit-exact is the only bar (integer/byte output).
"""
import hashlib
import os

import numpy as np
import pytest

from imageencoder_amd import MODE_EXACT, MODE_FAST, synth
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    from imageencoder_amd import Codec
    return Codec(0)


def _md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


def _gpu_file(codec, oracle, c, raw: bytes, mode: int) -> bytes:
    """Whole reference file: the oracle writes the settings header (host side), the GPU
    appends every block record after it."""
    from imageencoder_amd import stream_bound
    n, w, h = c["n"], c["w"], c["h"]
    q = O.read_matrix(c["matrix"], n)
    codec.set_quant(q, n)
    if c["video"]:
        pitch = w * h * 3 // 2
        frames = len(raw) // pitch
        hdr, hb = oracle.header(n, q, c["rle"], w, h, video=True, frames=frames, gop=1, merange=16)
        y = np.frombuffer(raw, dtype=np.uint8)
    else:
        frames, pitch = 1, w * h
        hdr, hb = oracle.header(n, q, c["rle"], w, h)
        y = np.frombuffer(raw, dtype=np.uint8)
    out = np.zeros(stream_bound(w, h, n, frames, hb), dtype=np.uint8)
    m = min(len(hdr), len(out))
    out[:m] = hdr[:m]  # header bits, zero from bit hb on
    fb, end = codec.encode_frames(y, w, h, out, start_bit=hb, frame_pitch=pitch, nframes=frames,
                                  rle=bool(c["rle"]), mode=mode)
    assert int(fb.sum()) == end - hb
    return out[: (end + 7) // 8].tobytes()


def _golden(nonhuff_only=True, big=False):
    cs = []
    for c in O.manifest():
        if nonhuff_only and c["huffman"]:
            continue
        is_big = c["w"] * c["h"] >= 1920 * 1080
        if is_big == big:
            cs.append(c)
    return cs


EX_DIMS = {"ex0": (8, 8), "ex1": (936, 936), "ex2": (512, 512), "ex3": (400, 400), "ex4": (4096, 912),
           "ex6": (512, 256)}


@pytest.mark.parametrize("n,matrix", [(4, "matrix.txt"), (8, "matrix8_1.txt"), (4, "matrix4_2.txt"),
                                      (8, "matrix8_2.txt")])
def test_cos_table_pinned_on_device(codec, n, matrix):
    """the cos table this box's libm produced for ie_set_quant -- read back from the
    device, i.e. what the FP64 paths multiply with -- equals the reference's values (exact hex
    doubles printed by the reference build, tests/golden/cos_table.json)."""
    import json
    ref = json.load(open(f"{O.GOLDEN}/cos_table.json"))[str(n)]
    codec.set_quant(O.read_matrix(matrix, n), n)
    got = codec.cos_table().ravel()
    exp = np.array([float.fromhex(x) for x in ref])
    assert np.array_equal(got.view(np.uint64), exp.view(np.uint64)), \
        [(i, got[i].hex(), exp[i].hex()) for i in np.nonzero(got != exp)[0][:4]]


@pytest.mark.parametrize("mode", [MODE_FAST, MODE_EXACT], ids=["fast", "exact"])
@pytest.mark.parametrize("n,matrix", [(4, "matrix.txt"), (8, "matrix8_1.txt")])
@pytest.mark.parametrize("kind", ["ex0", "ex1", "ex2", "ex3", "ex4", "ex6", "U", "M"])
def test_quantized_coefficients(codec, oracle, kind, n, matrix, mode):
    """Block::processDCTDivQ alone: every quantised coefficient vs the oracle (the reference's
    example images ex0-ex4 and ex6, README.md:175-183, and seeded synthetic frames)."""
    if kind.startswith("ex"):
        raw = open(f"{O.GOLDEN}/{kind}.raw", "rb").read()
        w, h = EX_DIMS[kind]
        y = np.frombuffer(raw, dtype=np.uint8).reshape(h, w)
    else:
        y = synth.frame(kind, 320, 240, seed=5)
    q = O.read_matrix(matrix, n)
    codec.set_quant(q, n)
    got = codec.quantize_frames(y, y.shape[1], y.shape[0], mode=mode)
    exp = oracle.quantize(y, n, q)
    bad = np.argwhere(got != exp)
    assert bad.size == 0, (bad[:8].tolist(), got[tuple(bad[0])], exp[tuple(bad[0])])


@pytest.mark.parametrize("mode", [MODE_FAST, MODE_EXACT], ids=["fast", "exact"])
@pytest.mark.parametrize("case", _golden(), ids=lambda c: c["name"])
def test_golden_small(codec, oracle, case, mode):
    enc = _gpu_file(codec, oracle, case, O.case_input(case), mode)
    exp = O.case_expected(case)
    if exp is not None:
        assert enc == exp
    assert len(enc) == case["size"] and _md5(enc) == case["md5"]


@pytest.mark.parametrize("case", _golden(big=True), ids=lambda c: c["name"])
def test_golden_fullsize(codec, oracle, case):
    enc = _gpu_file(codec, oracle, case, O.case_input(case), MODE_FAST)
    assert len(enc) == case["size"] and _md5(enc) == case["md5"]


@pytest.mark.parametrize("n,matrix", [(4, "matrix.txt"), (8, "matrix8_1.txt"), (4, "matrix4_2.txt"),
                                      (8, "matrix8_2.txt")])
@pytest.mark.parametrize("start_bit", [0, 1, 31, 165, 549])
def test_random_frames_vs_oracle(codec, oracle, n, matrix, start_bit):
    """Seeded random sizes (ragged widths included), several frames concatenated, arbitrary
    start bits, RLE on and off -- GPU vs oracle, bit for bit."""
    rng = np.random.default_rng(1234 + n * 100 + start_bit)
    q = O.read_matrix(matrix, n)
    codec.set_quant(q, n)
    for trial in range(3):
        w = n * int(rng.integers(1, 90))
        h = n * int(rng.integers(1, 40))
        f = int(rng.integers(1, 4))
        rle = bool(trial % 2 == 0)
        kind = "U" if trial % 3 else "M"
        y = synth.frames(kind, w, h, f, seed=int(rng.integers(1 << 30)))
        from imageencoder_amd import stream_bound
        out = np.zeros(stream_bound(w, h, n, f, start_bit), dtype=np.uint8)
        fb, end = codec.encode_frames(y, w, h, out, start_bit=start_bit, nframes=f, rle=rle)
        exp, eend, efb = oracle.encode_blocks(y, n, q, rle, start_bit)
        assert end == eend and np.array_equal(fb, efb)
        nb = (end + 7) // 8
        assert out[:nb].tobytes() == exp[:nb].tobytes()


def test_device_pointers_and_images_batch(codec, oracle):
    """Device-resident input/output (torch tensors) and the independent-image batch mode."""
    import torch
    from imageencoder_amd import stream_bound
    n, q = 4, O.read_matrix("matrix.txt", 4)
    codec.set_quant(q, n)
    w, h, f, sb = 640, 360, 6, 165
    y = synth.frames("M", w, h, f, seed=77)
    dy = torch.from_numpy(y).cuda()
    pitch = (stream_bound(w, h, n, 1, sb) + 255) // 256 * 256
    dout = torch.zeros(pitch * f, dtype=torch.uint8, device="cuda")
    ends = codec.encode_images(dy, w, h, dout, out_pitch=pitch, nframes=f, start_bit=sb)
    host = dout.cpu().numpy()
    for i in range(f):
        exp, eend, _ = oracle.encode_blocks(y[i], n, q, True, sb)
        assert int(ends[i]) == eend
        nb = (eend + 7) // 8
        seg = host[i * pitch: i * pitch + nb]
        assert seg[sb // 8 + 1:].tobytes() == exp[sb // 8 + 1: nb].tobytes()
    # concatenated stream, device in / device out
    dcat = torch.zeros(stream_bound(w, h, n, f, sb), dtype=torch.uint8, device="cuda")
    fb, end = codec.encode_frames(dy, w, h, dcat, start_bit=sb, nframes=f)
    exp, eend, efb = oracle.encode_blocks(y, n, q, True, sb)
    assert end == eend and np.array_equal(fb, efb)
    nb = (end + 7) // 8
    assert dcat.cpu().numpy()[sb // 8 + 1: nb].tobytes() == exp[sb // 8 + 1: nb].tobytes()


@pytest.mark.parametrize("n,matrix", [(4, "matrix.txt"), (8, "matrix8_1.txt")])
def test_fast_equals_exact_large(codec, n, matrix):
    """FAST (FP32 + FP64 near-tie re-evaluation) must equal EXACT (all FP64) bit for bit on
    many blocks: 8 distinct 1080p frames of each generator (>= 1M 4x4 blocks)."""
    import torch
    from imageencoder_amd import stream_bound
    q = O.read_matrix(matrix, n)
    codec.set_quant(q, n)
    w, h, f = 1920, 1080, 8
    for kind in ("U", "M"):
        y = torch.from_numpy(synth.frames(kind, w, h, f, seed=4242)).cuda()
        a = torch.zeros(stream_bound(w, h, n, f), dtype=torch.uint8, device="cuda")
        b = torch.zeros_like(a)
        fa, ea = codec.encode_frames(y, w, h, a, nframes=f, mode=MODE_FAST)
        fb, eb = codec.encode_frames(y, w, h, b, nframes=f, mode=MODE_EXACT)
        assert ea == eb and np.array_equal(fa, fb)
        assert torch.equal(a[: (ea + 7) // 8], b[: (eb + 7) // 8])


def test_chain_prefix_beyond_2_31_bits(codec):
    """One concatenated launch whose tiles sit more than 2^31 and 2^32 bits into the stream: 96
    4K noise frames (~5.4e9 bits) in ONE ie_encode_frames launch == the same frames in four
    launches of 24 chained by start_bit (each chain's own prefix below 2^31 bits).  A tile's
    64-bit position once passed through a sign-extending 32-bit half (readfirstlane returns int):
    a prefix of 2^31 bits or more turned into an address past the device's aperture."""
    import torch
    from imageencoder_amd import stream_bound
    q = O.read_matrix("matrix.txt", 4)
    codec.set_quant(q, 4)
    w, h, f, k = 3840, 2160, 96, 24
    y = synth.uniform_device(w, h, f, synth.DEFAULT_SEED + 31, "cuda", torch)
    cap = stream_bound(w, h, 4, f, 165)
    a = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    fa, ea = codec.encode_frames(y, w, h, a, start_bit=165, nframes=f)
    assert ea > (1 << 32)
    b = torch.zeros_like(a)
    e, fb = 165, []
    for i in range(0, f, k):
        fi, ei = codec.encode_frames(y[i:i + k], w, h, b, start_bit=e, nframes=k)
        assert ei - e < (1 << 31)
        fb.append(fi)
        e = ei
    assert ea == e and np.array_equal(fa, np.concatenate(fb))
    assert torch.equal(a[: (ea + 7) // 8], b[: (e + 7) // 8])


def test_random_noise_stress(codec, oracle):
    """Uniform random bytes from numpy's generator (not the splitmix frames) against the oracle."""
    from imageencoder_amd import stream_bound
    rng = np.random.default_rng(99)
    for n, matrix in ((4, "matrix.txt"), (8, "matrix8_1.txt")):
        q = O.read_matrix(matrix, n)
        codec.set_quant(q, n)
        y = rng.integers(0, 256, size=(4, 512, 768), dtype=np.uint8)
        out = np.zeros(stream_bound(768, 512, n, 4), dtype=np.uint8)
        fb, end = codec.encode_frames(y, 768, 512, out, nframes=4)
        exp, eend, efb = oracle.encode_blocks(y, n, q, True, 0)
        assert end == eend and np.array_equal(fb, efb)
        assert out[: (end + 7) // 8].tobytes() == exp[: (end + 7) // 8].tobytes()


@pytest.mark.parametrize("n", [4, 8])
@pytest.mark.parametrize("qfill", [1, 3, 255])
def test_extreme_matrices_fill_the_tile_image(codec, oracle, n, qfill):
    """The LDS tile image is sized per matrix (the largest record any block can produce):
    all-ones / small / large constant matrices with extreme 0/255 pixels (the widest records) and
    with flat frames (the narrowest), RLE on and off, GPU vs oracle bit for bit."""
    from imageencoder_amd import stream_bound
    rng = np.random.default_rng(7 + qfill)
    q = np.full(n * n, qfill, dtype=np.uint16)
    codec.set_quant(q, n)
    w, h = 64 * n, 24 * n
    frames = [
        (rng.integers(0, 2, size=(h, w)) * 255).astype(np.uint8),           # 0/255 noise
        np.indices((h, w)).sum(axis=0).astype(np.uint8) % 2 * 255,            # checkerboard
        np.full((h, w), 128, dtype=np.uint8),                                  # all-zero blocks
    ]
    for rle in (True, False):
        for y in frames:
            y = np.ascontiguousarray(y, dtype=np.uint8)
            out = np.zeros(stream_bound(w, h, n, 1, 5), dtype=np.uint8)
            fb, end = codec.encode_frames(y, w, h, out, start_bit=5, rle=rle)
            exp, eend, efb = oracle.encode_blocks(y, n, q, rle, 5)
            assert end == eend and np.array_equal(fb, efb)
            nb = (end + 7) // 8
            assert out[:nb].tobytes() == exp[:nb].tobytes()


@pytest.mark.parametrize("w,h,f", [(3840, 2160, 1), (200, 56, 3), (1928, 1080, 2), (4, 4, 1)])
def test_small_launch_lookback_matches_batch_path(w, h, f, tmp_path):
    """Launches whose tiles would not fill the chip issue their look-back windows at once; the
    stream must be the one the batch path (IE_SMALL_TILES=0, fresh processes) writes -- ragged
    widths, several frames, concatenated and segmented output."""
    import subprocess
    import sys

    code = ("import sys, hashlib, numpy as np; sys.path.insert(0, %r)\n"
            "import torch\n"
            "from imageencoder_amd import Codec, read_matrix, stream_bound, synth\n"
            "from tests import oracle_lib as O\n"
            "w, h, f = %d, %d, %d\n"
            "c = Codec(0, read_matrix(O.GOLDEN + '/matrix.txt', 4), 4)\n"
            "y = torch.from_numpy(synth.frames('M', w, h, f, seed=77)).cuda()\n"
            "out = torch.zeros(stream_bound(w, h, 4, f, 13) + 64, dtype=torch.uint8, device='cuda')\n"
            "_, end = c.encode_frames(y, w, h, out, start_bit=13, nframes=f)\n"
            "pitch = (stream_bound(w, h, 4, 1, 5) + 255) // 256 * 256\n"
            "seg = torch.zeros(pitch * f, dtype=torch.uint8, device='cuda')\n"
            "ends = c.encode_images(y, w, h, seg, out_pitch=pitch, nframes=f, start_bit=5)\n"
            "print(end, hashlib.md5(out[:(end + 7) // 8].cpu().numpy().tobytes()).hexdigest(),\n"
            "      hashlib.md5(seg.cpu().numpy().tobytes()).hexdigest(), list(map(int, ends)))\n") % (O.ROOT, w, h, f)
    outs = []
    for extra in ({"IE_SMALL_TILES": "1024"}, {"IE_SMALL_TILES": "0"}):
        env = dict(os.environ, **extra)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env, cwd=O.ROOT)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(r.stdout.strip().splitlines()[-1])
    assert outs[0] == outs[1]
