"""GPU parity of the whole-file path (libie_host.so over libie_hip.so): settings header, block
records, the Huffman post-pass (device histogram + host tree replay + device re-encode) and the
inverse path (ie_decode_frames), against the reference's golden files and the CPU oracle.
Bit-exact is the bar for every byte and pixel.
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


def _cases(pred):
    return [c for c in O.manifest() if pred(c)]


def _ids(cs):
    return [c["name"] for c in cs]


def _check(c, got: bytes):
    assert len(got) == c["size"], (c["name"], len(got), c["size"])
    exp = O.case_expected(c)
    if exp is not None:
        if got != exp:
            a = np.frombuffer(got, np.uint8)
            b = np.frombuffer(exp, np.uint8)
            i = int(np.nonzero(a != b)[0][0])
            pytest.fail(f"{c['name']}: first differing byte {i}: {a[i]:#04x} != {b[i]:#04x}")
    else:
        assert _md5(got) == c["md5"], c["name"]


def _encode_case(codec, c, mode=MODE_FAST) -> bytes:
    raw = O.case_input(c)
    q = O.read_matrix(c["matrix"], c["n"])
    y = np.frombuffer(raw, dtype=np.uint8)
    if c["video"]:
        return codec.encode_video_file(y, c["w"], c["h"], q, c["n"], rle=bool(c["rle"]), huffman=c["huffman"],
                                       merange=16, mode=mode)
    return codec.encode_image_file(y, c["w"], c["h"], q, c["n"], rle=bool(c["rle"]), huffman=c["huffman"],
                                   mode=mode)


SMALL = _cases(lambda c: c["w"] * c["h"] < 1920 * 1080)
BIG = _cases(lambda c: c["w"] * c["h"] >= 1920 * 1080)


@pytest.mark.parametrize("c", SMALL, ids=_ids(SMALL))
def test_file_golden_small(codec, c):
    """Every small golden file (image + video, Huffman on/off, RLE on/off, 4x4/8x8)."""
    _check(c, _encode_case(codec, c))


@pytest.mark.parametrize("c", BIG, ids=_ids(BIG))
def test_file_golden_full_size(codec, c):
    """4K / 1080p golden files, including the 4K Huffman file (config C5)."""
    _check(c, _encode_case(codec, c))


def test_file_exact_mode_matches(codec):
    c = next(c for c in SMALL if c["name"] == "synU256_8x8_huff")
    _check(c, _encode_case(codec, c, MODE_EXACT))


# ---------------------------------------------------------------------------- Huffman stages
def _byte_sets():
    rng = np.random.default_rng(7)
    yield "uniform", rng.integers(0, 256, 200_003, dtype=np.uint8).tobytes()
    yield "skewed", np.minimum(rng.geometric(0.08, 150_001), 255).astype(np.uint8).tobytes()
    yield "few", rng.choice(np.array([3, 9, 200], np.uint8), 70_001, p=[0.7, 0.2, 0.1]).tobytes()
    yield "two", bytes([5, 6] * 50)
    yield "tiny", bytes([1, 2, 3])
    yield "one_byte", bytes([42])
    yield "fib", b"".join(bytes([i]) * f for i, f in enumerate([1, 1, 2, 3, 5, 8, 13, 21, 34, 55, 89, 144]))
    enc = O.load().encode_blocks(synth.frame("U", 512, 256), 4, O.read_matrix("matrix.txt", 4))[0]
    yield "encoded", enc[:60_000].tobytes()
    # values that first appear past the first-occurrence scan's prefix (64 x 4 KiB): the full pass
    late = rng.integers(0, 200, 1_200_003, dtype=np.uint8)
    for v, at in ((230, 300_000), (201, 700_001), (255, 1_200_002), (210, 262_144), (220, 262_143)):
        late[at] = v
    late[900_000:900_016] = 240
    yield "late_values", late.tobytes()


BYTE_SETS = list(_byte_sets())


@pytest.mark.parametrize("name,data", BYTE_SETS, ids=[n for n, _ in BYTE_SETS])
def test_huffman_hist(codec, name, data):
    hist, first = codec.huffman_hist(np.frombuffer(data, np.uint8).copy())
    eh, ef = O.load().histogram(data)
    assert np.array_equal(hist, eh)
    assert np.array_equal(first, ef)


@pytest.mark.parametrize("name,data", BYTE_SETS, ids=[n for n, _ in BYTE_SETS])
def test_huffman_encode(codec, name, data):
    got = codec.huffman_encode(np.frombuffer(data, np.uint8).copy())
    assert got == O.load().huffman_encode(data)


def test_huffman_encode_device_input(codec):
    torch = pytest.importorskip("torch")
    data = BYTE_SETS[1][1]
    t = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
    assert codec.huffman_encode(t) == O.load().huffman_encode(data)


def test_huffman_encode_batch(codec):
    """One histogram launch + one pack launch over a batch of strings (every byte set above, an
    empty one, a no-gain one) equals the per-string reference Huffman pass; the output pitch
    starts out as garbage (the batch writes every byte it returns, dictionary included)."""
    torch = pytest.importorskip("torch")
    datas = [d for _, d in BYTE_SETS] + [b""]
    pitch = (max(len(d) for d in datas) + 255) // 256 * 256
    src = torch.zeros(pitch * len(datas), dtype=torch.uint8)
    for k, d in enumerate(datas):
        if d:
            src[k * pitch:k * pitch + len(d)] = torch.from_numpy(np.frombuffer(d, np.uint8).copy())
    src = src.cuda()
    opitch = (4 * pitch + 4096 + 255) // 256 * 256
    out = torch.full((opitch * len(datas),), 0xAB, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the codec runs on its own stream
    sizes = codec.huffman_encode_batch(src, pitch, [len(d) for d in datas], out, opitch)
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    oracle = O.load()
    for k, d in enumerate(datas):
        got = host[k * opitch:k * opitch + sizes[k]].tobytes()
        want = oracle.huffman_encode(d) if d else b"\x00"  # empty: the bare stop bit
        assert got == want, (k, len(d))


def test_huffman_no_gain_revert(codec):
    """Uniform bytes do not compress: '0' + the input (Huffman.cpp:329-341), n + 1 bytes."""
    data = BYTE_SETS[0][1]
    got = codec.huffman_encode(np.frombuffer(data, np.uint8).copy())
    assert len(got) == len(data) + 1
    bits = np.unpackbits(np.frombuffer(got, np.uint8))
    assert bits[0] == 0
    assert np.packbits(bits[1:1 + 8 * len(data)]).tobytes() == data


@pytest.mark.parametrize("start_bit", [0, 1, 7, 8, 13, 31, 32, 45])
def test_bitcopy(codec, start_bit):
    rng = np.random.default_rng(start_bit)
    data = rng.integers(0, 256, 9_999, dtype=np.uint8)
    out = np.zeros((start_bit + 8 * data.size) // 8 + 64, np.uint8)
    head = rng.integers(0, 256, (start_bit + 7) // 8, dtype=np.uint8)
    hb = np.unpackbits(head)[:start_bit] if start_bit else np.zeros(0, np.uint8)
    if start_bit:
        out[: head.size] = np.packbits(np.concatenate([hb, np.zeros(head.size * 8 - start_bit, np.uint8)]))
    codec.bitcopy(data, out, start_bit)
    bits = np.unpackbits(out)
    assert np.array_equal(bits[:start_bit], hb)
    assert np.array_equal(bits[start_bit:start_bit + 8 * data.size], np.unpackbits(data))


@pytest.mark.parametrize("start_bit,n,off", [(0, 1, 0), (3, 5, 1), (165, 100_003, 0), (210, 77_777, 3),
                                             (31, 4, 2), (32 * 1000 + 7, 1_000_000, 1)])
def test_bitcopy_device(codec, start_bit, n, off):
    """Device to device (the multi-GPU segment re-shift): arbitrary start bits, input slices that
    are not word-aligned, the caller's bits before start_bit kept, the rest of the last word zero,
    nothing written past it (the output is pre-filled with garbage)."""
    import torch
    rng = np.random.default_rng(start_bit + n)
    data = rng.integers(0, 256, n + off, dtype=np.uint8)
    garbage = rng.integers(0, 256, (start_bit + 8 * n) // 8 + 64, dtype=np.uint8)
    din = torch.from_numpy(data).cuda()[off:]
    dout = torch.from_numpy(garbage).cuda()
    codec.bitcopy(din, dout, start_bit)
    codec.sync()
    bits = np.unpackbits(dout.cpu().numpy())
    g = np.unpackbits(garbage)
    end = start_bit + 8 * n
    wend = (end + 31) // 32 * 32
    assert np.array_equal(bits[:start_bit], g[:start_bit])
    assert np.array_equal(bits[start_bit:end], np.unpackbits(data[off:]))
    assert not bits[end:wend].any()
    assert np.array_equal(bits[wend:], g[wend:])


def test_huffman_pack_codes(codec):
    """Variable-length codes up to 32 bits land MSB-first at arbitrary start bits."""
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, 30_011, dtype=np.uint8)
    length = rng.integers(0, 33, 256).astype(np.uint8)
    code = np.array([int(rng.integers(0, 1 << int(l))) if l else 0 for l in length], np.uint64).astype(np.uint32)
    for start in (0, 5, 77):
        out = np.zeros(start // 8 + 4 * data.size + 64, np.uint8)
        end = codec.huffman_pack(data, code, length, out, start)
        ref = []
        for b in data:
            l = int(length[b])
            ref.extend((int(code[b]) >> (l - 1 - k)) & 1 for k in range(l))
        assert end == start + len(ref)
        bits = np.unpackbits(out)
        assert np.array_equal(bits[start:end], np.array(ref, np.uint8))
        assert not bits[:start].any()


# ---------------------------------------------------------------------------------- decoder
DEC = _cases(lambda c: c.get("decode") and not c["video"])


@pytest.mark.parametrize("c", DEC, ids=_ids(DEC))
def test_decode_golden(codec, c):
    """ImageDecoder parity: the reference decoder's pixels from the reference's own file."""
    enc = O.case_expected(c)
    if enc is None:
        enc = _encode_case(codec, c)
        assert _md5(enc) == c["md5"]
    pix = codec.decode_image_file(enc, c["n"])
    assert pix.shape == (c["h"], c["w"])
    assert _md5(pix.tobytes()) == c["dec_md5"], c["name"]


@pytest.mark.parametrize("n,gen", [(4, "U"), (8, "U"), (4, "M"), (8, "M")])
@pytest.mark.parametrize("rle", [True, False])
def test_decode_random_vs_oracle(codec, n, gen, rle):
    y = synth.frame(gen, 328, 176, seed=1234 + n)
    q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
    enc = codec.encode_image_file(y, 328, 176, q, n, rle=rle, huffman=False)
    assert enc == O.load().encode_image(y, n, q, rle=rle)
    pix = codec.decode_image_file(enc, n)
    assert np.array_equal(pix, O.load().decode_image(enc, n))


def test_decode_4k_roundtrip(codec):
    """Full-size inverse path against the pinned reference decode (md5 of synM4k)."""
    c = next(c for c in O.manifest() if c["name"] == "synM4k_4x4")
    enc = _encode_case(codec, c)
    assert _md5(enc) == c["md5"]
    pix = codec.decode_image_file(enc, 4)
    assert _md5(pix.tobytes()) == c["dec_md5"]


def test_decode_video_gop1(codec):
    c = next(c for c in O.manifest() if c["name"] == "vidM64x48x5_4x4_huff")
    enc = _encode_case(codec, c)
    _check(c, enc)
    out, (w, h, f) = codec.decode_video_file(enc, 4)
    assert (w, h, f) == (64, 48, 5)
    frames = out.reshape(f, h * w * 3 // 2)
    assert (frames[:, w * h:] == 0x80).all()
    yuv = np.frombuffer(O.case_input(c), np.uint8).reshape(f, -1)
    q = O.read_matrix("matrix.txt", 4)
    for k in range(f):
        one = O.load().encode_image(yuv[k, : w * h].reshape(h, w).copy(), 4, q)
        assert np.array_equal(frames[k, : w * h].reshape(h, w), O.load().decode_image(one, 4))


# ---------------------------------------------------------------------------- Huffman decode
HUFF = _cases(lambda c: c["huffman"])


@pytest.mark.parametrize("c", HUFF, ids=_ids(HUFF))
def test_huffman_decode_golden(codec, c):
    """Huffman<uint8_t>::decode on the device against the oracle's per-bit tree walk, on the
    reference's own Huffman-coded files (every byte, the padding symbols included)."""
    enc = O.case_expected(c)
    if enc is None:
        enc = _encode_case(codec, c)
    exp = O.load().huffman_decode(enc)
    assert exp is not None
    assert codec.huffman_decode(enc) == exp


def _huff_inputs():
    rng = np.random.default_rng(5)
    skew = rng.geometric(0.2, size=20000).clip(1, 255).astype(np.uint8)  # long codes (<= 15 bits)
    overlong = rng.geometric(0.3, size=50000).clip(1, 255).astype(np.uint8)  # a code > 15 bits
    return {
        "two_bytes": b"\x07\x08",
        "two_symbols": bytes(rng.integers(0, 2, size=3001, dtype=np.uint8) * 0xFF),
        "uniform": rng.integers(0, 256, size=20000, dtype=np.uint8).tobytes(),
        "skewed": skew.tobytes(),
        "overlong": overlong.tobytes(),
        "text": (b"the quick brown fox jumps over the lazy dog " * 300),
        "4k_payload": synth.frame("U", 512, 64, seed=3).tobytes(),
    }


@pytest.mark.parametrize("name", list(_huff_inputs()))
def test_huffman_roundtrip_vs_oracle(codec, name):
    """encode (device) -> decode (device): the reference's decode output, byte for byte (the input
    followed by whatever the padding bits of the last byte decode to), or the passthrough.
    (A single distinct byte value gets a 0-bit code, for which the reference's treeAddLeaf is
    undefined -- Huffman.cpp:155-172 shifts by len - 1 -- so that input is not a parity case.)"""
    data = _huff_inputs()[name]
    enc = codec.huffman_encode(np.frombuffer(data, np.uint8).copy())
    exp = O.load().huffman_decode(enc)
    if exp is None:
        # a code longer than 15 bits: the dictionary keeps 4 length bits (Huffman.cpp:41-42), so
        # the reference's own file does not decode; neither does ours
        from imageencoder_amd import IEError
        assert name == "overlong"
        with pytest.raises(IEError):
            codec.huffman_decode(enc)
        return
    got = codec.huffman_decode(enc)
    assert got == exp
    dec, passthrough = got
    if not passthrough:
        assert dec[: len(data)] == data


def test_huffman_decode_rejects_invalid(codec):
    """A bit string no code prefixes fails with IE_EFORMAT (the reference would follow a null
    child).  Dictionary: one block of two 2-bit codes, 00 -> 0x01 and 01 -> 0x02, so prefix 1x is
    no code; eight 00 symbols, then a 1."""
    from imageencoder_amd import IEError
    bw = "1" + format(2, "07b") + format(2, "04b") + format(1, "08b") + "00" + format(2, "08b") + "01" + "0"
    bw += "00" * 8 + "1"
    bw += "0" * (-len(bw) % 8)
    crafted = int(bw, 2).to_bytes(len(bw) // 8, "big")
    assert O.load().huffman_decode(crafted) is None
    with pytest.raises(IEError):
        codec.huffman_decode(crafted)


def test_huffman_after_encode_pipeline(codec):
    """encode_images -> Huffman pass with the lengths taken from the encoder's end bits on the
    device (the C5 pipeline): every image's Huffman-coded file equals the reference's."""
    import torch
    from imageencoder_amd import stream_bound, write_header
    n, q, w, h, f = 4, O.read_matrix("matrix.txt", 4), 320, 192, 5
    codec.set_quant(q, n)
    hdr, hb = write_header(n, q, True, w, h, huffman=True)
    pitch = (stream_bound(w, h, n, 1, hb) + 255) // 256 * 256
    y = synth.frames("M", w, h, f, seed=31)
    out = torch.zeros(pitch * f, dtype=torch.uint8)
    for k in range(f):  # each image's settings header, then the records from bit hb
        out[k * pitch: k * pitch + len(hdr)] = torch.from_numpy(np.frombuffer(hdr, np.uint8).copy())
    out = out.cuda()
    hpitch = 2 * pitch
    hout = torch.zeros(hpitch * f, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    codec.encode_images(torch.from_numpy(y).cuda(), w, h, out, out_pitch=pitch, nframes=f, start_bit=hb,
                        want_sizes=False)
    sizes = codec.huffman_encode_after_encode(out, pitch, f, hout, hpitch)
    torch.cuda.synchronize()
    host = hout.cpu().numpy()
    for k in range(f):
        want = O.load().encode_image(y[k], n, q, rle=True, huffman=True)
        assert host[k * hpitch: k * hpitch + sizes[k]].tobytes() == want, k


def _late_frames(w, h, f, seed):
    """Flat frames whose last 32 rows are noise: their streams' byte values other than the flat
    records' first appear past the first-occurrence scan's prefix (64 chunks of 4 KiB), so the
    counted pipeline takes its full-pass fallback."""
    rng = np.random.default_rng(seed)
    y = np.full((f, h, w), 77, dtype=np.uint8)
    y[:, h - 32:, :] = rng.integers(0, 256, (f, 32, w), dtype=np.uint8)
    return y


@pytest.mark.gpu
@pytest.mark.parametrize("counted,late", [(False, False), (True, False), (True, True)],
                         ids=["hist_pass", "counted_encode", "counted_late_values"])
def test_huffman_after_encode_pipelined(codec, counted, late):
    """Batches pipelined as in bench.py's C5 step: batch i+1's encode and histogram are issued
    before batch i's trees + pack (two output buffers, histogram slots alternating); every
    image's Huffman-coded file still equals the reference's.  counted: the byte counts come from
    the encoder itself (ie_encode_images_counted).  late: values first seen past the scanned
    prefix (the full first-occurrence pass, run from ie_huffman_hist_batch_wait)."""
    import torch
    from imageencoder_amd import stream_bound, write_header
    n, q, w, h, f, nb = 4, O.read_matrix("matrix.txt", 4), 256, 128, 3, 4
    if late:
        w, h, f, nb = 2048, 2048, 2, 3
    codec.set_quant(q, n)
    hdr, hb = write_header(n, q, True, w, h, huffman=True)
    pitch = (stream_bound(w, h, n, 1, hb) + 255) // 256 * 256
    ys = [_late_frames(w, h, f, 50 + b) if late else synth.frames("M" if b % 2 else "U", w, h, f, seed=50 + b)
          for b in range(nb)]
    outs = []
    for _ in range(2):
        o = torch.zeros(pitch * f, dtype=torch.uint8)
        for k in range(f):
            o[k * pitch: k * pitch + len(hdr)] = torch.from_numpy(np.frombuffer(hdr, np.uint8).copy())
        outs.append(o.cuda())
    hpitch = 2 * pitch
    houts = [torch.zeros(hpitch * f, dtype=torch.uint8, device="cuda") for _ in range(nb)]
    sizes = [None] * nb
    torch.cuda.synchronize()
    pending = None
    for b in range(nb):
        codec.encode_images(torch.from_numpy(ys[b]).cuda(), w, h, outs[b % 2], out_pitch=pitch, nframes=f,
                            start_bit=hb, want_sizes=False, count_bytes=counted)
        codec.huffman_begin_after_encode(outs[b % 2], pitch, f, b % 2)
        if pending is not None:
            p = pending
            sizes[p] = codec.huffman_finish_after_encode(outs[p % 2], pitch, f, p % 2, houts[p], hpitch)
        pending = b
    sizes[pending] = codec.huffman_finish_after_encode(outs[pending % 2], pitch, f, pending % 2, houts[pending],
                                                       hpitch)
    codec.sync()
    torch.cuda.synchronize()
    for b in range(nb):
        host = houts[b].cpu().numpy()
        for k in range(f):
            want = O.load().encode_image(ys[b][k], n, q, rle=True, huffman=True)
            assert host[k * hpitch: k * hpitch + sizes[b][k]].tobytes() == want, (b, k)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,f,start_bit,kind", [
    (320, 192, 3, 165, "M"),     # a settings header ending inside a word
    (200, 56, 4, 0, "U"),        # no header; ragged tile coverage
    (1000, 600, 3, 64, "U"),     # multi-tile chains, header of whole words
    (3840, 2160, 2, 171, "M"),   # 4K: hundreds of tiles per chain
    (2048, 2048, 2, 165, "late"),  # values first seen past the scanned prefix: the full pass
])
def test_counted_encode_histogram(codec, w, h, f, start_bit, kind):
    """ie_encode_images_counted's fused byte counts equal the separate histogram pass's and a
    host bincount of each stream's bytes [0, ceil(end / 8)) -- header words included, the last
    word's padding bytes excluded; the first positions match too."""
    import torch
    from imageencoder_amd import stream_bound
    n, q = 4, O.read_matrix("matrix.txt", 4)
    codec.set_quant(q, n)
    pitch = (stream_bound(w, h, n, 1, start_bit) + 255) // 256 * 256
    y = torch.from_numpy(_late_frames(w, h, f, 77) if kind == "late" else synth.frames(kind, w, h, f, seed=77)).cuda()
    rng = np.random.default_rng(5)
    out = torch.zeros(pitch * f, dtype=torch.uint8)
    nh = (start_bit + 7) // 8
    for k in range(f):  # header bytes (random), bits from start_bit on left zero
        hdr = rng.integers(0, 256, nh, dtype=np.uint8)
        if start_bit % 8:
            hdr[-1] &= np.uint8((0xFF00 >> (start_bit % 8)) & 0xFF)
        out[k * pitch: k * pitch + nh] = torch.from_numpy(hdr)
    out = out.cuda()
    codec.encode_images(y, w, h, out, out_pitch=pitch, nframes=f, start_bit=start_bit, count_bytes=True)
    h_fused, f_fused = codec.huffman_hist_after_encode(out, pitch, f)
    ends = codec.encode_images(y, w, h, out, out_pitch=pitch, nframes=f, start_bit=start_bit)
    h_pass, f_pass = codec.huffman_hist_after_encode(out, pitch, f)
    host = out.cpu().numpy()
    for k in range(f):
        nb = (int(ends[k]) + 7) // 8
        want = np.bincount(host[k * pitch: k * pitch + nb], minlength=256).astype(np.uint32)
        np.testing.assert_array_equal(h_pass[k], want)
        np.testing.assert_array_equal(h_fused[k], want)
    np.testing.assert_array_equal(f_fused, f_pass)
    if kind == "late":  # the case exercises the full pass: some value first seen past 64 chunks of 4 KiB
        assert int(f_pass[f_pass != np.uint64(2**64 - 1)].max()) >= 64 * 4096


@pytest.mark.gpu
def test_counted_encode_histogram_batch_sizes(codec):
    """The counted encoder's histogram rows across batches of different sizes: a
    counted batch of 8 that no fused pass reads, a batch of 4 that one does (clearing rows 0-3
    only), then a batch of 8 again -- its rows 4-7 must not keep the first batch's counts.  Every
    fused histogram equals a host bincount of the stream bytes."""
    import torch
    from imageencoder_amd import stream_bound
    n, q = 4, O.read_matrix("matrix.txt", 4)
    codec.set_quant(q, n)
    w, h = 256, 128
    pitch = (stream_bound(w, h, n, 1, 0) + 255) // 256 * 256
    out = torch.zeros(pitch * 8, dtype=torch.uint8, device="cuda")

    def check(f, seed, read):
        y = torch.from_numpy(synth.frames("M", w, h, f, seed=seed)).cuda()
        out.zero_()
        codec.encode_images(y, w, h, out, out_pitch=pitch, nframes=f, count_bytes=True)
        if not read:
            return
        hist, _ = codec.huffman_hist_after_encode(out, pitch, f)
        ends = codec.encode_images(y, w, h, out, out_pitch=pitch, nframes=f)
        host = out.cpu().numpy()
        for k in range(f):
            nb = (int(ends[k]) + 7) // 8
            want = np.bincount(host[k * pitch: k * pitch + nb], minlength=256).astype(np.uint32)
            np.testing.assert_array_equal(hist[k], want, err_msg=f"batch of {f}, image {k}")

    check(8, 1, read=False)
    check(4, 2, read=True)
    check(8, 3, read=True)
    check(8, 4, read=True)


@pytest.mark.gpu
def test_stage_timing_opt_in(codec):
    """ie_last_stage_ms reports the batched Huffman stages only while ie_set_stage_timing is on
    (off by default: the events idle the pipelined step); the outputs do not depend on it."""
    import torch
    from imageencoder_amd import IEError, stream_bound, write_header
    n, q, w, h, f = 4, O.read_matrix("matrix.txt", 4), 256, 128, 3
    codec.set_quant(q, n)
    hdr, hb = write_header(n, q, True, w, h, huffman=True)
    pitch = (stream_bound(w, h, n, 1, hb) + 255) // 256 * 256
    y = torch.from_numpy(synth.frames("U", w, h, f, seed=9)).cuda()
    out = torch.zeros(pitch * f, dtype=torch.uint8, device="cuda")
    hout = torch.zeros(2 * pitch * f, dtype=torch.uint8, device="cuda")
    results = []
    for on in (False, True):
        codec.set_stage_timing(on)
        codec.encode_images(y, w, h, out, out_pitch=pitch, nframes=f, start_bit=hb, want_sizes=False)
        codec.huffman_begin_after_encode(out, pitch, f, 0)  # (the batched calls that record the events)
        sizes = codec.huffman_finish_after_encode(out, pitch, f, 0, hout, 2 * pitch)
        codec.sync()
        torch.cuda.synchronize()
        results.append((sizes, hout.clone()))
        if on:
            assert codec.last_stage_ms(0) > 0.0 and codec.last_stage_ms(1) > 0.0
        else:
            with pytest.raises(IEError):
                codec.last_stage_ms(1)
    codec.set_stage_timing(False)
    assert results[0][0] == results[1][0] and torch.equal(results[0][1], results[1][1])


# ------------------------------------------------- multi-segment decode; one-launch path (opt-in)
@pytest.mark.parametrize("huffman", [False, True])
@pytest.mark.parametrize("n", [4, 8])
@pytest.mark.parametrize("kind", ["flat", "U", "M", "grad"])
def test_decode_multi_segment_vs_oracle(codec, n, kind, huffman):
    """Streams spanning many parse segments (4x4: 65536 bits, 8x8: 131072 bits each), with
    records from 5 bits (flat blocks) to the longest, and periodic record streams (flat image,
    regular gradient), with and without the Huffman pass (a periodic record stream makes a periodic
    code stream too): the decode == the oracle's."""
    w, h = 648, 488
    if kind == "flat":
        y = np.full((h, w), 77, dtype=np.uint8)
    elif kind == "grad":
        yy, xx = np.mgrid[0:h, 0:w]
        y = ((xx * 3 + yy * 5) % 256).astype(np.uint8)
    else:
        y = synth.frame(kind, w, h, seed=99 + n)
    q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
    enc = codec.encode_image_file(y, w, h, q, n, rle=True, huffman=huffman)
    pix = codec.decode_image_file(enc, n)
    assert np.array_equal(pix, O.load().decode_image(enc, n))


@pytest.mark.parametrize("spec", ["0", "1"])
@pytest.mark.parametrize("recs", ["1", "7", "200"])
@pytest.mark.parametrize("name", ["synM4k_4x4", "synU4k_4x4", "synM4k_8x8"])
def test_decode_chunking_matches(codec, tmp_path, name, recs, spec):
    """The exact parse (IE_DEC_SPEC=0) and the speculative one give the reference decoder's pixels
    for any chunking (IE_DEC_R records per chunk: 1 = many groups and the cross-group chase from
    global memory, 200 = long chunks), in a fresh process."""
    import subprocess
    import sys
    c = next((c for c in O.manifest() if c["name"] == name), None)
    if c is None:
        pytest.skip(name + " not in the manifest")
    enc = _encode_case(codec, c)
    default = codec.decode_image_file(enc, c["n"])
    (tmp_path / "s.enc").write_bytes(enc)
    code = ("import sys, hashlib; sys.path.insert(0, %r)\n"
            "from imageencoder_amd import Codec\n"
            "c = Codec(0)\n"
            "pix = c.decode_image_file(open(%r, 'rb').read(), %d)\n"
            "print(hashlib.md5(pix.tobytes()).hexdigest(), *c.last_decode_info())\n") % (
        O.ROOT, str(tmp_path / "s.enc"), c["n"])
    env = dict(os.environ, IE_DEC_R=recs, IE_DEC_SPEC=spec)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env,
                       cwd=O.ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    md5, chunks, groups = r.stdout.strip().splitlines()[-1].split()
    assert int(chunks) >= 1 and (int(groups) >= 1 or spec == "1")
    assert md5 == _md5(default.tobytes())
    if "dec_md5" in c:
        assert md5 == c["dec_md5"]


@pytest.mark.parametrize("n", [4, 8])
def test_decode_truncated_stream_fails(codec, n):
    """A payload cut short holds fewer records than the header's frame needs: the decode fails with
    IE_EFORMAT ("stream ends before the last block") instead of returning pixels."""
    from imageencoder_amd import IEError
    w, h = 256, 128
    y = synth.frame("U", w, h, seed=5)
    q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
    enc = codec.encode_image_file(y, w, h, q, n, rle=True, huffman=False)
    assert np.array_equal(codec.decode_image_file(enc, n), O.load().decode_image(enc, n))
    with pytest.raises(IEError):
        codec.decode_image_file(enc[: len(enc) * 9 // 10], n)
    # the context stays usable
    assert np.array_equal(codec.decode_image_file(enc, n), O.load().decode_image(enc, n))


@pytest.mark.parametrize("n", [4, 8])
@pytest.mark.parametrize("k", [0, 1, 2, 3])
def test_decode_device_stream_in_place(codec, n, k):
    """An aligned device stream is parsed in place: bytes past its length in the last word (here
    0xFF) are cleared by the kernels, so the pixels and end bit equal those of the staged copy
    (host bytes) and of an unaligned device view (staged on the device)."""
    import torch

    from imageencoder_amd import Codec, stream_bound
    w, h = 264, 136
    y = synth.frame("M", w, h, seed=11 + n)
    c = Codec(0, O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n), n)
    dev = torch.zeros(stream_bound(w, h, n, 1, 0) + 64, dtype=torch.uint8, device="cuda")
    _, end = c.encode_frames(torch.from_numpy(y).cuda(), w, h, dev)
    length = (end + 7) // 8 + k
    dev[length:length + 16] = 0xFF
    host = dev[:length].cpu().numpy().copy()
    pix_h = torch.zeros((h, w), dtype=torch.uint8, device="cuda")
    pix_d = torch.zeros_like(pix_h)
    pix_u = torch.zeros_like(pix_h)
    e_h = c.decode_frames(host, w, h, pix_h, length=length)
    e_d = c.decode_frames(dev, w, h, pix_d, length=length)
    assert e_h == e_d == end
    assert torch.equal(pix_h, pix_d)
    # device views at every offset of a 16-byte line: only 16-byte aligned ones are read in place
    for off in (1, 4, 8, 12, 16):
        shifted = torch.full((length + 33,), 0xFF, dtype=torch.uint8, device="cuda")
        shifted[off:length + off] = dev[:length]
        pix_u.zero_()
        e_u = c.decode_frames(shifted[off:], w, h, pix_u, length=length)
        assert e_u == end, off
        assert torch.equal(pix_h, pix_u), off


@pytest.mark.parametrize("n", [4, 8])
@pytest.mark.parametrize("kind", ["U", "M", "grad", "flat", "flat_noise"])
def test_decode_speculative_equals_exact(codec, n, kind):
    """The optional speculative record parse (each chunk entered where its predecessor's walk from
    its first bit left it, every exit verified by the counting walks) and the exact parse over
    composed transfer tables decode the same pixels and end bit, both == the oracle; where a
    speculative entry is wrong (periodic content) the call hands over to the exact parse."""
    import torch

    from imageencoder_amd import Codec, stream_bound
    w, h = 1032, 520
    if kind == "flat":
        y = np.full((h, w), 77, dtype=np.uint8)
    elif kind == "flat_noise":  # flat halves around a noise band: both kinds of chunks in one stream
        y = np.full((h, w), 200, dtype=np.uint8)
        y[h // 3: h // 2] = synth.frame("U", w, h // 2 - h // 3, seed=5)
    elif kind == "grad":
        yy, xx = np.mgrid[0:h, 0:w]
        y = ((xx * 3 + yy * 5) % 256).astype(np.uint8)
    else:
        y = synth.frame(kind, w, h, seed=21 + n)
    q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
    c = Codec(0, q, n)
    dev = torch.zeros(stream_bound(w, h, n, 1, 0) + 64, dtype=torch.uint8, device="cuda")
    _, end = c.encode_frames(torch.from_numpy(y).cuda(), w, h, dev)
    length = (end + 7) // 8
    pix_s = torch.zeros((h, w), dtype=torch.uint8, device="cuda")
    pix_e = torch.zeros_like(pix_s)
    c.set_exact_parse(False)
    e_s = c.decode_frames(dev, w, h, pix_s, length=length)
    used_spec = c.last_decode_spec()
    c.set_exact_parse(True)
    e_e = c.decode_frames(dev, w, h, pix_e, length=length)
    assert not c.last_decode_spec()
    assert e_s == e_e == end
    assert torch.equal(pix_s, pix_e)
    ref = O.load().decode_image(O.load().encode_image(y, n, q, rle=True), n)
    assert np.array_equal(pix_s.cpu().numpy(), np.asarray(ref).reshape(h, w))
    if kind == "flat":  # measured: the flat frames' speculative walks meet the true path
        assert used_spec


@pytest.mark.parametrize("n", [4, 8])
@pytest.mark.parametrize("warm", [1, 8])
def test_decode_speculative_warm(codec, n, warm):
    """Speculative parse with warm-up chunks (ie_set_spec_warm(ctx, warm)): noise frames make
    the longest chunks (8x8: C = 8192 bits), where warm = 8 would exceed the count pass's LDS
    unless the host clamps it; the pixels equal the exact parse's either way."""
    import torch

    from imageencoder_amd import Codec, stream_bound
    w, h = 1024, 256
    y = synth.frame("U", w, h, seed=31 + n)
    q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
    c = Codec(0, q, n)
    dev = torch.zeros(stream_bound(w, h, n, 1, 0) + 64, dtype=torch.uint8, device="cuda")
    _, end = c.encode_frames(torch.from_numpy(y).cuda(), w, h, dev)
    length = (end + 7) // 8
    pix_s = torch.zeros((h, w), dtype=torch.uint8, device="cuda")
    pix_e = torch.zeros_like(pix_s)
    c.set_exact_parse(False, warm=warm)
    e_s = c.decode_frames(dev, w, h, pix_s, length=length)
    c.set_exact_parse(True)
    e_e = c.decode_frames(dev, w, h, pix_e, length=length)
    assert e_s == e_e == end
    assert torch.equal(pix_s, pix_e)


@pytest.mark.gpu
@pytest.mark.parametrize("short", [0, 1, 777])
def test_huffman_decode_device_output(codec, short):
    """ie_huffman_decode with device stream, table and output (one read-back: the emit runs before
    the symbol count is known and is bounded by the output's size): the symbols (the walk runs to
    the buffer's end, the last byte's padding bits included, as the reference's does); an output
    `short` bytes below the count raises IE_ECAP and leaves the bytes past it untouched."""
    import torch
    from imageencoder_amd import IE_ECAP, IEError
    rng = np.random.default_rng(9)
    data = np.minimum(rng.geometric(0.25, 300_000), 24).astype(np.uint8)  # skewed, codes <= 15 bits
    enc = codec.huffman_encode(data)
    lut, sb = codec.huffman_table(enc)
    d_enc = torch.from_numpy(np.frombuffer(enc, np.uint8).copy()).cuda()
    d_lut = torch.from_numpy(lut.view(np.int16).copy()).cuda()
    guard = 4096
    out = torch.full((data.size + guard,), 0xA5, dtype=torch.uint8, device="cuda")
    n = codec.huffman_decode_device(d_enc, len(enc), d_lut, sb, out)
    host = out.cpu().numpy()
    assert data.size <= n < data.size + 8
    np.testing.assert_array_equal(host[: data.size], data)
    assert (host[n:] == 0xA5).all()
    if short:
        full = host[:n].copy()
        out.fill_(0xA5)
        with pytest.raises(IEError) as e:
            codec.huffman_decode_device(d_enc, len(enc), d_lut, sb, out[: n - short])
        assert e.value.code == IE_ECAP
        host = out.cpu().numpy()
        assert (host[n - short:] == 0xA5).all()
        np.testing.assert_array_equal(host[: n - short], full[: n - short])
