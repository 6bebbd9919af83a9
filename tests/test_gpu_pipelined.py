"""encode4q_kernel -- the software-pipelined persistent 4x4 encoder that large segmented FAST
batches run when IE_PIPELINED=1 (ie_encode.hip; launch_encode4w routes batches of >= 2 grids of
tiles to it; opt-in: measured slower than encode4p_kernel).  Its
streams must be, byte for byte, what one-frame launches (encode4p_kernel) and the all-FP64 EXACT
kernel write: ImageEncoder::process per frame (ImageEncoder.cpp:96-147), Block::streamEncoded
(Block.cpp:372-413) and BitStreamWriter (BitStream.cpp:61-77) are the reference behaviour; those
two paths are pinned against the reference-generated goldens in test_gpu_encode.py."""
import numpy as np
import pytest

from imageencoder_amd import MODE_EXACT, MODE_FAST, synth
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    from imageencoder_amd import Codec
    return Codec(0)


@pytest.fixture(autouse=True)
def pipelined(monkeypatch):
    monkeypatch.setenv("IE_PIPELINED", "1")  # read by the library at every launch


def _batch(codec, y, w, h, f, start_bit, mode):
    import torch
    from imageencoder_amd import stream_bound
    pitch = (stream_bound(w, h, 4, 1, start_bit) + 63) // 64 * 64
    out = torch.zeros(pitch * f, dtype=torch.uint8, device="cuda")
    ends = codec.encode_images(y, w, h, out, out_pitch=pitch, nframes=f, start_bit=start_bit, mode=mode)
    return out.view(f, pitch), np.asarray(ends, dtype=np.uint64), pitch


@pytest.mark.parametrize("start_bit", [0, 165])
@pytest.mark.parametrize("kind", ["U", "M"])
def test_pipelined_batch_equals_single_launches(codec, kind, start_bit):
    """6 4K frames in one launch (3 036 tiles: the pipelined kernel, tiles of two rounds per
    workgroup, deferred back ends, tile-boundary words by exchange) == each frame in a launch of
    its own (one tile per workgroup) == the EXACT kernel's batch."""
    import torch
    q = O.read_matrix("matrix.txt", 4)
    codec.set_quant(q, 4)
    w, h, f = 3840, 2160, 6
    y = torch.from_numpy(synth.frames(kind, w, h, f, seed=2024 + start_bit)).cuda()
    a, ea, pitch = _batch(codec, y, w, h, f, start_bit, MODE_FAST)
    b, eb, _ = _batch(codec, y, w, h, f, start_bit, MODE_EXACT)
    assert np.array_equal(ea, eb)
    for i in range(f):
        nb = int(ea[i] + 7) // 8
        assert torch.equal(a[i, :nb], b[i, :nb]), f"frame {i}: pipelined FAST != EXACT"
        one, e1, _ = _batch(codec, y[i:i + 1], w, h, 1, start_bit, MODE_FAST)  # (one tile per workgroup)
        assert int(e1[0]) == int(ea[i])
        assert torch.equal(a[i, :nb], one[0, :nb]), f"frame {i}: batch != single launch"


def test_pipelined_slot_pairs(codec):
    """All-ones matrix on 0/255 noise: the widest records, wave images larger than a buffer, so
    every tile's back end runs at once in slot pairs (the non-deferred branch); == EXACT."""
    import torch
    codec.set_quant(np.ones(16, dtype=np.uint16), 4)
    w, h, f = 3840, 2160, 5
    rng = np.random.default_rng(11)
    y = torch.from_numpy((rng.integers(0, 2, size=(f, h, w)) * 255).astype(np.uint8)).cuda()
    a, ea, _ = _batch(codec, y, w, h, f, 7, MODE_FAST)
    b, eb, _ = _batch(codec, y, w, h, f, 7, MODE_EXACT)
    assert np.array_equal(ea, eb)
    for i in range(f):
        nb = int(ea[i] + 7) // 8
        assert torch.equal(a[i, :nb], b[i, :nb]), f"frame {i}"


def test_pipelined_mixed_tiles(codec):
    """Frames alternating flat / noise / gradient content in one batch: tiles whose images fit
    (deferred back ends) next to tiles that do not (immediate), under a mid-range matrix."""
    import torch
    codec.set_quant(np.full(16, 2, dtype=np.uint16), 4)
    w, h, f = 3840, 2160, 6
    rng = np.random.default_rng(5)
    fr = []
    for i in range(f):
        if i % 3 == 0:
            fr.append(np.full((h, w), 128, dtype=np.uint8))
        elif i % 3 == 1:
            fr.append(rng.integers(0, 256, size=(h, w), dtype=np.uint8))
        else:
            fr.append((np.indices((h, w)).sum(axis=0) % 256).astype(np.uint8))
    y = torch.from_numpy(np.stack(fr)).cuda()
    a, ea, _ = _batch(codec, y, w, h, f, 31, MODE_FAST)
    b, eb, _ = _batch(codec, y, w, h, f, 31, MODE_EXACT)
    assert np.array_equal(ea, eb)
    for i in range(f):
        nb = int(ea[i] + 7) // 8
        assert torch.equal(a[i, :nb], b[i, :nb]), f"frame {i}"
