"""BASELINE configs[3] (C4) per rank, on the PRODUCT kernel (no ticket mode): the launch a real
8-GPU run makes on every rank -- 64 1920x1080 frames, one gop=1 stream, one 8 128-tile look-back
chain through encode4p_kernel -- checked against an independent result, the EXACT mode
(encode_kernel<4, true>: FP64 for every coefficient, pinned to the oracle and the reference's
goldens in test_gpu_encode.py / test_gpu_files.py).  Then the same frames through
imageencoder_amd.dist.PipelinedGather at world 1 with K = 4 sub-batches (real encode4p launches +
ie_bitcopy + the in-place assembly on the device) must equal that single launch.
Reference semantics: VideoEncoder.cpp:83-91 (frames in order), Frame.cpp:31-45 (records
concatenated at bit granularity).
"""
import os

import pytest

from imageencoder_amd import MODE_EXACT, MODE_FAST, synth

pytestmark = pytest.mark.gpu

W, H, F, N = 1920, 1080, 64, 4


@pytest.fixture(scope="module")
def c4():
    import torch

    from imageencoder_amd import Codec, read_matrix, stream_bound, write_header
    from tests import oracle_lib as O
    assert "IE_FORCE_TICKET" not in os.environ or os.environ["IE_FORCE_TICKET"] == "0"
    q = read_matrix(os.path.join(O.GOLDEN, "matrix.txt"), N)
    dev = torch.device("cuda", 0)
    y = synth.uniform_device(W, H, F, synth.DEFAULT_SEED + 77, dev, torch)
    hdr, hb = write_header(N, q, True, W, H, video=True, frames=F, gop=1, merange=16)
    cap = stream_bound(W, H, N, F, hb) + 64
    codec = Codec(0, q, N)

    def encode(mode, env=None):
        old = {k: os.environ.get(k) for k in (env or {})}
        os.environ.update(env or {})
        try:
            out = torch.zeros(cap, dtype=torch.uint8, device=dev)
            out[: hdr.size].copy_(torch.from_numpy(hdr).to(dev))
            fb, end = codec.encode_frames(y, W, H, out, start_bit=hb, nframes=F, mode=mode)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        return out, fb, end

    exact = encode(MODE_EXACT)
    yield dict(torch=torch, codec=codec, y=y, q=q, hdr=hdr, hb=hb, exact=exact, encode=encode, dev=dev)
    codec.close()


def test_c4_rank_launch_product_equals_exact(c4):
    """One launch of 64 1080p frames (one chain of 8 128 tiles) through the FAST product kernel
    (encode4p_kernel) is byte-identical to the EXACT mode's stream, frame bits and end bit."""
    torch = c4["torch"]
    out, fb, end = c4["encode"](MODE_FAST)
    xo, xfb, xend = c4["exact"]
    assert end == xend
    assert (fb == xfb).all()
    nb = (end + 7) // 8
    assert torch.equal(out[:nb], xo[:nb])
    assert int(out[nb:].count_nonzero()) == 0  # nothing written past the stream


def test_c4_pipelined_gather_world1_equals_single_launch(c4):
    """PipelinedGather at world 1, K = 4: the product encode of each 16-frame sub-batch from bit 0,
    re-shifted on the device by ie_bitcopy and assembled in place after the header, over two
    consecutive steps (the root buffer is reused), equals the single 64-frame launch."""
    torch = c4["torch"]
    from imageencoder_amd import Codec, stream_bound
    from imageencoder_amd import dist as D
    K, m = 4, F // 4
    dev = c4["dev"]
    enc, shifter = Codec(0, c4["q"], N), Codec(0, c4["q"], N)
    E, Cs = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    enc.set_stream(E.cuda_stream)
    shifter.set_stream(Cs.cuda_stream)
    y = c4["y"]

    def encode(k, step, seg, bits):
        fr = D.chunk_frames(k, 0, 1, F, K)
        assert len(fr) == m
        enc.encode_frames(y[fr.start:fr.stop], W, H, seg, start_bit=0, nframes=m, want_sizes=False)
        enc.end_bits_into(bits)

    def shift(src, nbytes, start, dst):
        shifter.bitcopy(src[:nbytes], dst, start)

    hb = c4["hb"]
    G = D.PipelinedGather(None, 0, 1, F, K, c4["hdr"], hb, stream_bound(W, H, N, m, 0) + 64,
                          stream_bound(W, H, N, F, hb) + 64, encode, shift, dev, enc_stream=E, comm_stream=Cs)
    xo, _, xend = c4["exact"]
    try:
        for s in range(2):
            G.step(s)
            torch.cuda.synchronize()
            enc.sync()
            shifter.sync()
            assert G.total == xend
            nb = (xend + 7) // 8
            assert torch.equal(G.out[:nb], xo[:nb])
    finally:
        enc.close()
        shifter.close()
