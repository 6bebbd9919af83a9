"""Multi-rank gop=1 stream assembly THROUGH THE HIP ENCODER: ranks are
spawned processes sharing cuda:0 (one GPU on the test box; RCCL refuses two ranks on one device,
so the control plane is gloo with host-staged transfers), each encoding its frames with
libie_hip.so, re-shifting with ie_bitcopy and handing its segment to imageencoder_amd.dist's
PipelinedGather -- the product protocol bench.py runs over RCCL.  The assembled stream must equal
the reference encoder's golden gop=1 stream (tests/golden manifest md5) byte for byte, for several
consecutive steps (the root buffer is reused between steps).
"""
import hashlib
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, nchunks, steps, q_out):
    import torch
    import torch.distributed as dist

    from imageencoder_amd import Codec, read_matrix, stream_bound, synth, write_header
    from imageencoder_amd import dist as D
    from tests import oracle_lib as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # the ranks share one GPU: order tiles by atomic ticket, so concurrent look-back kernels of the
    # two processes can never hold each other's predecessor tiles off the CUs
    os.environ["IE_FORCE_TICKET"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = {x["name"]: x for x in O.manifest()}[name]
        w, h, F, n = c["w"], c["h"], c["input"]["frames"], c["n"]
        q = read_matrix(os.path.join(O.GOLDEN, c["matrix"]), n)
        dev = torch.device("cuda", 0)
        ys = torch.from_numpy(synth.frames(c["input"]["gen"], w, h, F, seed=c["input"]["seed"])).to(dev)
        enc, shifter = Codec(0, q, n), Codec(0, q, n)
        E, C = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        enc.set_stream(E.cuda_stream)
        shifter.set_stream(C.cuda_stream)
        hdr, hb = write_header(n, q, True, w, h, video=True, frames=F, gop=1, merange=16)

        def encode(k, step, seg, bits):
            fr = D.chunk_frames(k, rank, world, F, nchunks)
            if len(fr) == 0:
                bits.zero_()
                return
            enc.encode_frames(ys[fr.start:fr.stop], w, h, seg, start_bit=0, nframes=len(fr), want_sizes=False)
            enc.end_bits_into(bits)

        def shift(src, nbytes, start, dst):
            shifter.bitcopy(src[:nbytes], dst, start)

        G = D.PipelinedGather(dist, rank, world, F, nchunks, hdr, hb, stream_bound(w, h, n, F, 0) + 64,
                              stream_bound(w, h, n, F, hb) + 64, encode, shift, dev, comm_dev="cpu",
                              enc_stream=E, comm_stream=C)
        md5s = []
        for s in range(steps):
            G.step(s)
            torch.cuda.synchronize()
            enc.sync()
            shifter.sync()
            if rank == 0:
                md5s.append(hashlib.md5(G.out[: (G.total + 7) // 8].cpu().numpy().tobytes()).hexdigest())
        if rank == 0:
            q_out.put((md5s, c["md5"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,world,nchunks", [("vidU1080x3_4x4", 2, 1), ("vidU1080x3_4x4", 2, 2),
                                                ("vidM64x48x5_4x4", 2, 2), ("vidM64x48x5_4x4", 3, 2)])
def test_multirank_hip_stream_matches_golden(name, world, nchunks):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, nchunks, 3, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        md5s, want = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert md5s == [want] * 3
