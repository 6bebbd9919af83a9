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


def _worker_c4(rank, world, port, F, nchunks, steps, q_out):
    """BASELINE configs[3] at its shape: F 1920x1080 frames, 4x4, matrix.txt, one gop=1 stream
    assembled on rank 0 by PipelinedGather (K pipelined sub-batches, round-robin frame ownership),
    compared with ONE ie_encode_frames launch over the same F frames on rank 0."""
    import torch
    import torch.distributed as dist

    from imageencoder_amd import MODE_EXACT, Codec, read_matrix, stream_bound, synth, write_header
    from imageencoder_amd import dist as D
    from tests import oracle_lib as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ["IE_FORCE_TICKET"] = "1"  # ranks share one GPU (see _worker)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w, h, n = 1920, 1080, 4
        q = read_matrix(os.path.join(O.GOLDEN, "matrix.txt"), n)
        dev = torch.device("cuda", 0)
        m = F // (world * nchunks)  # frames per rank per sub-batch
        seed = synth.DEFAULT_SEED + 4242
        mine = torch.empty((nchunks, m, h, w), dtype=torch.uint8, device=dev)
        for k in range(nchunks):
            fr = D.chunk_frames(k, rank, world, F, nchunks)
            assert len(fr) == m
            mine[k].copy_(synth.uniform_device(w, h, m, seed + fr.start, dev, torch))
        enc, shifter = Codec(0, q, n), Codec(0, q, n)
        E, C = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        enc.set_stream(E.cuda_stream)
        shifter.set_stream(C.cuda_stream)
        hdr, hb = write_header(n, q, True, w, h, video=True, frames=F, gop=1, merange=16)

        def encode(k, step, seg, bits):
            enc.encode_frames(mine[k], w, h, seg, start_bit=0, nframes=m, want_sizes=False)
            enc.end_bits_into(bits)

        def shift(src, nbytes, start, dst):
            shifter.bitcopy(src[:nbytes], dst, start)

        G = D.PipelinedGather(dist, rank, world, F, nchunks, hdr, hb, stream_bound(w, h, n, m, 0) + 64,
                              stream_bound(w, h, n, F, hb) + 64, encode, shift, dev, comm_dev="cpu",
                              enc_stream=E, comm_stream=C)
        res, counts = [], []
        for s in range(steps):
            G.step(s)
            torch.cuda.synchronize()
            enc.sync()
            shifter.sync()
            if rank == 0:
                res.append((G.total, hashlib.md5(G.out[: (G.total + 7) // 8].cpu().numpy().tobytes()).hexdigest()))
                counts.append(G.counts_host.tolist())
        del mine
        if rank == 0:
            allf = synth.uniform_device(w, h, F, seed, dev, torch)
            ref = torch.zeros(stream_bound(w, h, n, F, hb) + 64, dtype=torch.uint8, device=dev)
            ref[: hdr.size].copy_(torch.from_numpy(hdr).to(dev))
            # the reference launch in EXACT mode (encode_kernel<4, true>, FP64 everywhere, pinned to
            # the oracle): independent of the ticket-mode FAST kernel the ranks ran
            _, end = enc.encode_frames(allf, w, h, ref, start_bit=hb, nframes=F, mode=MODE_EXACT)
            q_out.put((res, (end, hashlib.md5(ref[: (end + 7) // 8].cpu().numpy().tobytes()).hexdigest()), counts))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_c4_shape_512_frames_8_ranks():
    """configs[3] (C4) at its configured shape: all 512 1920x1080 frames through PipelinedGather with
    K = 4 sub-batches over 8 ranks (spawned processes sharing cuda:0, gloo control plane).  The
    assembled stream of two consecutive steps equals one single-launch encode of the 512 frames
    (VideoEncoder.cpp:83-91 / Frame.cpp:31-45 semantics; the 1080p x 3 reference golden pins that
    single launch in test_multirank_hip_stream_matches_golden and tests/test_gpu_files.py)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    world, F, K = 8, 512, 4
    procs = [ctx.Process(target=_worker_c4, args=(r, world, port, F, K, 2, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res, single, counts = q.get(timeout=480)
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    # (on failure: every step's per-chunk, per-rank segment bits as rank 0 received them)
    assert res == [single] * 2, counts
