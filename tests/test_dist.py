"""Multi-rank stream assembly (imageencoder_amd/dist.py) on CPU with gloo: frame-sharded gop=1
video encode, all_gather of segment sizes, per-rank bit re-shift, point-to-point gather to rank 0.
The per-rank encode here is the CPU oracle (test infrastructure); the protocol under test is the
product's.  The assembled stream must equal the single-process reference stream byte for byte.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from imageencoder_amd import dist as D
from imageencoder_amd import synth, write_header
from tests import oracle_lib as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, w, h, nframes, gen, n, rle, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
        ys = synth.frames(gen, w, h, nframes, seed=77)
        f0, f1 = D.frame_range(nframes, rank, world)
        hdr, hb = write_header(n, q, rle, w, h, video=True, frames=nframes, gop=1, merange=16)
        oracle = O.load()
        cap = (hb + 7) // 8 + nframes * (w * h * 17 // 8 + w * h // (n * n)) + 64
        out_root = torch.zeros(cap, dtype=torch.uint8)
        seg, seg_bits = None, 0
        if f1 > f0:
            if rank == 0:
                buf = np.zeros(cap, np.uint8)
                buf[:hdr.size] = hdr
                _, end, _ = oracle.encode_blocks(ys[f0:f1], n, q, rle=rle, start_bit=hb, out=buf)
                out_root = torch.from_numpy(buf)
                seg_bits = end - hb
            else:
                buf, end, _ = oracle.encode_blocks(ys[f0:f1], n, q, rle=rle, start_bit=0)
                seg, seg_bits = torch.from_numpy(buf), end
        elif rank == 0:
            out_root[:hdr.size] = torch.from_numpy(hdr)

        def shift(src, nbytes, start):
            return torch.from_numpy(D.numpy_shift(src.numpy(), nbytes, start))

        total = D.gather_stream(dist, rank, world, seg, seg_bits, hb, out_root, shift,
                                lambda k: torch.zeros(k, dtype=torch.uint8))
        if rank == 0:
            result_q.put((total, out_root[: (total + 7) // 8].numpy().tobytes()))
    finally:
        dist.destroy_process_group()


def _run(world, w, h, nframes, gen, n=4, rle=True):
    ctx = mp.get_context("spawn")
    qres = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, nframes, gen, n, rle, qres))
             for r in range(world)]
    for p in procs:
        p.start()
    total, got = qres.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ys = synth.frames(gen, w, h, nframes, seed=77)
    q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
    ref = O.load().encode_video(synth.yuv420(ys), w, h, n, q, rle=rle, huffman=False, merange=16)
    return total, got, ref


@pytest.mark.parametrize("world,nframes,gen", [(2, 5, "U"), (2, 4, "M"), (3, 7, "M")])
def test_sharded_video_stream_matches_reference(world, nframes, gen):
    total, got, ref = _run(world, 64, 48, nframes, gen)
    assert got == ref
    assert (total + 7) // 8 == len(ref)


def test_sharded_more_ranks_than_frames():
    """Ranks with no frames contribute empty segments."""
    total, got, ref = _run(3, 32, 16, 2, "U")
    assert got == ref


def test_segment_starts_and_ranges():
    assert D.segment_starts(210, [5, 0, 11]) == [210, 215, 215, 226]
    rs = [D.frame_range(512, r, 8) for r in range(8)]
    assert rs[0] == (0, 64) and rs[-1] == (448, 512)
    assert sum(b - a for a, b in rs) == 512


@pytest.mark.parametrize("start", range(8))
def test_numpy_shift(start):
    rng = np.random.default_rng(start)
    src = rng.integers(0, 256, 37, dtype=np.uint8)
    out = D.numpy_shift(src, 37, start)
    bits = np.unpackbits(out)
    assert not bits[:start].any()
    assert np.array_equal(bits[start:start + 37 * 8], np.unpackbits(src))


def _pipe_worker(rank, world, port, w, h, F, nchunks, gen, steps, result_q, subgroup=False):
    """PipelinedGather on CPU/gloo: round-robin chunks, the oracle as each rank's encoder.
    subgroup: the transfers run on an explicit gloo group (the count communicator PipelinedGather
    creates takes that group's backend) and the object is closed and rebuilt once (no leak)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 4
        q = O.read_matrix("matrix.txt", n)
        oracle = O.load()
        hdr, hb = write_header(n, q, True, w, h, video=True, frames=F, gop=1, merange=16)
        cap = (hb + 7) // 8 + F * (w * h * 17 // 8 + w * h // (n * n)) + 64
        seg_cap = F * (w * h * 17 // 8 + w * h // (n * n)) + 64

        def frames_for(k, step):  # each step encodes a different batch (seed offset)
            fr = D.chunk_frames(k, rank, world, F, nchunks)
            return synth.frames(gen, w, h, F, seed=77 + step)[fr.start:fr.stop]

        def encode(k, step, seg, bits):
            y = frames_for(k, step)
            seg.zero_()
            if len(y) == 0:
                bits.fill_(0)
                return
            buf, end, _ = oracle.encode_blocks(y, n, q, rle=True, start_bit=0)
            seg[: buf.size].copy_(torch.from_numpy(buf))
            bits.fill_(end)

        def shift(src, nbytes, start, dst):
            v = torch.from_numpy(D.numpy_shift(src.numpy(), nbytes, start))
            dst[: v.numel()].copy_(v)

        grp = dist.new_group(ranks=list(range(world)), backend="gloo") if subgroup else None
        if subgroup:  # a throw-away gather: its count communicator is destroyed by close()
            D.PipelinedGather(dist, rank, world, F, nchunks, hdr, hb, seg_cap, cap, encode, shift, "cpu",
                              group=grp).close()
        g = D.PipelinedGather(dist, rank, world, F, nchunks, hdr, hb, seg_cap, cap, encode, shift, "cpu", group=grp)
        outs = []
        for step in range(steps):
            g.step(step)
            if rank == 0:
                outs.append((g.total, g.out[: (g.total + 7) // 8].numpy().tobytes()))
        g.close()
        if rank == 0:
            result_q.put(outs)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,F,nchunks,gen,subgroup",
                         [(2, 8, 2, "U", False), (3, 9, 3, "M", False), (2, 5, 2, "M", True), (3, 2, 1, "U", False)])
def test_pipelined_gather_matches_reference(world, F, nchunks, gen, subgroup):
    """Round-robin chunks assembled by PipelinedGather equal the single-process gop=1 stream of
    the same frames in global order, for two consecutive steps over different frames (the root
    buffer is reused: stale bytes must not leak into the next stream)."""
    w, h, steps = 64, 48, 2
    ctx = mp.get_context("spawn")
    qres = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, w, h, F, nchunks, gen, steps, qres, subgroup))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = qres.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    q = O.read_matrix("matrix.txt", 4)
    for step, (total, got) in enumerate(outs):
        ys = synth.frames(gen, w, h, F, seed=77 + step)
        ref = O.load().encode_video(synth.yuv420(ys), w, h, 4, q, rle=True, huffman=False, merange=16)
        assert got == ref, f"step {step}"
        assert (total + 7) // 8 == len(ref)


def test_chunk_frames_round_robin():
    got = [list(D.chunk_frames(k, r, 3, 12, 2)) for k in range(2) for r in range(3)]
    assert got == [[0, 1], [2, 3], [4, 5], [6, 7], [8, 9], [10, 11]]
    got = [list(D.chunk_frames(k, r, 2, 5, 2)) for k in range(2) for r in range(2)]
    assert sum(got, []) == list(range(5))
