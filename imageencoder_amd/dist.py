"""Frame-sharded gop=1 video encode across ranks with ONE bit-contiguous stream assembled on
rank 0 (the reference's serial frame loop is VideoEncoder.cpp:83-91 and its
frame concatenation Frame.cpp:31-45).

Protocol (one process per GPU, torch.distributed over RCCL -- or gloo on CPU in the tests):

1. Rank r owns frames [r*F/R, (r+1)*F/R).  Rank 0 encodes its frames straight into the root
   buffer after the settings header (start bit H); every other rank encodes into a local
   segment from bit 0.  ``seg_bits[r]`` = payload bits of rank r.
2. all_gather of the R bit counts (8 bytes each) -> every rank knows every global start bit
   S_r = H + sum_{q<r} seg_bits[q].
3. Rank r > 0 re-shifts its segment by S_r mod 8 on its own device (``ie_bitcopy``, a funnel
   shift), so its bytes line up with the root stream's bytes.
4. Point-to-point batch to root: the segment's first byte (it shares a byte with rank r-1's
   tail unless S_r is byte-aligned) goes to a small staging tensor, the rest lands in place at
   out[S_r/8 + 1 ...].  Root then ORs (or stores, when aligned) the first bytes.

The result is byte-identical to the single-device / reference gop=1 stream.  Only the segment
bytes cross xGMI (7/8 of the stream into root at N=8); the encode itself needs no collective.

:class:`PipelinedGather` is the production form of the same protocol: the batch is cut into
sub-batches ("chunks") assigned round-robin -- chunk k holds global frames
[k*R*m, (k+1)*R*m) and rank r encodes m of them, [(k*R + r)*m, (k*R + r + 1)*m) (chunk_frames) --
so the layout of chunk k depends only on chunks <= k.  Rank r's encode of chunk k+1 then overlaps the all_gather,
re-shift and point-to-point transfer of chunk k (separate HIP streams; RCCL orders its own).
RCCL message sizes are host arguments, so the chunk's bit counts are read back -- from a pinned
copy issued behind the all_gather.  The counts travel on a process group of their own (a second
communicator with its own stream), so a step issues every chunk's encode and count all_gather
before it waits for any count: the host blocks once per chunk only where that chunk's counts have
not yet arrived, and the device's encode queue never drains while the host assembles a chunk (the
data transfers, on the first group, do not queue behind later chunks' count gathers).
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np


def frame_range(nframes: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous frame range of ``rank`` (SURVEY §8e partitioning)."""
    return nframes * rank // world, nframes * (rank + 1) // world


def segment_starts(header_bits: int, seg_bits: Sequence[int]) -> list[int]:
    """Global start bit of every rank's segment."""
    s, out = header_bits, []
    for b in seg_bits:
        out.append(s)
        s += int(b)
    out.append(s)  # end of stream
    return out


def gather_stream(dist, rank: int, world: int, seg, seg_bits: int, header_bits: int, out_root,
                  shift: Callable, new_bytes: Callable, group=None) -> int:
    """Assemble the ranks' payload segments into ``out_root`` on rank 0.

    dist       torch.distributed
    seg        rank > 0: uint8 tensor holding seg_bits bits from bit 0 (ignored on rank 0, whose
               payload is already in out_root after the header)
    shift      shift(src_tensor, nbytes, start_bit) -> uint8 tensor with the src bits moved to
               start at bit ``start_bit`` (< 8), zero before it (ie_bitcopy on the GPU)
    new_bytes  new_bytes(n) -> zeroed uint8 tensor on this rank's device
    Returns the total stream length in bits (on every rank).
    """
    import torch

    counts = new_bytes(8 * world).view(torch.int64)
    mine = new_bytes(8).view(torch.int64)
    mine.fill_(int(seg_bits))
    dist.all_gather_into_tensor(counts, mine, group=group)
    bits = [int(v) for v in counts.cpu().tolist()]
    starts = segment_starts(header_bits, bits)
    total = starts[-1]
    ops = []
    if rank > 0 and bits[rank] > 0:
        s = starts[rank]
        nbytes = (bits[rank] + 7) // 8
        sh = shift(seg, nbytes, s % 8)
        span = (s % 8 + bits[rank] + 7) // 8
        ops.append(dist.P2POp(dist.isend, sh[:1], 0, group=group))
        if span > 1:
            ops.append(dist.P2POp(dist.isend, sh[1:span], 0, group=group))
    firsts = None
    if rank == 0:
        firsts = new_bytes(max(world, 1))
        for r in range(1, world):
            if bits[r] == 0:
                continue
            s = starts[r]
            span = (s % 8 + bits[r] + 7) // 8
            b0 = s // 8
            ops.append(dist.P2POp(dist.irecv, firsts[r:r + 1], r, group=group))
            if span > 1:
                ops.append(dist.P2POp(dist.irecv, out_root[b0 + 1:b0 + span], r, group=group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank == 0:
        for r in range(1, world):
            if bits[r] == 0:
                continue
            s = starts[r]
            b0 = s // 8
            if s % 8:
                out_root[b0:b0 + 1].bitwise_or_(firsts[r:r + 1])
            else:
                out_root[b0:b0 + 1].copy_(firsts[r:r + 1])
        # bits after the end of the stream in its last byte are zero
        if total % 8:
            last = total // 8
            keep = (0xFF << (8 - total % 8)) & 0xFF
            out_root[last:last + 1].bitwise_and_(keep)
    return total


def numpy_shift(src: np.ndarray, nbytes: int, start_bit: int) -> np.ndarray:
    """Reference bit shift for CPU tests: src bytes moved right by start_bit bits."""
    bits = np.unpackbits(np.asarray(src[:nbytes], dtype=np.uint8))
    out = np.concatenate([np.zeros(start_bit, np.uint8), bits])
    pad = (-out.size) % 8
    return np.packbits(np.concatenate([out, np.zeros(pad, np.uint8)]))


def chunk_frames(k: int, rank: int, world: int, nframes: int, nchunks: int) -> range:
    """Global frame indices of ``rank``'s part of chunk ``k``: chunk k is frames
    [k*F/K, (k+1)*F/K), split into ``world`` contiguous parts (a part may be empty).  With
    F = m*R*K this is rank r encoding frames [(k*R + r)*m, (k*R + r + 1)*m)."""
    c0, c1 = nframes * k // nchunks, nframes * (k + 1) // nchunks
    return range(c0 + (c1 - c0) * rank // world, c0 + (c1 - c0) * (rank + 1) // world)


class PipelinedGather:
    """Frame-sharded gop=1 stream assembly with encode / gather overlap (module docstring).

    encode(k, step, seg, bits)  launch the encode of this rank's part of chunk k (frames
                                ``chunk_frames(k, rank, world, nframes, nchunks)``, possibly none)
                                into ``seg`` from bit 0 (asynchronous, on ``enc_stream``) and
                                leave its payload bit count in the 1-element int64 device tensor
                                ``bits`` (stream-ordered)
    shift(src, nbytes, start, dst)  move src's bits to start at bit ``start`` (< 8) of ``dst``
                                (bits before it zero); runs on ``comm_stream``
    comm_dev                    device of the tensors handed to torch.distributed: the encode
                                device for RCCL, "cpu" for gloo (staged copies; rehearsal/tests)
    count_group                 the process group of the bit-count all_gathers (default: a new group
                                over ``group``'s ranks -- ``new_group`` is collective over the
                                default group, so then every process constructs this object)
    Rank 0's assembled stream is ``out[: (total + 7) // 8]`` after :meth:`step`.
    """

    def __init__(self, dist, rank: int, world: int, nframes: int, nchunks: int, header, header_bits: int,
                 seg_cap: int, root_cap: int, encode, shift, dev, comm_dev=None, enc_stream=None,
                 comm_stream=None, group=None, count_group=None):
        import torch
        self.torch, self.dist, self.group = torch, dist, group
        self.rank, self.world, self.F, self.K = rank, world, nframes, nchunks
        self.hb = header_bits
        self.encode, self.shift = encode, shift
        self.dev = torch.device(dev)
        self.cdev = torch.device(comm_dev) if comm_dev is not None else self.dev
        self.E, self.C = enc_stream, comm_stream
        cuda = self.dev.type == "cuda"
        z = lambda *shape, dt=torch.uint8, d=None: torch.zeros(*shape, dtype=dt, device=d or self.dev)  # noqa: E731
        self.segs = [z(seg_cap) for _ in range(nchunks)]
        self.shifted = [z(seg_cap + 8) for _ in range(nchunks)]
        self.bits = z(nchunks, dt=torch.int64)
        self.counts = z(nchunks, world, dt=torch.int64, d=self.cdev)
        self.counts_host = torch.zeros((nchunks, world), dtype=torch.int64, pin_memory=cuda)
        self.ev_enc = [torch.cuda.Event() for _ in range(nchunks)] if cuda else None
        self.ev_cnt = [torch.cuda.Event() for _ in range(nchunks)] if cuda else None
        self.ev_sent = [None] * nchunks  # comm work on seg k of the previous step
        hdr = torch.as_tensor(header, dtype=torch.uint8)
        self.out = None
        if rank == 0:
            self.out = z(root_cap)
            self.out[: hdr.numel()].copy_(hdr)
            self.hdr_last = hdr[-1:].to(self.dev) if header_bits % 8 else None
            self.firsts = z(nchunks, world)
        self.total = header_bits
        self._base = header_bits
        # the counts' own communicator (collective: every rank constructs this object in step)
        self.cgroup = count_group if count_group is not None else group
        self._own_cgroup = False
        if world > 1 and count_group is None:
            ranks = dist.get_process_group_ranks(group) if group is not None else list(range(world))
            # the counts travel on the transfers' backend: a gloo group under an NCCL default
            # group keeps its counts (CPU tensors) on gloo
            self.cgroup = dist.new_group(ranks=ranks, backend=dist.get_backend(group))
            self._own_cgroup = True
        self.CC = torch.cuda.Stream(self.dev) if (cuda and comm_stream is not None) else None

    def close(self) -> None:
        """Destroy the count communicator this object created (collective, like the constructor)."""
        if self._own_cgroup and self.cgroup is not None:
            self.dist.destroy_process_group(self.cgroup)
        self.cgroup = None
        self._own_cgroup = False

    # -- stream helpers (no-ops on the CPU)
    def _on(self, s):
        return self.torch.cuda.stream(s) if s is not None else _Null()

    def step(self, i: int) -> None:
        """Encode and assemble one whole batch (all chunks)."""
        if self.E is not None:
            # whatever the caller queued on its current stream before this step -- the frames, this
            # object's zero-filled buffers on the first step -- comes before the encode and the
            # transfers (the encode's end bits would otherwise race the zero fill of self.bits)
            cur = self.torch.cuda.current_stream(self.dev)
            self.E.wait_stream(cur)
            if self.C is not None:
                self.C.wait_stream(cur)
            if self.CC is not None:
                self.CC.wait_stream(cur)
        self._base = self.hb
        if self.rank == 0 and self.hdr_last is not None:  # the header's partial byte: ORed into below
            with self._on(self.C):
                self.out[self.hb // 8: self.hb // 8 + 1].copy_(self.hdr_last)
        # every encode and count gather first (no host wait), then each chunk's re-shift and
        # transfer as soon as its counts are on the host
        for k in range(self.K):
            self._encode(k, i)
            self._gather_counts(k)
        for k in range(self.K):
            self._finish(k)
        self.total = self._base

    def _encode(self, k, i):
        with self._on(self.E):
            if self.ev_sent[k] is not None:  # the previous step's transfer of this segment
                self.E.wait_event(self.ev_sent[k])
            self.encode(k, i, self.segs[k], self.bits[k:k + 1])
            if self.ev_enc:
                self.ev_enc[k].record(self.E)

    def _gather_counts(self, k):
        cs = self.CC if self.CC is not None else self.C
        with self._on(cs):
            if self.ev_enc:
                cs.wait_event(self.ev_enc[k])
            mine = self.bits[k:k + 1]
            if self.cdev != self.dev:
                mine = mine.to(self.cdev)
            if self.world == 1:  # one rank: no collective
                self.counts[k].copy_(mine)
            elif self.cdev.type == "cuda":
                self.dist.all_gather_into_tensor(self.counts[k], mine, group=self.cgroup)
            else:  # gloo
                self.dist.all_gather(list(self.counts[k].view(self.world, 1).unbind(0)), mine, group=self.cgroup)
            self.counts_host[k].copy_(self.counts[k], non_blocking=self.ev_cnt is not None)
            if self.ev_cnt:
                self.ev_cnt[k].record(cs)

    def _finish(self, k):
        """Re-shift and transfer chunk k (its counts are on the host once ev_cnt[k] fired)."""
        torch, dist, world, rank = self.torch, self.dist, self.world, self.rank
        if self.ev_cnt:
            self.ev_cnt[k].synchronize()
        bits = [int(v) for v in self.counts_host[k].tolist()]
        starts = segment_starts(self._base, bits)
        self._base = starts[-1]
        ops, tails = [], []
        with self._on(self.C):
            if bits[rank] > 0:
                s = starts[rank]
                nbytes = (bits[rank] + 7) // 8
                span = (s % 8 + bits[rank] + 7) // 8
                sh = self.shifted[k]
                sh[:8].zero_()
                self.shift(self.segs[k], nbytes, s % 8, sh)
                if rank == 0:
                    self.firsts[k, 0:1].copy_(sh[:1])
                    if span > 1:
                        self.out[s // 8 + 1: s // 8 + span].copy_(sh[1:span])
                else:
                    src = sh[:span] if self.cdev == self.dev else sh[:span].to(self.cdev)
                    ops.append(dist.P2POp(dist.isend, src[:1], 0, group=self.group))
                    if span > 1:
                        ops.append(dist.P2POp(dist.isend, src[1:span], 0, group=self.group))
            if rank == 0:
                for r in range(1, world):
                    if bits[r] == 0:
                        continue
                    s = starts[r]
                    span = (s % 8 + bits[r] + 7) // 8
                    b0 = s // 8
                    if self.cdev == self.dev:
                        ops.append(dist.P2POp(dist.irecv, self.firsts[k, r:r + 1], r, group=self.group))
                        if span > 1:
                            ops.append(dist.P2POp(dist.irecv, self.out[b0 + 1:b0 + span], r, group=self.group))
                    else:  # staged through host tensors (gloo)
                        f = torch.zeros(1, dtype=torch.uint8, device=self.cdev)
                        ops.append(dist.P2POp(dist.irecv, f, r, group=self.group))
                        body = None
                        if span > 1:
                            body = torch.zeros(span - 1, dtype=torch.uint8, device=self.cdev)
                            ops.append(dist.P2POp(dist.irecv, body, r, group=self.group))
                        tails.append((r, b0, span, f, body))
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
            if rank == 0:
                for r, b0, span, f, body in tails:
                    self.firsts[k, r:r + 1].copy_(f)
                    if body is not None:
                        self.out[b0 + 1:b0 + span].copy_(body)
                # after every byte of the chunk is in place: the first bytes.  A segment starting
                # inside a byte shares it with the stream before it (written earlier in this step:
                # OR); a byte-aligned one owns it (the buffer still holds the previous step: copy)
                for r in range(world):
                    if bits[r]:
                        b0 = starts[r] // 8
                        if starts[r] % 8:
                            self.out[b0:b0 + 1].bitwise_or_(self.firsts[k, r:r + 1])
                        else:
                            self.out[b0:b0 + 1].copy_(self.firsts[k, r:r + 1])
            if self.C is not None:
                ev = torch.cuda.Event()
                ev.record(self.C)
                self.ev_sent[k] = ev


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
