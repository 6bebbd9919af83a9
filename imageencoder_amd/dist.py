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
