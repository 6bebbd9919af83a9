"""Seeded, portable synthetic 8-bit frames.

Counter-based splitmix64, so any pixel can be generated independently and numpy, a C harness
or a GPU can reproduce the same bytes.  Two generators:

* ``uniform`` (U): ``u8 = splitmix64(seed, i) & 0xFF`` over the frame in raster order -- the
  worst case (no all-zero blocks, many RLE-truncation blocks).
* ``mixed``   (M): 64x64 tiles whose kind is ``splitmix64(seed ^ TILE_SALT, tile) % 3``:
  0 = flat 128 (all-zero blocks, the ``ffs(0)`` path), 1 = slow gradient + [-2, 2] noise,
  2 = uniform noise.
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
TILE_SALT = 0x5EED7115
DEFAULT_SEED = 0x1E0C0DE


def splitmix64(seed: int, start: int, count: int) -> np.ndarray:
    """Outputs ``start .. start+count-1`` of the splitmix64 sequence seeded with ``seed``."""
    with np.errstate(over="ignore"):
        i = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * GAMMA
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def uniform(w: int, h: int, seed: int = DEFAULT_SEED) -> np.ndarray:
    return (splitmix64(seed, 0, w * h) & np.uint64(0xFF)).astype(np.uint8).reshape(h, w)


def mixed(w: int, h: int, seed: int = DEFAULT_SEED, tile: int = 64) -> np.ndarray:
    tx, ty = -(-w // tile), -(-h // tile)
    kind = (splitmix64(seed ^ TILE_SALT, 0, tx * ty) % np.uint64(3)).astype(np.int64).reshape(ty, tx)
    kmap = np.repeat(np.repeat(kind, tile, axis=0), tile, axis=1)[:h, :w]
    r = splitmix64(seed, 0, w * h).reshape(h, w)
    noise = (r & np.uint64(0xFF)).astype(np.int64)
    small = ((r >> np.uint64(8)) % np.uint64(5)).astype(np.int64) - 2
    yy, xx = np.mgrid[0:h, 0:w]
    grad = ((xx + 2 * yy) * 255) // max(1, (w + 2 * h))
    out = np.where(kmap == 0, 128, np.where(kmap == 1, np.clip(grad + small, 0, 255), noise))
    return out.astype(np.uint8)


def frame(kind: str, w: int, h: int, seed: int = DEFAULT_SEED) -> np.ndarray:
    if kind in ("U", "uniform"):
        return uniform(w, h, seed)
    if kind in ("M", "mixed"):
        return mixed(w, h, seed)
    raise ValueError(f"unknown synthetic kind {kind!r}")


def frames(kind: str, w: int, h: int, count: int, seed: int = DEFAULT_SEED) -> np.ndarray:
    """``count`` distinct frames (seed + frame index), shape (count, h, w).  Kind "P" (panning):
    windows of one larger "mixed" picture moving by (3, 2) px per frame plus +-2 noise -- content
    a motion search can follow (the P-frame tests)."""
    out = np.empty((count, h, w), dtype=np.uint8)
    if kind in ("P", "panning"):
        base = mixed(w + 3 * count + 8, h + 2 * count + 8, seed).astype(np.int64)
        for f in range(count):
            noise = (splitmix64(seed + 1 + f, 0, w * h) % np.uint64(5)).astype(np.int64).reshape(h, w) - 2
            out[f] = np.clip(base[2 * f: 2 * f + h, 3 * f: 3 * f + w] + noise, 0, 255).astype(np.uint8)
        return out
    for f in range(count):
        out[f] = frame(kind, w, h, seed + f)
    return out


def yuv420(y: np.ndarray, fill: int = 0x80) -> bytes:
    """Pack (count, h, w) Y planes as a YUV420 file: Y then w*h/2 chroma bytes per frame
    (VideoBase.cpp:8-9,39-40 read only the Y plane)."""
    count, h, w = y.shape
    buf = np.full((count, h * w + h * w // 2), fill, dtype=np.uint8)
    buf[:, : h * w] = y.reshape(count, h * w)
    return buf.tobytes()


def _u64(v: int) -> int:
    """A 64-bit constant as the signed int64 torch stores (two's complement)."""
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >> 63 else v


def uniform_device(w: int, h: int, count: int, seed: int, device, torch=None):
    """``frames("U", w, h, count, seed)`` generated on a torch device: the same splitmix64 bytes
    (int64 arithmetic wraps like uint64; right shifts are masked to be logical).  Bench and test
    data only -- the generator, not the product."""
    if torch is None:
        import torch
    out = torch.empty((count, h, w), dtype=torch.uint8, device=device)
    n = w * h
    i = torch.arange(1, n + 1, dtype=torch.int64, device=device)
    g, m1, m2 = _u64(0x9E3779B97F4A7C15), _u64(0xBF58476D1CE4E5B9), _u64(0x94D049BB133111EB)

    def srl(z, k):
        return (z >> k) & ((1 << (64 - k)) - 1)

    for f in range(count):
        z = i * g + _u64(seed + f)
        z = (z ^ srl(z, 30)) * m1
        z = (z ^ srl(z, 27)) * m2
        z = z ^ srl(z, 31)
        out[f].view(-1).copy_((z & 0xFF).to(torch.uint8))
    return out
