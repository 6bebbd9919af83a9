"""Summarise IE_STAMPS per-tile phase timestamps (s_memtime: shader clock, one counter per XCD)
of one encode launch.  usage: python tools/stamps.py stamps.bin [clock_ghz]"""
import sys

import numpy as np

names = ["start", "-", "load", "quant", "fix", "size", "scan", "emit", "lookback", "store"]
# kStamps (ie_device.h) words per tile; encode_kernel's thread 0 writes the first 16 (the rest
# belong to encode4w/4p's per-wave stamps, tools/stamps_w.py)
raw16 = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 64)[:, :16].astype(np.int64)
raw = raw16[:, :10].copy()
ghz = float(sys.argv[2]) if len(sys.argv) > 2 else 2.4
dbg = raw[:, 1]
print(f"look-back: retry rounds/tile {np.mean((dbg >> 32) & 0xFFFF):.2f} (max {((dbg >> 32) & 0xFFFF).max()}), "
      f"extra windows/tile {np.mean(dbg >> 48):.3f}, tail polls/tile {np.mean(dbg & 0xFFFFFFFF):.2f}, "
      f"tiles that polled the tail {np.mean((dbg & 0xFFFFFFFF) > 0):.3f}")
raw[:, 1] = 1
cols = [0, 2, 3, 4, 5, 6, 7, 8, 9]
st = raw[:, cols]
tiles = np.arange(len(raw))
ok = (st > 0).all(axis=1)
st, tiles = st[ok], tiles[ok]
d = np.diff(st, axis=1) / ghz / 1e3
print(f"tiles {len(st)}")
print("phase        mean_us  p50_us  p90_us")
for i in range(1, len(cols)):
    print(f"{names[cols[i]]:10s} {d[:, i - 1].mean():8.3f} {np.median(d[:, i - 1]):7.3f} {np.percentile(d[:, i - 1], 90):7.3f}")
life = (st[:, -1] - st[:, 0]) / ghz / 1e3
print(f"tile lifetime mean {life.mean():.2f} us  p50 {np.median(life):.2f}")
for x in range(2):  # timelines of two XCDs (tile % 8 = XCD for a one-tile-per-workgroup grid)
    sel = (tiles % 8) == x
    rel = (st[sel] - st[sel][:, 0].min()) / ghz / 1e3
    span = rel[:, -1].max()
    T = np.linspace(0, span, 30)
    inflight = [int(((rel[:, 0] <= v) & (rel[:, -1] > v)).sum()) for v in T]
    print(f"xcd {x}: span {span:.1f} us, tiles in flight over time:", " ".join(map(str, inflight)))

fx = raw16[:, [3, 10, 11, 12]]
sel = (fx > 0).all(axis=1)
if sel.any():
    dd = np.diff(fx[sel], axis=1) / ghz / 1e3
    print(f"fix-up (tiles whose wave 0 had tasks: {sel.mean():.2f}): to task list {dd[:, 0].mean():.3f} us, "
          f"round compute {dd[:, 1].mean():.3f} us, read-back {dd[:, 2].mean():.3f} us")
