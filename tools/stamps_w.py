"""Summarise encode4w_kernel's per-wave phase stamps (IE_PROFILE build, IE_STAMPS=file: s_memtime at
each phase boundary by every wave's lane 0, [tile][4 waves][12]) of one launch.
usage: python tools/stamps_w.py stamps.bin [clock_ghz]"""
import sys

import numpy as np

names = ["load", "transform", "fix-up", "size+scan", "barrier(count)", "emit pair 0", "look-back",
         "barrier(position)", "store pair 0", "refill+store pair 1"]
raw = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 64).astype(np.int64)
ghz = float(sys.argv[2]) if len(sys.argv) > 2 else 2.3
w16 = raw.reshape(-1, 4, 16)
w = w16[:, :, :11]
rows = w.reshape(-1, 11)
wave = np.tile(np.arange(4), len(w))
ok = (rows > 0).all(axis=1)
rows, wave = rows[ok], wave[ok]
d = np.diff(rows, axis=1) / ghz / 1e3
print(f"waves {len(rows)}")
print("phase                 all_mean  wave0  waves1-3   p90")
for i, nm in enumerate(names):
    print(f"{nm:20s} {d[:, i].mean():8.3f} {d[wave == 0, i].mean():7.3f} {d[wave > 0, i].mean():8.3f} "
          f"{np.percentile(d[:, i], 90):7.3f}")
life = (rows[:, -1] - rows[:, 0]) / ghz / 1e3
print(f"wave lifetime mean {life.mean():.2f} us  p50 {np.median(life):.2f}")
rt = w16.reshape(-1, 16)[:, 14:16]
rt = rt[(rt > 0).all(axis=1)]
if len(rt):  # chip-wide 100 MHz clock: starts and ends across the launch
    st = (rt[:, 0] - rt[:, 0].min()) / 100.0
    en = (rt[:, 1] - rt[:, 0].min()) / 100.0
    print(f"launch span {en.max():.2f} us: wave starts p50 {np.median(st):.2f} p90 {np.percentile(st, 90):.2f} "
          f"max {st.max():.2f}; ends p50 {np.median(en):.2f} p90 {np.percentile(en, 90):.2f}")
# encode4p_kernel's prologue on the 100 MHz clock (words 13 entry, 12 own loads landed, 11 past
# the first barrier, 14 the tile's start; tools/conc.py reads the same words)
pr = w16.reshape(-1, 16)[:, [13, 12, 11, 14]]
pr = pr[(pr > 0).all(axis=1)]
if len(pr):
    dd = np.diff(pr, axis=1) / 100.0
    print(f"prologue ({len(pr)} waves): entry -> loads landed {dd[:, 0].mean():.2f}, -> past the barrier "
          f"{dd[:, 1].mean():.2f}, -> tile start {dd[:, 2].mean():.2f} us")
