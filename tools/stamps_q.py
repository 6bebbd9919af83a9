"""Summarise encode4q_kernel's per-iteration phase stamps (IE_PROFILE build, IE_STAMPS=file:
s_memtime by every wave's lane 0, row = the iteration's tile [tile][4 waves][16]).
Iteration k of a workgroup: pixel wait (11-0), transform (0-1), fix-up (1-2), sizing (2-3),
count (3-4: wave 0 polls the four counts), back end of tile k-1 -- look-back (4-5, wave 0),
position barrier (5-6 wave 0 / 4-6 others), store (6-7) --, DMA + zero (7-8), emission (8-9),
an immediate back end (9-10).  usage: python tools/stamps_q.py stamps.bin [clock_ghz]"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4, 16).astype(np.int64)
ghz = float(sys.argv[2]) if len(sys.argv) > 2 else 2.4
rows = raw.reshape(-1, 16)
wave = np.tile(np.arange(4), raw.shape[0])
ok = (rows[:, [11, 0, 1, 2, 3, 4, 8, 9, 10]] > 0).all(axis=1)
rows, wave = rows[ok], wave[ok]
us = lambda a, b: (rows[:, b] - rows[:, a]) / ghz / 1e3
hb = (rows[:, 6] > 0) & (rows[:, 7] > 0)  # iterations that ran a deferred back end
w0 = wave == 0
print(f"wave-iterations {len(rows)} (with a deferred back end {hb.sum()})")
print("phase                    all     wave0   waves1-3   p90")
def line(nm, d, m=None):
    m = np.ones(len(d), bool) if m is None else m
    a, z, o = d[m], d[m & w0], d[m & ~w0]
    print(f"{nm:22s} {a.mean():7.3f} {z.mean() if len(z) else 0:8.3f} {o.mean() if len(o) else 0:9.3f} "
          f"{np.percentile(a, 90):7.3f}")
line("pixel wait", us(11, 0))
line("transform", us(0, 1))
line("fix-up", us(1, 2))
line("size+scan", us(2, 3))
line("count", us(3, 4))
lb = (rows[:, 5] > 0) & hb & w0
if lb.any():
    line("look-back (w0)", us(4, 5), lb)
    line("barrier (w0)", us(5, 6), lb)
line("to position (1-3)", us(4, 6), hb & ~w0)
line("store", us(6, 7), hb)
line("dma+zero", np.where(hb, us(7, 8), us(4, 8)))
line("emission", us(8, 9))
line("immediate back", us(9, 10))
it = us(11, 10)
print(f"iteration mean {it.mean():.2f} us  p50 {np.median(it):.2f}")
rt = raw.reshape(-1, 16)[:, 14:16]
rt = rt[(rt > 0).all(axis=1)]
if len(rt):
    st = (rt[:, 0] - rt[:, 0].min()) / 100.0
    en = (rt[:, 1] - rt[:, 0].min()) / 100.0
    print(f"launch span {en.max():.2f} us: iteration starts p50 {np.median(st):.2f} max {st.max():.2f}; "
          f"ends p50 {np.median(en):.2f} p90 {np.percentile(en, 90):.2f}")
