"""Tile concurrency over one encode4p launch from its stamps (IE_PROFILE build): the workgroup's
entry (wave 0 word 13), wave 0's tile start after the first pixels landed (14) and its end (15),
all on the chip-wide 100 MHz clock.  usage: python tools/conc.py stamps.bin [--issue]"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 64).astype(np.int64)
ent, st, en = raw[:, 13], raw[:, 14], raw[:, 15]
ok = (ent > 0) & (st > 0) & (en > 0)
ent, st, en = ent[ok], st[ok], en[ok]
t0 = ent.min()
ent, st, en = (ent - t0) / 100.0, (st - t0) / 100.0, (en - t0) / 100.0
span = en.max()
pro = st - ent
print(f"tiles {ok.sum()} span {span:.2f} us")
print(f"prologue (entry -> pixels landed) mean {pro.mean():.2f} p50 {np.median(pro):.2f} p90 {np.percentile(pro, 90):.2f} us")
life = en - ent
print(f"lifetime from entry mean {life.mean():.2f} p50 {np.median(life):.2f}; tile work {np.mean(en - st):.2f} us")
T = np.arange(0.0, span, 5.0)
occ = [int(((ent <= v) & (en > v)).sum()) for v in T]
wrk = [int(((st <= v) & (en > v)).sum()) for v in T]
print("t(us) resident working")
for v, o, w in zip(T, occ, wrk):
    print(f"{v:6.1f} {o:6d} {w:6d}")
# refill gap: on each CU-slot a tile's entry follows some earlier tile's end; the gap from the
# nearest earlier end (any tile) is a lower bound of the dispatch delay
ends = np.sort(en)
sel = ent > 5.0
idx = np.searchsorted(ends, ent[sel]) - 1
gap = ent[sel] - ends[np.clip(idx, 0, None)]
w = raw[ok].reshape(-1, 4, 16)
e4, l4 = w[:, :, 13], w[:, :, 12]
skew = (e4.max(axis=1) - e4.min(axis=1)) / 100.0
lat = (l4 - e4) / 100.0
bar = (w[:, 0, 11] - l4.max(axis=1)) / 100.0
top = (w[:, 0, 14] - w[:, 0, 11]) / 100.0
print(f"wave entry skew in a workgroup mean {skew.mean():.2f} p90 {np.percentile(skew, 90):.2f} us; "
      f"entry -> own loads landed mean {lat.mean():.2f} (wave0 {lat[:, 0].mean():.2f}, wave3 {lat[:, 3].mean():.2f}) "
      f"p90 {np.percentile(lat, 90):.2f} us; last landed -> past the barrier {bar.mean():.2f} us, "
      f"-> tile start {top.mean():.2f} us")
if "--issue" in sys.argv:  # an IE_PROFILE=2 build: word 1 = the chip clock when the pixel DMA was issued
    iss = (w[:, :, 1] - e4) / 100.0
    print(f"entry -> pixel DMA issued mean {iss.mean():.2f} p90 {np.percentile(iss, 90):.2f} us")
print(f"entries after the first round: {sel.sum()}, gap from the latest earlier end mean {gap.mean():.3f} us")
