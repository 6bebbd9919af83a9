"""Kernel timeline of a rocprofv3 --kernel-trace run: the last N dispatches in start order with
their duration and the idle gap before each (the device had no kernel of this process running),
then the mean duration / gap per kernel name over the steady state (the last third of the run).

usage: python tools/trace_gaps.py run_kernel_trace.csv [N]
"""
import collections
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48]))
rows.sort()
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
busy_end = 0
out = []
for s, e, k in rows:
    gap = max(0, s - busy_end) if busy_end else 0
    out.append((s, e, k, gap))
    busy_end = max(busy_end, e)
t0 = out[-n][0]
for s, e, k, gap in out[-n:]:
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.2f}  gap {gap / 1e3:7.2f}  {k}")
tail = out[len(out) * 2 // 3:]
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for s, e, k, gap in tail:
    a = agg[k]
    a[0] += 1
    a[1] += (e - s) / 1e3
    a[2] += gap / 1e3
span = (tail[-1][1] - tail[0][0]) / 1e3
print(f"steady state: {len(tail)} dispatches over {span:.1f} us, idle {sum(g for *_, g in tail) / 1e3:.1f} us")
for k, (c, d, g) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {k:48s} n={c:4d} mean dur {d / c:8.2f} us  mean gap before {g / c:6.2f} us")
