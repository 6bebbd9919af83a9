#!/usr/bin/env python3
"""Per-(kernel, grid) durations and dispatch gaps from a rocprofv3 kernel trace CSV.

usage: trace_grid.py <kernel_trace.csv> [kernel-substring]

For every kernel name (matching the substring) and grid size: dispatches, mean / median / min
duration (us), and the median gap between the end of one dispatch and the start of the next
dispatch of the same kernel and grid -- a gap near zero means back-to-back launches are
GPU-bound, a large one that the host (or something else on the stream) sets the pace.
"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            if sub and sub not in name:
                continue
            grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
            rows[(name[:60], grid)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for (name, grid), ev in sorted(rows.items(), key=lambda kv: -len(kv[1])):
        ev.sort()
        d = [(e - s) / 1e3 for s, e in ev]
        gaps = [(ev[i + 1][0] - ev[i][1]) / 1e3 for i in range(len(ev) - 1)]
        gm = statistics.median(gaps) if gaps else float("nan")
        print(f"{name:60s} grid {grid:9d} n {len(d):5d}  mean {statistics.mean(d):8.2f}  "
              f"median {statistics.median(d):8.2f}  min {min(d):8.2f} us  gap median {gm:8.2f} us")


if __name__ == "__main__":
    main()
