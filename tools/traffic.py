"""HBM traffic per launch of the dominant kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).

FETCH_SIZE / WRITE_SIZE are reported in KiB.  MI355X_MICROARCH.md (HBM [CDNA4]): on gfx950
FETCH_SIZE counts exactly half the bytes of wide (16 B/lane) coalesced streaming reads -- the
encoder's pixel loads are 16 B/lane (4x4 blocks) -- so it is doubled; WRITE_SIZE is exact for
16 B/lane stores.  Usage:
    python tools/traffic.py KERNEL_SUBSTR fetch_counter_collection.csv write_counter_collection.csv OUT.json [GRID]
GRID (optional): only dispatches of that Grid_Size (threads), e.g. the 16-frame sub-batch launches of
c4 beside its 64-frame ones.
"""
import csv
import json
import sys


def mean_counter(path, kernel, counter, grid=None):
    vals = {}
    for r in csv.DictReader(open(path)):
        if grid is not None and int(float(r.get("Grid_Size", 0))) != grid:
            continue
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            key = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(vals))
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    v = sorted(vals.values())
    # drop the smallest launches (warm-up / sizing launches with fewer frames) if sizes differ
    top = [x for x in v if x >= 0.5 * v[-1]]
    return sum(top) / len(top), len(top)


def main():
    kernel, fcsv, wcsv, out = sys.argv[1:5]
    grid = int(sys.argv[5]) if len(sys.argv) > 5 else None
    f_kib, nf = mean_counter(fcsv, kernel, "FETCH_SIZE", grid)
    w_kib, nw = mean_counter(wcsv, kernel, "WRITE_SIZE", grid)
    fetch = 2.0 * f_kib * 1024.0
    write = w_kib * 1024.0
    res = {
        "kernel": kernel,
        "fetch_size_kib_raw": f_kib,
        "write_size_kib": w_kib,
        "hbm_read_bytes_per_launch": int(fetch),
        "hbm_write_bytes_per_launch": int(write),
        "hbm_bytes_per_launch": int(fetch + write),
        "launches_averaged": [nf, nw],
        "grid_size": grid,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (--kernel-trace only); "
                  "FETCH_SIZE x2 per the gfx950 correction for 16 B/lane streaming reads",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
