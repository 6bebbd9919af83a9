"""Raw PCIe copy rates between pinned host memory and HBM: H2D alone, D2H alone, both at once on
two streams (what the streamed host path can reach).  usage: python tools/pcie.py [MiB]"""
import sys
import time

import torch

n = int(float(sys.argv[1]) if len(sys.argv) > 1 else 128) << 20
h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
h_out = torch.empty(n, dtype=torch.uint8).pin_memory()
d_a = torch.empty(n, dtype=torch.uint8, device="cuda")
d_b = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def run(h2d, d2h, reps=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        if h2d:
            with torch.cuda.stream(s1):
                d_a.copy_(h_in, non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                h_out.copy_(d_b, non_blocking=True)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


run(True, True, 2)
for name, a, b in (("H2D", True, False), ("D2H", False, True), ("both", True, True)):
    t = run(a, b)
    gb = n * (int(a) + int(b)) / t / 1e9
    print(f"{name:5s} {n >> 20} MiB each: {t * 1e3:7.2f} ms  {gb:6.1f} GB/s total", flush=True)
