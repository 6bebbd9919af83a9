"""FAST == EXACT fuzz on the GPU: the FP32 fast path with
its FP64 near-tie re-evaluation must produce exactly the stream of the all-FP64 EXACT path (the
reference's operation order) on every block.  Batches of 4K frames from several generators --
uniform noise, low-amplitude noise around a random level (many structural ties), random
gradients, checkerboards of two levels -- are encoded both ways on the device and the streams
compared with torch.equal; any difference is reported with its frame.  A time budget bounds the
run; the summary (blocks compared, mismatches, FP64 fix-up requests) goes to a JSON file.

usage: python tools/fuzz_exact.py --n 4 --blocks 1e9 --budget 600 --out profiles/r02_fuzz_4x4.json
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from imageencoder_amd import MODE_EXACT, MODE_FAST, Codec, stream_bound, synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4)
ap.add_argument("--blocks", type=float, default=1e9)
ap.add_argument("--budget", type=float, default=600.0, help="seconds")
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--out", default="")
args = ap.parse_args()

n, w, h, B = args.n, 3840, 2160, args.batch
q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
codec = Codec(0, q, n)
dev = "cuda"
pitch = (stream_bound(w, h, n, 1, 0) + 255) // 256 * 256
o_fast = torch.zeros(pitch * B, dtype=torch.uint8, device=dev)
o_exact = torch.zeros(pitch * B, dtype=torch.uint8, device=dev)
g = torch.Generator(device=dev)
blocks_per_frame = (w // n) * (h // n)
KINDS = ["uniform", "lownoise", "gradient", "checker"]


def make(kind: str, seed: int) -> torch.Tensor:
    g.manual_seed(seed)
    if kind == "uniform":
        return synth.uniform_device(w, h, B, seed, dev, torch)
    if kind == "lownoise":  # a random level per 64x64 tile, +-amp noise: flat-ish blocks, structural ties
        lvl = torch.randint(0, 256, (B, h // 64 + 1, w // 64 + 1), generator=g, device=dev)
        lvl = lvl.repeat_interleave(64, 1).repeat_interleave(64, 2)[:, :h, :w]
        amp = int(torch.randint(1, 6, (1,), generator=g, device=dev))
        noise = torch.randint(-amp, amp + 1, (B, h, w), generator=g, device=dev)
        return (lvl + noise).clamp(0, 255).to(torch.uint8)
    if kind == "gradient":
        yy = torch.arange(h, device=dev).view(1, h, 1).float()
        xx = torch.arange(w, device=dev).view(1, 1, w).float()
        a = torch.rand((B, 1, 1), generator=g, device=dev) * 4 - 2
        b = torch.rand((B, 1, 1), generator=g, device=dev) * 4 - 2
        c = torch.rand((B, 1, 1), generator=g, device=dev) * 255
        return torch.remainder(a * xx + b * yy + c, 256).to(torch.uint8)
    # checker: two random levels in a per-frame random period
    lo = torch.randint(0, 256, (B, 1, 1), generator=g, device=dev)
    hi = torch.randint(0, 256, (B, 1, 1), generator=g, device=dev)
    p = int(torch.randint(1, 9, (1,), generator=g, device=dev))
    yy = torch.arange(h, device=dev).view(1, h, 1) // p
    xx = torch.arange(w, device=dev).view(1, 1, w) // p
    return torch.where(((yy + xx) % 2) == 0, lo, hi).to(torch.uint8)


t0 = time.time()
done = mism = fix = 0
per_kind = {k: 0 for k in KINDS}
bad = []
it = 0
while done < args.blocks and time.time() - t0 < args.budget:
    kind = KINDS[it % len(KINDS)]
    y = make(kind, 1000 + it)
    ef = codec.encode_images(y, w, h, o_fast, pitch, B, mode=MODE_FAST)
    fix += codec.last_fallbacks()
    ee = codec.encode_images(y, w, h, o_exact, pitch, B, mode=MODE_EXACT)
    if list(ef) != list(ee) or not torch.equal(o_fast, o_exact):
        # locate the differing frames
        for f in range(B):
            nb = (int(max(ef[f], ee[f])) + 7) // 8
            a_, b_ = o_fast[f * pitch:f * pitch + nb], o_exact[f * pitch:f * pitch + nb]
            if ef[f] != ee[f] or not torch.equal(a_, b_):
                mism += 1
                diff = torch.nonzero(a_ != b_)
                first = int(diff[0]) if diff.numel() else -1
                bad.append({"kind": kind, "batch_seed": 1000 + it, "frame": f, "end_fast": int(ef[f]),
                            "end_exact": int(ee[f]), "first_diff_byte": first, "ndiff": int(diff.numel())})
    done += B * blocks_per_frame
    per_kind[kind] += B * blocks_per_frame
    it += 1
    if it % 10 == 0:
        print(f"{done:.3e} blocks, {mism} mismatching frames, {time.time() - t0:.0f} s", flush=True)
res = {"n": n, "blocks_compared": done, "target_blocks": args.blocks, "frames_mismatching": mism,
       "mismatches": bad[:20], "per_kind_blocks": per_kind, "fp64_fixup_requests_fast": fix,
       "seconds": round(time.time() - t0, 1), "complete": done >= args.blocks,
       "method": "4K frames, FAST (FP32 + FP64 near-tie) vs EXACT (all FP64, reference order) streams "
                 "compared byte for byte on the device"}
print(json.dumps(res), flush=True)
if args.out:
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
sys.exit(1 if mism else 0)
