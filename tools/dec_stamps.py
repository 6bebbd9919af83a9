"""Per-wave phase times of the record parse's table pass (profiling build: IE_LIB=.../var_prof,
IE_DEC_STAMPS=file).  Decodes one 4K frame of the given content, then summarises the stamps of the
LAST call: phase durations, walk iterations, concurrency over time.
usage: python tools/dec_stamps.py [n] [kind] [out.bin]"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
kind = sys.argv[2] if len(sys.argv) > 2 else "U"
path = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/dec_stamps.bin"
if os.environ.get("IE_DEC_STAMPS") != path:
    raise SystemExit("run with IE_DEC_STAMPS=" + path + " and IE_LIB=<profiling build>")
if os.path.exists(path):
    os.remove(path)
import torch  # noqa: E402

from imageencoder_amd import Codec, stream_bound, synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

w, h = 3840, 2160
q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
c = Codec(0, q, n)
y = (synth.frame("U", w, h, synth.DEFAULT_SEED) if kind == "G"  # the bench's image 0
     else synth.frame(kind, w, h, 5) if kind in ("U", "M") else np.full((h, w), 77, np.uint8))
out = torch.zeros(stream_bound(w, h, n, 1, 0), dtype=torch.uint8, device="cuda")
pix = torch.empty((h, w), dtype=torch.uint8, device="cuda")
_, end = c.encode_frames(torch.from_numpy(y).cuda(), w, h, out)
nb = (end + 7) // 8
for _ in range(2):
    c.decode_frames(out[:nb], w, h, pix, length=nb)
torch.cuda.synchronize()
os.remove(path)  # keep the last call's stamps only
c.decode_frames(out[:nb], w, h, pix, length=nb)
torch.cuda.synchronize()
chunks, _ = c.last_decode_info()
st = np.fromfile(path, dtype=np.uint64).astype(np.int64).reshape(-1, 8)
st = st[st[:, 0] > 0]
t = st[:, :6].astype(np.float64) * 0.01  # realtime ticks (100 MHz) -> us
t -= t[:, 0].min()
names = ["init", "bitmap", "walklist", "walks", "resolve+store"]
print(f"waves {len(st)} chunks {chunks}  launch span {t[:, 5].max() - t[:, 0].min():.1f} us")
for i, nm in enumerate(names):
    d = t[:, i + 1] - t[:, i]
    print(f"{nm:8s} mean {d.mean():7.2f} us  p50 {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f}")
life = t[:, 5] - t[:, 0]
print(f"wave life mean {life.mean():.2f} us  p50 {np.median(life):.2f}  p90 {np.percentile(life, 90):.2f}")
it = st[:, 6]
mx, sm = it >> 32, it & 0xFFFFFFFF
tmc = max(1, round(chunks / len(st)))
print(f"walk iterations per wave: max-lane mean {mx.mean():.1f} p90 {np.percentile(mx, 90):.0f} max {mx.max()}; "
      f"lane-steps per chunk {sm.mean() / tmc:.1f}")
# concurrency: waves alive at 200 sample times
ts = np.linspace(0, t[:, 5].max(), 200)
alive = [(np.sum((t[:, 0] <= x) & (t[:, 5] > x))) for x in ts]
print("alive waves over the launch (every 10th sample):", [int(a) for a in alive[::10]])
nwk, rst = st[:, 7] >> 32, st[:, 7] & 0xFFFFFFFF
print(f"per chunk: walks {nwk.mean() / tmc:.1f}, steps of walks that left the chunk {rst.mean() / tmc:.1f}, "
      f"steps of merged walks {(sm.mean() - rst.mean()) / tmc:.1f}")
first = t[:, 0]
print(f"wave start times: p10 {np.percentile(first, 10):.1f} p50 {np.median(first):.1f} p90 {np.percentile(first, 90):.1f} "
      f"max {first.max():.1f} us")
