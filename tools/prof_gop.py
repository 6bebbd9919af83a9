"""P-frame video timing (ie_encode_gop, device-resident frames and stream): a panning video whose
frames a motion search can follow, gop = 1 (I-frames only) against gop = F (one I-frame, F-1
P-frames); per-frame time of the P-frames = (t_gop - t_I / F) / (F - 1).  Also times the
reference's own encoder binary on a small sample when oracle/_ref is present (CPU baseline).
usage: python tools/prof_gop.py [w h frames merange]"""
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from imageencoder_amd import Codec, synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

w, h, F, mer = (int(a) for a in sys.argv[1:5]) if len(sys.argv) > 4 else (1920, 1080, 16, 16)
q = O.read_matrix("matrix.txt", 4)
c = Codec(0, q, 4)
y = synth.frames("P", w, h, F, synth.DEFAULT_SEED + 7)
dy = torch.from_numpy(y).cuda()
cap = c.gop_stream_bound(w, h, F, mer, 0)
out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
res = {}
for gop in (1, F):
    fb, end = c.encode_gop(dy, w, h, out, gop, mer, nframes=F)  # warm-up (and allocations)
    k = 10
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        out.zero_()
        c.encode_gop(dy, w, h, out, gop, mer, nframes=F)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / k
    res[gop] = (t, int(end), [int(v) for v in fb])
# decode (ie_decode_gop, device-resident stream and frames) of both streams
dec_t = {}
dout = torch.zeros(F * h * w, dtype=torch.uint8, device="cuda")
for gop in ((1, F) if w % 16 == 0 and h % 16 == 0 else ()):  # (P-frames decode at multiples of 16 only)
    _, end = c.encode_gop(dy, w, h, out, gop, mer, nframes=F)
    nb = (int(end) + 7) // 8
    c.decode_gop(out, w, h, dout, gop, mer, nframes=F, length=nb)  # warm-up
    torch.cuda.synchronize()
    k = 10
    t0 = time.perf_counter()
    for _ in range(k):
        c.decode_gop(out, w, h, dout, gop, mer, nframes=F, length=nb)
    torch.cuda.synchronize()
    dec_t[gop] = (time.perf_counter() - t0) / k
if dec_t:
    print(f"decode_gop {w}x{h} x{F}: gop=1 {dec_t[1] * 1e3:.3f} ms ({dec_t[1] / F * 1e6:.1f} us/frame), "
          f"gop={F} {dec_t[F] * 1e3:.3f} ms ({dec_t[F] / F * 1e6:.1f} us/frame)")
# the stream zeroing is part of each timed call above; time it alone to subtract it
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    out.zero_()
torch.cuda.synchronize()
tz = (time.perf_counter() - t0) / 10
tI, tG = res[1][0] - tz, res[F][0] - tz
p_frame = (tG - tI / F) / (F - 1)
px = w * h
print(f"{w}x{h} x{F} merange={mer}: gop=1 {tI * 1e3:.3f} ms ({tI / F * 1e6:.1f} us/frame), "
      f"gop={F} {tG * 1e3:.3f} ms -> P-frame {p_frame * 1e6:.1f} us ({px / p_frame / 1e6:.0f} Mpx/s); "
      f"bits I-only {res[1][1]} / gop {res[F][1]} (P-frame payload {np.mean(res[F][2][1:]):.0f} bits)")

# reference CPU baseline: its own encoder binary (OpenMP) on a 4-frame sample, whole-program time
ref = os.path.join(ROOT, "oracle", "_ref", "encoder")
if os.path.exists(ref) and not os.environ.get("IE_NO_REF"):
    Fs = 4
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "in.raw"), "wb").write(synth.yuv420(y[:Fs]))
        open(os.path.join(d, "m.txt"), "w").write(open(os.path.join(ROOT, "tests", "golden", "matrix.txt")).read())
        for gop in (1, Fs):
            keys = dict(rawfile="in.raw", encfile="out.enc", decfile="out.dec", width=w, height=h, rle=1,
                        quantfile="m.txt", logfile="", gop=gop, merange=mer)
            open(os.path.join(d, "c.conf"), "w").write("".join(f"{k}={v}\n" for k, v in keys.items()))
            t0 = time.perf_counter()
            subprocess.run([ref, "c.conf"], cwd=d, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            t = time.perf_counter() - t0
            print(f"reference encoder (OpenMP, whole program) {w}x{h} x{Fs} gop={gop}: {t * 1e3:.0f} ms "
                  f"({Fs * px / t / 1e6:.1f} Mpx/s)")
