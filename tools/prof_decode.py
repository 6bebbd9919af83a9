"""Decode timing per content kind (4K, device-resident stream and pixels): the speculative parse,
or the exact table parse with IE_DEC_SPEC=0 (IE_DEC_R in the environment sets the records per chunk).
usage: python tools/prof_decode.py [n] [kind,kind...]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from imageencoder_amd import Codec, stream_bound, synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
w, h = 3840, 2160
q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
c = Codec(0, q, n)
yy, xx = np.mgrid[0:h, 0:w]
kinds = {"G": synth.frame("U", w, h, synth.DEFAULT_SEED),  # the bench's image 0 (the golden synU4k frame)
         "U": synth.frame("U", w, h, 5), "M": synth.frame("M", w, h, 5),
         "grad": ((xx * 3 + yy * 5) % 256).astype(np.uint8), "flat": np.full((h, w), 77, np.uint8)}
# the reference's example images (natural content; README.md:175-183 sizes)
for name, (ew, eh) in {"ex1": (936, 936), "ex2": (512, 512), "ex3": (400, 400), "ex4": (4096, 912)}.items():
    f = os.path.join(O.ROOT, "tests", "golden", name + ".raw")
    if os.path.exists(f):
        kinds[name] = np.fromfile(f, dtype=np.uint8)[: ew * eh].reshape(eh, ew)
tag = "R=" + os.environ.get("IE_DEC_R", "dflt")
hdr = int(os.environ.get("IE_HDR_BITS", "0"))  # a settings header of this many bits before the records (bench.py: 165 / 549)
tag += f" hdr={hdr}"
only = sys.argv[2].split(",") if len(sys.argv) > 2 else list(kinds)
for name, y in kinds.items():
    if name not in only:
        continue
    h, w = y.shape
    out = torch.zeros(stream_bound(w, h, n, 1, hdr), dtype=torch.uint8, device="cuda")
    pix = torch.empty((h, w), dtype=torch.uint8, device="cuda")
    _, end = c.encode_frames(torch.from_numpy(y).cuda(), w, h, out, start_bit=hdr)
    nb = (end + 7) // 8
    c.decode_frames(out[:nb], w, h, pix, length=nb, start_bit=hdr)
    ok = torch.equal(pix.cpu(), torch.from_numpy(y)) or True  # lossy: no pixel identity expected
    chunks, groups = c.last_decode_info()
    spec = c.last_decode_spec()
    torch.cuda.synchronize()
    k = 5
    t0 = time.perf_counter()
    for _ in range(k):
        c.decode_frames(out[:nb], w, h, pix, length=nb, start_bit=hdr)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / k
    print(f"{tag:12s} n={n} {name:5s} {nb:9d} B  {t * 1e6:9.1f} us  chunks={chunks} groups={groups} spec={int(spec)}", flush=True)
