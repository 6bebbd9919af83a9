"""Decode one 4K image (4x4 or 8x8, IE_N env) repeatedly: rocprofv3 --kernel-trace --stats target
for the inverse path's kernels."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from imageencoder_amd import Codec, stream_bound, synth, write_header  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

n = int(os.environ.get("IE_N", "4"))
q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
w, h = 3840, 2160
codec = Codec(0, q, n)
hb = write_header(n, q, True, w, h)[1]
y = torch.from_numpy(synth.frame("U", w, h, 9)).cuda()
out = torch.zeros(stream_bound(w, h, n, 1, hb), dtype=torch.uint8, device="cuda")
_, end = codec.encode_frames(y, w, h, out, start_bit=hb)
nb = (end + 7) // 8
pix = torch.empty((h, w), dtype=torch.uint8, device="cuda")
codec.decode_frames(out[:nb], w, h, pix, start_bit=hb, length=nb)
torch.cuda.synchronize()
k = 20
t0 = time.perf_counter()
for _ in range(k):
    codec.decode_frames(out[:nb], w, h, pix, start_bit=hb, length=nb)
torch.cuda.synchronize()
print(f"n={n} decode {(time.perf_counter() - t0) / k * 1e6:.1f} us per 4K image")
