"""Host overhead of one record decode call (profiling build prints its own phase times at exit):
wall per call against a no-op C-ABI call and an idle stream sync.
usage: IE_LIB=imageencoder_amd/lib/var_prof/libie_hip.so python tools/dec_host.py"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from imageencoder_amd import Codec, stream_bound, synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

w, h, n = 3840, 2160, 4
c = Codec(0, O.read_matrix("matrix.txt", n), n)
out = torch.zeros(stream_bound(w, h, n, 1, 0), dtype=torch.uint8, device="cuda")
pix = torch.empty((h, w), dtype=torch.uint8, device="cuda")
_, end = c.encode_frames(torch.from_numpy(synth.frame("U", w, h, 5)).cuda(), w, h, out)
nb = (end + 7) // 8
one = out[:nb]
for _ in range(5):
    c.decode_frames(one, w, h, pix, length=nb)
torch.cuda.synchronize()
k = 50
t0 = time.perf_counter()
for _ in range(k):
    c.decode_frames(one, w, h, pix, length=nb)
t1 = time.perf_counter()
for _ in range(k):
    c.last_decode_info()
t2 = time.perf_counter()
for _ in range(k):
    c.sync()
t3 = time.perf_counter()
print(f"decode call {1e6 * (t1 - t0) / k:.1f} us, no-op C-ABI call {1e6 * (t2 - t1) / k:.2f} us, "
      f"idle codec sync {1e6 * (t3 - t2) / k:.2f} us", flush=True)
