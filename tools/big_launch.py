"""One ie_encode_frames launch over F 1920x1080 uniform-noise frames (default 512: the C4 test's
single-launch reference), repeated REPS times: wall time per launch and the stream's md5.
IE_FORCE_TICKET=1 orders tiles by ticket; IE_LIB picks a library build."""
import hashlib
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from imageencoder_amd import Codec, stream_bound, synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

w, h, n = 1920, 1080, 4
F = int(os.environ.get("F", "512"))
reps = int(os.environ.get("REPS", "3"))
c = Codec(0, O.read_matrix("matrix.txt", n), n)
y = synth.uniform_device(w, h, F, synth.DEFAULT_SEED + 4242, "cuda", torch)
out = torch.zeros(stream_bound(w, h, n, F, 165) + 64, dtype=torch.uint8, device="cuda")
for r in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, end = c.encode_frames(y, w, h, out, start_bit=165, nframes=F)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    md5 = hashlib.md5(out[: (end + 7) // 8].cpu().numpy().tobytes()).hexdigest()
    print(f"F {F} rep {r}: {dt * 1e3:.2f} ms end {end} md5 {md5}", flush=True)
