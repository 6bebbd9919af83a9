"""Host time of each call of the pipelined C5 step (bench.py's order: counted encode, histogram
begin, finish of the previous batch), averaged over the steps after a warm-up, beside the step's
wall time: shows whether the device waits for the host between the step's launches."""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from imageencoder_amd import Codec, stream_bound, synth, write_header  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

w, h, n, B, steps = 3840, 2160, 4, 16, 12
q = O.read_matrix("matrix.txt", 4)
codec = Codec(0, q, n)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
codec.set_stream(s.cuda_stream)
frames = synth.uniform_device(w, h, B, 3, "cuda", torch)
hdr, hb = write_header(n, q, True, w, h, huffman=True)
pitch = (stream_bound(w, h, n, 1, hb) + 255) // 256 * 256
outs = [torch.zeros(pitch * B, dtype=torch.uint8, device="cuda") for _ in range(2)]
hpitch = 2 * pitch
houts = torch.zeros(hpitch * B, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
T = {"encode": [], "begin": [], "finish": [], "step": []}
pending = []
for i in range(steps):
    t0 = time.perf_counter()
    out = outs[i % 2]
    codec.encode_images(frames, w, h, out, out_pitch=pitch, nframes=B, start_bit=hb, want_sizes=False, count_bytes=True)
    t1 = time.perf_counter()
    codec.huffman_begin_after_encode(out, pitch, B, i % 2)
    t2 = time.perf_counter()
    if pending:
        o, sl = pending.pop()
        codec.huffman_finish_after_encode(o, pitch, B, sl, houts, hpitch)
    t3 = time.perf_counter()
    pending.append((out, i % 2))
    if i >= 4:
        T["encode"].append(t1 - t0)
        T["begin"].append(t2 - t1)
        T["finish"].append(t3 - t2)
        T["step"].append(t3 - t0)
torch.cuda.synchronize()
for k, v in T.items():
    print(f"{k:7s} host {np.mean(v) * 1e6:8.1f} us  (min {np.min(v) * 1e6:.1f})")
