"""Streamed host path timing: ie_encode_images from host buffers (pageable numpy / pinned
ie_host_alloc), 16 x 4K frames, for a few chunk sizes (IE_CHUNK_MB).  usage: python tools/e2e.py [MB ...]
(E2E_N=8 in the environment: 8x8 blocks with matrix8_1.txt)"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from imageencoder_amd import Codec, stream_bound, synth, write_header  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

w, h, B = 3840, 2160, 16
n = int(os.environ.get("E2E_N", "4"))
q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
c = Codec(0, q, n)
if os.environ.get("E2E_TORCH_STREAM"):  # the bench's setting: kernels on a torch stream
    import torch
    _big = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    _st = torch.cuda.Stream()
    torch.cuda.set_stream(_st)
    c.set_stream(_st.cuda_stream)
hdr, hb = write_header(n, q, True, w, h)
pitch = (stream_bound(w, h, n, 1, hb) + 255) // 256 * 256
fr = synth.frames("U", w, h, B, seed=3).ravel()
bufs = {"pageable": (fr, np.zeros(pitch * B, dtype=np.uint8))}
yp, op = c.host_array(fr.size), c.host_array(pitch * B)
yp[:] = fr
bufs["pinned"] = (yp, op)
ref = None
for mb in sys.argv[1:] or ["4", "8", "16", "32"]:
    os.environ["IE_CHUNK_MB"] = mb
    for kind, (y, o) in bufs.items():
        o[:] = 0
        o.reshape(B, pitch)[:, : hdr.size] = hdr
        ends = c.encode_images(y, w, h, o, pitch, B, start_bit=hb)
        if ref is None:
            ref = o.copy()
        same = bool(np.array_equal(o, ref))
        t0 = time.perf_counter()
        for _ in range(5):
            c.encode_images(y, w, h, o, pitch, B, start_bit=hb)
        t = (time.perf_counter() - t0) / 5
        print(f"chunk {mb:>3} MiB {kind:8s} {t * 1e3:7.2f} ms  same={same}", flush=True)
