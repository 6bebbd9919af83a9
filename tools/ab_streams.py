"""Does splitting a batch over concurrent launches fill the launch's ramp and tail?  One 16-frame
ie_encode_images launch against K launches of 16/K frames on K contexts / K HIP streams issued
back to back (independent images: the same streams either way), HIP-event timed around each,
medians over rounds.  usage: python tools/ab_streams.py [frames] [K...]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from imageencoder_amd import synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

nf = int(sys.argv[1]) if len(sys.argv) > 1 else 16
Ks = [int(k) for k in sys.argv[2:]] or [2, 4]
w, h = 3840, 2160
q = np.ascontiguousarray(np.asarray(O.read_matrix("matrix.txt", 4), dtype=np.uint16).ravel())
y = synth.uniform_device(w, h, nf, 3, "cuda", torch)
L = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "imageencoder_amd", "lib", "libie_hip.so"))
vp = C.c_void_p
L.ie_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
L.ie_set_stream.argtypes = [vp, vp]
L.ie_set_quant.argtypes = [vp, vp, C.c_int]
L.ie_stream_bound.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64]
L.ie_stream_bound.restype = C.c_size_t
L.ie_encode_images.argtypes = [vp, vp, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int,
                               vp, C.c_size_t, C.c_uint64, C.POINTER(C.c_uint64)]
pitch = (int(L.ie_stream_bound(w, h, 4, 1, 165)) + 255) // 256 * 256
out = torch.zeros(pitch * nf, dtype=torch.uint8, device="cuda")
kmax = max(Ks)
streams = [torch.cuda.Stream() for _ in range(kmax)]
ctxs = []
for i in range(kmax):
    hnd = C.c_void_p()
    assert L.ie_create(0, C.byref(hnd)) == 0
    assert L.ie_set_stream(hnd, C.c_void_p(streams[i].cuda_stream)) == 0
    assert L.ie_set_quant(hnd, q.ctypes.data, 4) == 0
    ctxs.append(hnd)


def launch(i, f0, m):
    r = L.ie_encode_images(ctxs[i], C.c_void_p(y[f0:].data_ptr()), w, h, w, w * h, m, 1, 0,
                           C.c_void_p(out[f0 * pitch:].data_ptr()), pitch, 165, None)
    assert r == 0


def run(K):
    m = nf // K
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream()
    ev0.record(cur)
    for i in range(K):
        streams[i].wait_stream(cur)
    for i in range(K):
        launch(i, i * m, m)
    for i in range(K):
        cur.wait_stream(streams[i])
    ev1.record(cur)
    ev1.synchronize()
    return ev0.elapsed_time(ev1) * 1000.0


res = {k: [] for k in [1] + Ks}
for _ in range(3):
    for k in res:
        run(k)
for r in range(15):
    for k in res:
        res[k].append(run(k))
for k, t in res.items():
    print(f"K={k}: {nf // k} frames x {k} launches on {k} streams: median {np.median(t):.2f} us  min {np.min(t):.2f}")
