"""Time the pieces of the c5 step (encode with size read-back, batched Huffman) on the GPU."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time

import numpy as np
import torch

from imageencoder_amd import Codec, synth, write_header, stream_bound
from tests import oracle_lib as O

w, h, n, B = 3840, 2160, 4, 16
q = O.read_matrix("matrix.txt", 4)
codec = Codec(0, q, n)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
codec.set_stream(s.cuda_stream)
frames = torch.empty((B, h, w), dtype=torch.uint8, device="cuda")
for i in range(B):
    frames[i].copy_(torch.from_numpy(synth.frame("U", w, h, 7 + i)))
hb = write_header(n, q, True, w, h, huffman=True)[1]
pitch = (stream_bound(w, h, n, 1, hb) + 255) // 256 * 256
out = torch.zeros(pitch * B, dtype=torch.uint8, device="cuda")
hpitch = 2 * pitch
hout = torch.zeros(hpitch * B, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()


def t(f, k=10):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


ends = codec.encode_images(frames, w, h, out, out_pitch=pitch, nframes=B, start_bit=hb)
sizes = [(int(e) + 7) // 8 for e in ends]
print("encode+sizes ms", t(lambda: codec.encode_images(frames, w, h, out, out_pitch=pitch, nframes=B, start_bit=hb)))
print("encode async ms", t(lambda: codec.encode_images(frames, w, h, out, out_pitch=pitch, nframes=B, start_bit=hb,
                                                       want_sizes=False)))
hist = np.zeros(B * 256, np.uint32)
first = np.zeros(B * 256, np.uint64)
nn = np.asarray(sizes, np.uint64)
import ctypes as C
L = codec.L
u64 = C.POINTER(C.c_uint64)
args = (codec.h, C.cast(out.data_ptr(), C.POINTER(C.c_uint8)), pitch, nn.ctypes.data_as(u64), B,
        hist.ctypes.data_as(C.POINTER(C.c_uint32)), first.ctypes.data_as(u64))
print("hist batch ms", t(lambda: L.ie_huffman_hist_batch(*args)))
print("huffman batch ms", t(lambda: codec.huffman_encode_batch(out, pitch, sizes, hout, hpitch)))
