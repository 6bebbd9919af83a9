"""Huffman decode of one 4K image's Huffman-coded payload (~6.5 MB): (a) host bytes -> host bytes
through the host library (dictionary + table on the host, walk on the device), (b) device-resident
(stream, table and output in HBM; ie_huffman_decode).  usage: python tools/prof_hufdec.py"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from imageencoder_amd import Codec, stream_bound, synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

q = O.read_matrix("matrix.txt", 4)
w, h = 3840, 2160
codec = Codec(0, q, 4)
y = torch.from_numpy(synth.frame("U", w, h, 9)).cuda()
out = torch.zeros(stream_bound(w, h, 4, 1, 0), dtype=torch.uint8, device="cuda")
_, end = codec.encode_frames(y, w, h, out, start_bit=0)
payload = out[: (end + 7) // 8]
enc = codec.huffman_encode(payload)
dec, _ = codec.huffman_decode(enc)
ref = payload.cpu().numpy().tobytes()
assert dec[: len(ref)] == ref
k = 10
t0 = time.perf_counter()
for _ in range(k):
    codec.huffman_decode(enc)
th = (time.perf_counter() - t0) / k
lut, sb = codec.huffman_table(enc)
denc = torch.from_numpy(np.frombuffer(enc, np.uint8).copy()).cuda()
dlut = torch.from_numpy(lut.view(np.int16).copy()).cuda()
dout = torch.zeros(len(dec) + 16, dtype=torch.uint8, device="cuda")
nsym = codec.huffman_decode_device(denc, len(enc), dlut, sb, dout)
assert nsym == len(dec) and dout[:nsym].cpu().numpy().tobytes() == dec
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(k):
    codec.huffman_decode_device(denc, len(enc), dlut, sb, dout)
torch.cuda.synchronize()
td = (time.perf_counter() - t0) / k
print(f"huffman decode of {len(enc)} bytes -> {nsym} symbols: host->host {th * 1e3:.2f} ms, "
      f"device-resident {td * 1e3:.3f} ms", flush=True)
