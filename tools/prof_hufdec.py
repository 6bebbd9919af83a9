"""Huffman-decode one 4K image's Huffman pass output (~6.5 MB) repeatedly and print the time per
call (IE_HUF_CHUNK tunes the walk chunk)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
assert dec[: payload.numel()] == payload.cpu().numpy().tobytes()
k = 10
t0 = time.perf_counter()
for _ in range(k):
    codec.huffman_decode(enc)
print(f"huffman decode {(time.perf_counter() - t0) / k * 1e6:.1f} us for {len(enc)} bytes")
