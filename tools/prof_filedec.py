"""Whole-file decode timing (ImageDecoder: Huffman decode, then the record decode) for 4K images of
several content kinds, Huffman on and off.  usage: python tools/prof_filedec.py [n]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from imageencoder_amd import Codec, synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
w, h = 3840, 2160
q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
c = Codec(0, q, n)
yy, xx = np.mgrid[0:h, 0:w]
kinds = {"U": synth.frame("U", w, h, 5), "grad": ((xx * 3 + yy * 5) % 256).astype(np.uint8),
         "flat": np.full((h, w), 77, np.uint8)}
for name, y in kinds.items():
    for huff in (False, True):
        enc = c.encode_image_file(y, w, h, q, n, rle=True, huffman=huff)
        pix = c.decode_image_file(enc, n)
        k = 3
        t0 = time.perf_counter()
        for _ in range(k):
            c.decode_image_file(enc, n)
        t = (time.perf_counter() - t0) / k
        print(f"n={n} {name:5s} huffman={int(huff)} {len(enc):9d} B  {t * 1e3:8.2f} ms", flush=True)
