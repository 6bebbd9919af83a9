"""Check one fuzz frame three ways: FAST, EXACT and the CPU oracle (usage: dbg_fuzz.py seed frame [n])."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from imageencoder_amd import MODE_EXACT, MODE_FAST, Codec, stream_bound, synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

seed, fr = int(sys.argv[1]), int(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 4
w, h, B = 3840, 2160, 16
q = O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n)
c = Codec(0, q, n)
y = synth.uniform_device(w, h, B, seed, "cuda", torch)
pitch = (stream_bound(w, h, n, 1, 0) + 255) // 256 * 256
res = {}
for name, mode, nf in (("fast16", MODE_FAST, B), ("exact16", MODE_EXACT, B), ("fast1", MODE_FAST, 1), ("exact1", MODE_EXACT, 1)):
    o = torch.zeros(pitch * nf, dtype=torch.uint8, device="cuda")
    src = y if nf == B else y[fr:fr + 1]
    e = c.encode_images(src, w, h, o, pitch, nf, mode=mode)
    k = fr if nf == B else 0
    res[name] = o[k * pitch: k * pitch + (int(e[k]) + 7) // 8].cpu().numpy().tobytes()
    print(name, int(e[k]), flush=True)
ref, end, _ = O.load().encode_blocks(y[fr].cpu().numpy(), n, q)
ref = ref[: (end + 7) // 8].tobytes()
print("oracle", end)
for k, v in res.items():
    d = next((i for i in range(min(len(v), len(ref))) if v[i] != ref[i]), None)
    print(k, "== oracle" if v == ref else f"differs at byte {d} (len {len(v)} vs {len(ref)})")
