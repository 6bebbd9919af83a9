"""One C2-shaped launch (NF 4K uniform-noise frames, default 16) with IE_STAMPS set (run with IE_LIB = an
IE_PROFILE build): writes the per-tile stamps file named by IE_STAMPS.  SHAPE=c4: NF 1080p frames
(default 64) as ONE concatenated stream (ie_encode_frames: the C4 per-rank launch, one chain)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from imageencoder_amd import Codec, stream_bound, synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

c4 = os.environ.get("SHAPE") == "c4"
w, h, nf = (1920, 1080, int(os.environ.get("NF", "64"))) if c4 else (3840, 2160, int(os.environ.get("NF", "16")))
c = Codec(0, O.read_matrix("matrix.txt", 4), 4)
y = synth.uniform_device(w, h, nf, 3, "cuda", torch)
pitch = (stream_bound(w, h, 4, 1, 165) + 255) // 256 * 256
out = torch.zeros(pitch * nf, dtype=torch.uint8, device="cuda")
for _ in range(3):
    if c4:
        c.encode_frames(y, w, h, out, start_bit=210, nframes=nf)
    else:
        c.encode_images(y, w, h, out, out_pitch=pitch, nframes=nf, start_bit=165)
torch.cuda.synchronize()
print("stamps written to", os.environ.get("IE_STAMPS"))
