import sys, os, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from imageencoder_amd import Codec, stream_bound, synth, MODE_FAST, MODE_EXACT
from tests import oracle_lib as O
mode = MODE_EXACT if len(sys.argv) > 1 and sys.argv[1] == "exact" else MODE_FAST
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 4
N = int(os.environ.get("IE_N", "4"))
q = O.read_matrix("matrix.txt" if N == 4 else "matrix8_1.txt", N)
c = Codec(0, q, N)
w, h = 3840, 2160
y = torch.from_numpy(synth.frames("U", w, h, nf, seed=3)).cuda()
pitch = (stream_bound(w, h, N, 1, 165) + 255)//256*256
out = torch.zeros(pitch*nf, dtype=torch.uint8, device="cuda")
for i in range(3):
    c.encode_images(y, w, h, out, out_pitch=pitch, nframes=nf, start_bit=165, mode=mode)
torch.cuda.synchronize()
t0=time.perf_counter()
for i in range(5):
    c.encode_images(y, w, h, out, out_pitch=pitch, nframes=nf, start_bit=165, mode=mode, want_sizes=False)
c.sync()
print("mode", mode, "nf", nf, "us/launch", (time.perf_counter()-t0)/5*1e6)
