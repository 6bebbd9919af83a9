import os, sys, subprocess, json
sys.path.insert(0, "/root/repo")
import numpy as np
from imageencoder_amd import Codec
from tests import oracle_lib as O
names = sys.argv[1:] or ["ex0_4x4"]
c = Codec(0)
for name in names:
    case = next(x for x in O.manifest() if x["name"] == name)
    enc = O.case_expected(case)
    pix = c.decode_image_file(enc, case["n"])
    ref = O.load().decode_image(enc, case["n"])
    print(name, c.last_decode_info(), "equal", np.array_equal(pix, ref))
    if not np.array_equal(pix, ref):
        n = case["n"]
        d = (pix != ref)
        bad = sorted({(int(i)//n, int(j)//n) for i, j in zip(*np.nonzero(d))})
        print("bad blocks", bad[:20], "of", (case["h"]//n)*(case["w"]//n))
        print(pix[:8, :16]); print(ref[:8, :16])
