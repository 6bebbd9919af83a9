"""INTEGRATION.md §B compiled and run: the reference's OWN encoder classes (built from
/root/reference by oracle/Makefile) with ImageEncoder.cpp's block loop replaced by one
ie_encode_frames call (integration/ImageEncoder_hip.cpp, compiled against the reference's
unmodified headers) must write files byte-identical to the reference encoder's.

The binaries are test infrastructure under oracle/_ref (built where the reference sources exist,
then shipped with the tree); the GPU tests only run them.
"""
import hashlib
import os
import subprocess

import pytest

from tests import oracle_lib as O

REF = os.path.join(O.ROOT, "oracle", "_ref")
HIP = {False: os.path.join(REF, "ref_harness_hip"), True: os.path.join(REF, "ref_harness_hip_huff")}


def _need(p):
    if not os.path.exists(p):
        pytest.skip(f"{os.path.relpath(p, O.ROOT)} not built (make ref, needs /root/reference)")
    return p


@pytest.mark.parametrize("huff", [False, True])
def test_dropin_links_the_gpu_library(huff):
    """The drop-in resolves its block loop from libie_hip.so (not from the reference's loop)."""
    exe = _need(HIP[huff])
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True, timeout=60).stdout
    assert "libie_hip.so" in ldd and "not found" not in ldd.split("libie_hip.so")[1].splitlines()[0]
    und = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, timeout=60).stdout
    for sym in ("ie_create", "ie_set_quant", "ie_encode_frames", "ie_stream_bound"):
        assert sym in und, sym


CASES = [c for c in O.manifest() if c["input"]["kind"] == "asset" and c["n"] == 4 and c["rle"] == 1
         and c["matrix"] == "matrix.txt" and not c["video"]]


@pytest.mark.gpu
@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_dropin_encoder_matches_reference_files(tmp_path, c):
    exe = _need(HIP[bool(c["huffman"])])
    raw = tmp_path / "in.raw"
    raw.write_bytes(open(os.path.join(O.GOLDEN, c["input"]["file"]), "rb").read())
    mat = tmp_path / "matrix.txt"  # the reference opens it read-write
    mat.write_bytes(open(os.path.join(O.GOLDEN, "matrix.txt"), "rb").read())
    out = tmp_path / "out.enc"
    r = subprocess.run([exe, "time4", str(raw), str(c["w"]), str(c["h"]), "1", str(mat), "1", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    got = out.read_bytes()
    assert len(got) == c["size"], c["name"]
    if c["huffman"] and got[:1] < b"\x80":
        # Huffman "no gain" file ('0' + the record bytes, Huffman.cpp:326-338): the reference
        # writes 8*n+1 bits into an n-byte BitStreamWriter, and put_bit never grows it
        # (BitStream.cpp:61-71), so the last byte's low 7 bits are whatever heap memory follows
        # the allocation -- zero in the golden's process, anything in this one.  Every defined bit
        # must match.
        want = open(os.path.join(O.GOLDEN, c["file"]), "rb").read()
        assert got[:-1] == want[:-1] and (got[-1] & 0x80) == (want[-1] & 0x80), c["name"]
        return
    assert hashlib.md5(got).hexdigest() == c["md5"], c["name"]
