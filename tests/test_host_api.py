"""The host library's C++ surface mirrors the reference's class interface (include/ie_host.hpp):
dc::MatrixReader<N> (MatrixReader.hpp:15-37), dc::ImageProcessor with the virtual
process()/saveResult() pair (ImageBase.hpp:35-77) and ImageEncoder / ImageDecoder deriving from it.
tests/cpp/host_api.cpp is compiled against the header and linked to libie_host.so here; the
matrix round trip runs on the CPU, the encode / decode through the base class on the GPU.
"""
import hashlib
import os
import subprocess

import pytest

from tests import oracle_lib as O

LIB = os.path.join(O.ROOT, "imageencoder_amd", "lib")
SRC = os.path.join(O.ROOT, "tests", "cpp", "host_api.cpp")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    if not os.path.exists(os.path.join(LIB, "libie_host.so")):
        pytest.skip("libie_host.so not built (make host)")
    out = str(tmp_path_factory.mktemp("host_api") / "host_api")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-I" + os.path.join(O.ROOT, "include"), SRC, "-L" + LIB,
                        "-lie_host", "-lie_hip", "-Wl,-rpath," + LIB, "-o", out],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    return out


@pytest.mark.parametrize("name,n", [("matrix.txt", 4), ("matrix4_2.txt", 4), ("matrix8_1.txt", 8)])
def test_matrix_reader_template(exe, name, n):
    r = subprocess.run([exe, "matrix", os.path.join(O.GOLDEN, name), str(n)], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    bits, qb, last = r.stdout.split("\n")[0].split()
    q = O.read_matrix(name, n)
    want_qb = max(int(v).bit_length() for v in q)
    assert int(qb) == want_qb and int(bits) == 5 + want_qb * n * n and float(last) == float(q[-1])
    # the same bits as the header the oracle writes after its leading 0 bit and before rle/w/h
    hdr, hb = O.load().header(n, q, True, 8, 8, huffman=True)
    ours = bytes.fromhex(r.stdout.split("\n")[1])
    nb = int(bits)
    a = "".join(f"{b:08b}" for b in ours)[:nb]
    b = "".join(f"{x:08b}" for x in hdr.tobytes())[:nb]
    assert a == b


def test_matrix_reader_rejects_wrong_size(exe):
    r = subprocess.run([exe, "matrix", os.path.join(O.GOLDEN, "matrix8_1.txt"), "4"], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 4 and "Too many" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["ex6_4x4", "ex6_8x8"])
def test_encoder_decoder_through_the_base_class(exe, tmp_path, case):
    c = {x["name"]: x for x in O.manifest()}[case]
    raw = tmp_path / "in.raw"
    raw.write_bytes(open(os.path.join(O.GOLDEN, c["input"]["file"]), "rb").read())
    enc = tmp_path / "out.enc"
    r = subprocess.run([exe, "encode", str(raw), str(c["w"]), str(c["h"]), os.path.join(O.GOLDEN, c["matrix"]),
                        str(c["n"]), str(enc)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert hashlib.md5(enc.read_bytes()).hexdigest() == c["md5"]
    if c.get("decode"):
        dec = tmp_path / "out.dec"
        r = subprocess.run([exe, "decode", str(enc), str(dec), str(c["n"])], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        assert hashlib.md5(dec.read_bytes()).hexdigest() == c["dec_md5"]
