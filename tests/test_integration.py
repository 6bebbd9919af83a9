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


# ------------------------------------------------------------------------------------------------
# The whole drop-in: the reference's UNMODIFIED main.cpp and objects, with the image / video
# encoders and decoders replaced by integration/*_hip.cpp and the decoder's Huffman decode routed to
# the device by the linker (oracle/Makefile: encoder_hip, encoder_hip_huff, decoder_hip).  These are
# the reference's own command lines -- settings file in, files out -- running on libie_hip.so.
DROP = {"enc": os.path.join(REF, "encoder_hip"), "enc_huff": os.path.join(REF, "encoder_hip_huff"),
        "dec": os.path.join(REF, "decoder_hip")}
WRAPPED = "_ZN4algo7HuffmanIhE6decodeERN4util15BitStreamReaderE"


@pytest.mark.parametrize("kind,syms", [
    ("enc", ("ie_encode_frames", "ie_encode_gop")),
    ("enc_huff", ("ie_encode_frames", "ie_encode_gop")),
    ("dec", ("ie_decode_frames", "ie_decode_gop", "ie_huffman_table", "ie_huffman_decode")),
])
def test_dropin_cli_links_the_gpu_library(kind, syms):
    """The drop-in command lines take their loops from libie_hip.so; the decoder's Huffman decode
    calls reach the wrapper (no call to the reference's own bit walk remains)."""
    exe = _need(DROP[kind])
    und = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, timeout=60).stdout
    for sym in syms:
        assert sym in und, sym
    if kind == "dec":
        dis = subprocess.run(["objdump", "-d", "--no-show-raw-insn", exe], capture_output=True, text=True,
                             timeout=120).stdout
        calls = [ln for ln in dis.splitlines() if "call" in ln and WRAPPED + ">" in ln]
        assert calls and all("<__wrap_" + WRAPPED + ">" in ln for ln in calls), calls[:4]


def _conf(d, **kv):
    p = os.path.join(d, "set.conf")
    with open(p, "w") as f:
        f.write("".join(f"{k}={v}\n" for k, v in kv.items()))
    return p


def _cli(exe, conf, cwd):
    return subprocess.run([exe, conf], cwd=cwd, capture_output=True, text=True, timeout=120)


def _md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


IMG = [c for c in O.manifest() if c["input"]["kind"] == "asset" and c["n"] == 4 and not c["video"]]


@pytest.mark.gpu
@pytest.mark.parametrize("c", IMG, ids=[c["name"] for c in IMG])
def test_dropin_cli_image_roundtrip(tmp_path, c):
    """encoder_hip[_huff] then decoder_hip, the reference's main() with the settings file of
    bin/ex*.conf: the encoded file is the reference encoder's (golden md5), the decoded image the
    reference decoder's.  The drop-in exits 0 (the reference's exit-time crash is not reached)."""
    d = str(tmp_path)
    open(os.path.join(d, "in.raw"), "wb").write(O.case_input(c))
    open(os.path.join(d, "m.txt"), "wb").write(open(os.path.join(O.GOLDEN, c["matrix"]), "rb").read())
    conf = _conf(d, rawfile="in.raw", encfile="out.enc", decfile="out.dec", width=c["w"], height=c["h"],
                 rle=c["rle"], quantfile="m.txt", logfile="")
    r = _cli(_need(DROP["enc_huff" if c["huffman"] else "enc"]), conf, d)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    enc = open(os.path.join(d, "out.enc"), "rb").read()
    if c["huffman"] and enc[:1] < b"\x80":
        # "no gain" Huffman file: the reference's last byte carries 7 bits of heap (see above)
        want = O.case_expected(c)
        assert want is not None and enc[:-1] == want[:-1] and (enc[-1] & 0x80) == (want[-1] & 0x80)
    else:
        assert len(enc) == c["size"] and _md5(enc) == c["md5"], c["name"]
    if not c.get("decode"):
        return
    r = _cli(_need(DROP["dec"]), conf, d)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    dec = open(os.path.join(d, "out.dec"), "rb").read()
    assert len(dec) == c["dec_size"] and _md5(dec) == c["dec_md5"], c["name"]


def _ref_decode(d, conf):
    """The reference decoder itself (oracle/_ref/decoder, built from its sources) as the checker for
    videos whose decoded output the manifest does not pin; it crashes at exit after writing
    (ImageBase.cpp:161-165), so success is judged by the file."""
    exe = _need(os.path.join(REF, "decoder"))
    subprocess.run([exe, conf], cwd=d, capture_output=True, timeout=300)
    return open(os.path.join(d, "ref.dec"), "rb").read()


VID = [c for c in O.manifest() if c["video"] and c["n"] == 4 and c["w"] * c["h"] <= 64 * 48]
GOP = [c for c in O.manifest_gop() if "dec1_md5" in c]


@pytest.mark.gpu
@pytest.mark.parametrize("c", VID + GOP, ids=[c["name"] for c in VID + GOP])
def test_dropin_cli_video_roundtrip(tmp_path, c):
    """Videos through the reference's main(): gop = 1 (Huffman on / off) and P-frame videos
    (gop, merange from the settings file) encode to the reference's files; decoder_hip, with
    motion compensation on and off, writes the reference decoder's frames."""
    d = str(tmp_path)
    open(os.path.join(d, "in.yuv"), "wb").write(O.case_input(c))
    open(os.path.join(d, "m.txt"), "wb").write(open(os.path.join(O.GOLDEN, c["matrix"]), "rb").read())
    gop, merange = c.get("gop", 1), c.get("merange", 16)
    conf = _conf(d, rawfile="in.yuv", encfile="v.enc", decfile="v.dec", width=c["w"], height=c["h"],
                 rle=c["rle"], quantfile="m.txt", logfile="", gop=gop, merange=merange)
    r = _cli(_need(DROP["enc_huff" if c["huffman"] else "enc"]), conf, d)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    enc = open(os.path.join(d, "v.enc"), "rb").read()
    assert len(enc) == c["size"] and _md5(enc) == c["md5"], c["name"]
    for mc in (1, 0):
        dconf = _conf(d, rawfile="in.yuv", encfile="v.enc", decfile="v.dec", width=c["w"], height=c["h"],
                      rle=c["rle"], quantfile="m.txt", logfile="", motioncompensation=mc)
        r = _cli(_need(DROP["dec"]), dconf, d)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        dec = open(os.path.join(d, "v.dec"), "rb").read()
        if f"dec{mc}_md5" in c:
            assert _md5(dec) == c[f"dec{mc}_md5"], (c["name"], mc)
        else:
            rconf = _conf(d, rawfile="in.yuv", encfile="v.enc", decfile="ref.dec", width=c["w"], height=c["h"],
                          rle=c["rle"], quantfile="m.txt", logfile="", motioncompensation=mc)
            assert dec == _ref_decode(d, rconf), (c["name"], mc)
