#!/usr/bin/env python3
"""Generate the golden vectors that pin the oracle (and, through it, the HIP path).

Every expected output here comes from the REFERENCE ITSELF: the encoder/decoder binaries and
the Block<8> harness that oracle/Makefile compiles from the unmodified sources under
/root/reference into oracle/_ref/.  This script therefore only runs where /root/reference and
oracle/_ref exist (the build container); its outputs are committed as data:

* ``*.enc`` / ``*.dec``     small reference outputs, stored whole;
* ``manifest.json``         every case: how to rebuild the input (a committed reference asset
                            or a seeded synthetic frame from imageencoder_amd.synth), the codec
                            settings, and size + md5 of the reference output (large cases are
                            pinned by md5 only);
* ``cos_table.json``        the reference's cos values as exact hex doubles.

Inputs taken from the reference are its example assets (bin/ex0-ex4.raw, bin/ex6.raw and the
quantisation matrices) -- data files, copied as fixtures.

Usage:  python tests/golden/make_golden.py      (rewrites tests/golden/)
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from imageencoder_amd import synth  # noqa: E402

REF_BIN = "/root/reference/bin"
REF = os.path.join(ROOT, "oracle", "_ref")
STORE_LIMIT = 64 * 1024  # outputs up to this size are stored whole

ASSETS = ["ex0.raw", "ex1.raw", "ex2.raw", "ex3.raw", "ex4.raw", "ex6.raw", "matrix.txt", "matrix4_2.txt", "matrix8_1.txt", "matrix8_2.txt"]


def md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


def run(cmd, cwd):
    # every reference encoder/decoder run segfaults in its destructor AFTER saving the output
    # (ImageBase.cpp:161-165); success is judged by the output file.
    subprocess.run(cmd, cwd=cwd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


def ref_cli(binary: str, raw: bytes, w: int, h: int, rle: int, matrix: str, video: bool = False) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "in.raw"), "wb").write(raw)
        shutil.copy(os.path.join(HERE, matrix), os.path.join(d, "m.txt"))
        keys = dict(rawfile="in.raw", encfile="out.enc", decfile="out.dec", width=w, height=h,
                    rle=rle, quantfile="m.txt", logfile="")
        if video:
            keys.update(gop=1, merange=16)
        open(os.path.join(d, "c.conf"), "w").write("".join(f"{k}={v}\n" for k, v in keys.items()))
        run([os.path.join(REF, binary), "c.conf"], d)
        return open(os.path.join(d, "out.enc"), "rb").read()


def ref_decode(enc: bytes) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "out.enc"), "wb").write(enc)
        keys = dict(rawfile="in.raw", encfile="out.enc", decfile="out.dec", width=0, height=0,
                    rle=1, quantfile="m.txt", logfile="")
        open(os.path.join(d, "c.conf"), "w").write("".join(f"{k}={v}\n" for k, v in keys.items()))
        run([os.path.join(REF, "decoder"), "c.conf"], d)
        return open(os.path.join(d, "out.dec"), "rb").read()


def ref_harness(args, huff=False) -> None:
    exe = os.path.join(REF, "ref_harness_huff" if huff else "ref_harness")
    subprocess.run([exe] + [str(a) for a in args], check=True, stdout=subprocess.DEVNULL)


def ref_enc8(raw: bytes, w: int, h: int, rle: int, matrix: str, huff: bool) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "in.raw"), "wb").write(raw)
        args = ["enc8", os.path.join(d, "in.raw"), w, h, rle, os.path.join(HERE, matrix), os.path.join(d, "o")]
        if huff:
            args.append("huff")
        ref_harness(args)
        return open(os.path.join(d, "o"), "rb").read()


def ref_dec8(enc: bytes) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "e"), "wb").write(enc)
        ref_harness(["dec8", os.path.join(d, "e"), os.path.join(d, "o")])
        return open(os.path.join(d, "o"), "rb").read()


def input_bytes(spec) -> bytes:
    if spec["kind"] == "asset":
        return open(os.path.join(HERE, spec["file"]), "rb").read()
    if spec["kind"] == "synth":
        y = synth.frames(spec["gen"], spec["w"], spec["h"], spec.get("frames", 1), spec["seed"])
        if spec.get("yuv420"):
            return synth.yuv420(y)
        return y.tobytes()
    raise ValueError(spec)


def cases():
    S = synth.DEFAULT_SEED
    out = []

    def add(name, inp, w, h, n, rle, matrix, huff=False, video=False, decode=False):
        out.append(dict(name=name, input=inp, w=w, h=h, n=n, rle=rle, matrix=matrix, huffman=huff,
                        video=video, decode=decode))

    ex0 = dict(kind="asset", file="ex0.raw")
    ex6 = dict(kind="asset", file="ex6.raw")
    for huff in (False, True):
        hs = "_huff" if huff else ""
        add(f"ex0_4x4{hs}", ex0, 8, 8, 4, 1, "matrix.txt", huff, decode=True)
        add(f"ex0_4x4_norle{hs}", ex0, 8, 8, 4, 0, "matrix.txt", huff, decode=True)
        add(f"ex0_8x8{hs}", ex0, 8, 8, 8, 1, "matrix8_1.txt", huff, decode=True)
        add(f"ex6_4x4{hs}", ex6, 512, 256, 4, 1, "matrix.txt", huff, decode=True)
        add(f"ex6_8x8{hs}", ex6, 512, 256, 8, 1, "matrix8_1.txt", huff, decode=True)
    # the reference's published example images (README.md:175-183; natural content at real
    # scale: long zero runs, smooth gradients), the sizes/md5s of SURVEY Appendix B
    for i, (w, h) in ((1, (936, 936)), (2, (512, 512)), (3, (400, 400)), (4, (4096, 912))):
        exi = dict(kind="asset", file=f"ex{i}.raw")
        add(f"ex{i}_4x4", exi, w, h, 4, 1, "matrix.txt", decode=True)
        add(f"ex{i}_4x4_huff", exi, w, h, 4, 1, "matrix.txt", True, decode=True)
        add(f"ex{i}_8x8", exi, w, h, 8, 1, "matrix8_1.txt", decode=True)
    add("ex6_4x4_m2", ex6, 512, 256, 4, 1, "matrix4_2.txt", decode=True)
    add("ex6_4x4_norle", ex6, 512, 256, 4, 0, "matrix.txt", decode=True)
    add("ex6_8x8_m2", ex6, 512, 256, 8, 1, "matrix8_2.txt", decode=True)
    add("ex6_8x8_norle", ex6, 512, 256, 8, 0, "matrix8_1.txt")
    for gen in ("U", "M"):
        sy = dict(kind="synth", gen=gen, w=256, h=256, seed=S)
        add(f"syn{gen}256_4x4", sy, 256, 256, 4, 1, "matrix.txt", decode=True)
        add(f"syn{gen}256_4x4_huff", sy, 256, 256, 4, 1, "matrix.txt", True, decode=True)
        add(f"syn{gen}256_4x4_norle", sy, 256, 256, 4, 0, "matrix.txt")
        add(f"syn{gen}256_8x8", sy, 256, 256, 8, 1, "matrix8_1.txt", decode=True)
        add(f"syn{gen}256_8x8_huff", sy, 256, 256, 8, 1, "matrix8_1.txt", True)
        # a ragged width (W not a multiple of 16 px) and tiny frames
        sr = dict(kind="synth", gen=gen, w=200, h=56, seed=S + 7)
        add(f"syn{gen}200x56_4x4", sr, 200, 56, 4, 1, "matrix.txt", decode=True)
        add(f"syn{gen}200x56_8x8", sr, 200, 56, 8, 1, "matrix8_1.txt", decode=True)
        st = dict(kind="synth", gen=gen, w=4, h=4, seed=S + 9)
        add(f"syn{gen}4x4px_4x4", st, 4, 4, 4, 1, "matrix.txt", decode=True)
        # video container, gop = 1 (VideoEncoder.cpp:22-107)
        sv = dict(kind="synth", gen=gen, w=64, h=48, frames=5, seed=S + 100, yuv420=True)
        add(f"vid{gen}64x48x5_4x4", sv, 64, 48, 4, 1, "matrix.txt", video=True)
        add(f"vid{gen}64x48x5_4x4_huff", sv, 64, 48, 4, 1, "matrix.txt", True, video=True)
        # full-size frames: pinned by md5 only
        s4 = dict(kind="synth", gen=gen, w=3840, h=2160, seed=S)
        add(f"syn{gen}4k_4x4", s4, 3840, 2160, 4, 1, "matrix.txt", decode=(gen == "M"))
        add(f"syn{gen}4k_8x8", s4, 3840, 2160, 8, 1, "matrix8_1.txt")
        add(f"syn{gen}4k_4x4_huff", s4, 3840, 2160, 4, 1, "matrix.txt", True)
        sv2 = dict(kind="synth", gen=gen, w=1920, h=1080, frames=3, seed=S + 200, yuv420=True)
        add(f"vid{gen}1080x3_4x4", sv2, 1920, 1080, 4, 1, "matrix.txt", video=True)
    return out


def main():
    if not os.path.exists(os.path.join(REF, "encoder")):
        sys.exit("oracle/_ref not built: run `make -C oracle ref` where /root/reference exists")
    for a in ASSETS:
        shutil.copy(os.path.join(REF_BIN, a), os.path.join(HERE, a))
    manifest = []
    for c in cases():
        raw = input_bytes(c["input"])
        if c["n"] == 8:
            enc = ref_enc8(raw, c["w"], c["h"], c["rle"], c["matrix"], c["huffman"])
        else:
            binary = "encoder_huff" if c["huffman"] else "encoder"
            enc = ref_cli(binary, raw, c["w"], c["h"], c["rle"], c["matrix"], c["video"])
        entry = dict(c, size=len(enc), md5=md5(enc))
        if len(enc) <= STORE_LIMIT:
            fn = c["name"] + ".enc"
            open(os.path.join(HERE, fn), "wb").write(enc)
            entry["file"] = fn
        if c["decode"]:
            dec = ref_dec8(enc) if c["n"] == 8 else ref_decode(enc)
            entry["dec_size"], entry["dec_md5"] = len(dec), md5(dec)
            if len(dec) <= STORE_LIMIT:
                fn = c["name"] + ".dec"
                open(os.path.join(HERE, fn), "wb").write(dec)
                entry["dec_file"] = fn
        manifest.append(entry)
        print(f"{c['name']:28s} {len(enc):9d} B  {entry['md5'][:12]}", flush=True)
    json.dump(manifest, open(os.path.join(HERE, "manifest.json"), "w"), indent=1)

    cos = {}
    for n in (4, 8):
        r = subprocess.run([os.path.join(REF, "ref_harness"), "cos", str(n)], check=True,
                           capture_output=True, text=True)
        cos[str(n)] = [line.split()[2] for line in r.stdout.strip().splitlines()]
    json.dump(cos, open(os.path.join(HERE, "cos_table.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
