"""The decoder's 32-positions-at-once header test (imageencoder_amd/csrc/ie_recbits.h,
valid_mask32) against the per-position test of the record parse (ie_decode.hip rec_len_head:
bl != 0 and, with RLE, the bl-bit value count <= N*N, Block.cpp:442-472): every 20-bit header
and 2 M random / sparse / dense windows, 4x4 and 8x8, RLE on and off (tests/csrc/recbits_check.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_valid_mask32_matches_per_position_test(tmp_path):
    exe = tmp_path / "recbits_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "imageencoder_amd", "csrc"),
                    os.path.join(ROOT, "tests", "csrc", "recbits_check.cpp"), "-o", str(exe)], check=True, timeout=120)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout
