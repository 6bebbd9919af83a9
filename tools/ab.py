"""Interleaved A/B timing of libie_hip.so variants in ONE process (cdna_hip_programming.md rule 24).

usage: python tools/ab.py [--n 4|8] [--frames 16] [--rounds 7] lib1.so lib2.so@ENV=VAL,ENV2=VAL ...
A variant "path@ENV=VAL,..." runs that library with those environment variables set around each of
its calls (knobs the library reads per launch, e.g. IE_P_GRID).
Each variant gets its own ie_ctx on torch's current stream; every round times every variant
(10 launches each, HIP events) in turn; prints the median / min us per launch, and whether the
variant's output for the batch matches the first variant's byte for byte.
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from imageencoder_amd import synth  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4)
ap.add_argument("--frames", type=int, default=16)
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--kind", default="U")
ap.add_argument("--op", default="encode", choices=["encode", "counted", "frames", "decode"],
                help="counted: time ie_encode_images_counted (the encoder with the fused byte histogram); "
                     "frames: ie_encode_frames, one concatenated stream (the C4 shape with --w 1920 --h 1080 "
                     "--frames 64); decode: ie_decode_frames of one frame's stream (--frames 1; encoded once "
                     "by the first variant, 165 header bits before it)")
ap.add_argument("--w", type=int, default=3840)
ap.add_argument("--h", type=int, default=2160)
ap.add_argument("--rotate", type=int, default=1,
                help="timed launches cycle over this many distinct input batches (4: 4 x 16 4K frames, "
                     "more than the MALL holds -- the pixels come from HBM as in bench.py)")
ap.add_argument("--rotate-out", type=int, default=1, help="timed launches cycle over this many output buffers")
ap.add_argument("libs", nargs="+")
args = ap.parse_args()

n = args.n
q = np.ascontiguousarray(np.asarray(O.read_matrix("matrix.txt" if n == 4 else "matrix8_1.txt", n), dtype=np.uint16).ravel())
w, h, nf = args.w, args.h, args.frames
y_all = (synth.uniform_device(w, h, nf * args.rotate, 3, "cuda", torch) if args.kind == "U"
         else torch.from_numpy(synth.frames(args.kind, w, h, nf * args.rotate, seed=3)).cuda())
y_rot = [y_all[i * nf:(i + 1) * nf] for i in range(args.rotate)]
y = y_rot[0]
rot = [0]
rot_o = [0]


def ybatch(sizes):
    """The batch a launch reads: batch 0 for the checked launch, the next one in turn otherwise."""
    if sizes:
        return y_rot[0]
    rot[0] = (rot[0] + 1) % args.rotate
    return y_rot[rot[0]]
stream = torch.cuda.Stream()  # a real stream handle (the default stream's handle is 0 = the ctx's own)
torch.cuda.set_stream(stream)
variants = []
shared_out = None
dec_stream = []
libs_loaded = {}
for spec in args.libs:
    path, _, envs = spec.partition("@")
    env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
    if path in libs_loaded:  # (the same library under several environments: one handle each)
        import shutil
        import tempfile
        cp = os.path.join(tempfile.mkdtemp(), "libie_hip.so")
        shutil.copy(path, cp)
        L = C.CDLL(cp, mode=C.RTLD_LOCAL)
    else:
        L = C.CDLL(os.path.abspath(path), mode=C.RTLD_LOCAL)
    libs_loaded[path] = L
    vp = C.c_void_p
    L.ie_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.ie_set_stream.argtypes = [vp, vp]
    L.ie_set_quant.argtypes = [vp, vp, C.c_int]
    L.ie_stream_bound.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64]
    L.ie_stream_bound.restype = C.c_size_t
    L.ie_encode_images.argtypes = [vp, vp, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                   vp, C.c_size_t, C.c_uint64, C.POINTER(C.c_uint64)]
    L.ie_last_error.argtypes = [vp]
    L.ie_last_error.restype = C.c_char_p
    hnd = C.c_void_p()
    assert L.ie_create(0, C.byref(hnd)) == 0
    assert L.ie_set_stream(hnd, C.c_void_p(stream.cuda_stream)) == 0
    assert L.ie_set_quant(hnd, q.ctypes.data, n) == 0
    pitch = (int(L.ie_stream_bound(w, h, n, 1, 165)) + 255) // 256 * 256
    if shared_out is None:  # one output buffer set for every variant (placement effects cancel)
        shared_out = [torch.zeros(pitch * nf, dtype=torch.uint8, device="cuda") for _ in range(args.rotate_out)]
    out = shared_out[0]
    out.zero_()
    eb = np.zeros(nf, dtype=np.uint64)

    if args.op == "counted":
        L.ie_encode_images_counted.argtypes = [vp, vp, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int,
                                               C.c_int, vp, C.c_size_t, C.c_uint64]

    if args.op == "frames":
        L.ie_encode_frames.argtypes = [vp, vp, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                       vp, C.c_size_t, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]

    if args.op == "decode":
        L.ie_decode_frames.argtypes = [vp, vp, C.c_size_t, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, vp,
                                       C.c_size_t, C.c_size_t, C.POINTER(C.c_uint64)]
        if not dec_stream:
            r = L.ie_encode_images(hnd, C.c_void_p(y.data_ptr()), w, h, w, w * h, 1, 1, 0, C.c_void_p(out.data_ptr()),
                                   pitch, 165, eb.ctypes.data_as(C.POINTER(C.c_uint64)))
            assert r == 0
            dec_stream.append((out[: (int(eb[0]) + 7) // 8].clone(), (int(eb[0]) + 7) // 8))
        out = torch.empty(h * w, dtype=torch.uint8, device="cuda")  # (this variant's pixels)

    def run(L=L, hnd=hnd, out=out, pitch=pitch, eb=eb, sizes=False, env=env):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            run1(L, hnd, out, pitch, eb, sizes)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    def run1(L, hnd, out, pitch, eb, sizes):
        if args.op == "decode":
            src, nbytes = dec_stream[0]
            e = C.c_uint64(0)
            r = L.ie_decode_frames(hnd, C.c_void_p(src.data_ptr()), nbytes, 165, w, h, 1, 1, C.c_void_p(out.data_ptr()),
                                   w, w * h, C.byref(e))
            if r != 0:
                raise RuntimeError(L.ie_last_error(hnd))
            eb[0] = e.value
            return
        y = ybatch(sizes)
        if not sizes:  # (the checked launch writes buffer 0)
            rot_o[0] = (rot_o[0] + 1) % args.rotate_out
            out = shared_out[rot_o[0]]
        if args.op == "frames":  # (eb[0] = the stream's end bit; compared over the whole stream)
            r = L.ie_encode_frames(hnd, C.c_void_p(y.data_ptr()), w, h, w, w * h, nf, 1, 0, C.c_void_p(out.data_ptr()),
                                   pitch * nf, 165, None,
                                   eb.ctypes.data_as(C.POINTER(C.c_uint64)) if sizes else None)  # (timed: async)
            if r != 0:
                raise RuntimeError(L.ie_last_error(hnd))
            return
        if args.op == "counted" and not sizes:
            r = L.ie_encode_images_counted(hnd, C.c_void_p(y.data_ptr()), w, h, w, w * h, nf, 1, 0,
                                           C.c_void_p(out.data_ptr()), pitch, 165)
            if r != 0:
                raise RuntimeError(L.ie_last_error(hnd))
            return
        r = L.ie_encode_images(hnd, C.c_void_p(y.data_ptr()), w, h, w, w * h, nf, 1, 0, C.c_void_p(out.data_ptr()),
                               pitch, 165, eb.ctypes.data_as(C.POINTER(C.c_uint64)) if sizes else None)
        if r != 0:
            raise RuntimeError(L.ie_last_error(hnd))

    print(f"running {spec}", flush=True)  # (a fault names its variant)
    run(sizes=True)
    torch.cuda.synchronize()
    fb = C.c_uint64(0)
    if hasattr(L, "ie_last_fallbacks") and L.ie_last_fallbacks(hnd, C.byref(fb)) == 0:
        print(f"{os.path.basename(os.path.dirname(path))}: FP64 fix-up requests per launch {fb.value}", flush=True)
    variants.append({"name": (os.path.basename(os.path.dirname(path)) or path) + ("@" + envs if envs else ""), "run": run, "out": out.clone(),
                     "pitch": pitch, "eb": eb.copy(), "t": []})

ref = variants[0]
for v in variants:
    ok = np.array_equal(v["eb"], ref["eb"])
    if args.op == "decode":
        ok = ok and torch.equal(v["out"], ref["out"])
    elif ok and args.op == "frames":
        nb = (int(v["eb"][0]) + 7) // 8
        ok = torch.equal(v["out"][:nb], ref["out"][:nb])
    elif ok:
        for f in range(nf):
            nb = (int(v["eb"][f]) + 7) // 8
            a = v["out"][f * v["pitch"]: f * v["pitch"] + nb]
            b = ref["out"][f * ref["pitch"]: f * ref["pitch"] + nb]
            if not torch.equal(a, b):
                ok = False
                break
    v["same"] = ok

order_rng = np.random.default_rng(0)
for r in range(args.rounds):
    for vi in order_rng.permutation(len(variants)):
        v = variants[vi]
        v["run"]()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            v["run"]()
        e1.record()
        e1.synchronize()
        v["t"].append(e0.elapsed_time(e1) * 1000.0 / args.iters)
for v in variants:
    t = np.array(v["t"])
    print(f"{v['name']:24s} median {np.median(t):8.2f} us  min {t.min():8.2f} us  same_as_first={v['same']}")
