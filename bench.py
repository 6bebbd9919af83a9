#!/usr/bin/env python3
"""Benchmark: Mpixels/s of the ImageEncoder encode hot path (DCT + quant + zig-zag RLE pack) on
MI355X, with the reference's own OpenMP CPU encoder timed beside it.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|c5]

A "step" is one launch of the encoder over one batch of distinct synthetic frames resident in
HBM (a rotating set larger than the 256 MiB Infinity Cache, so HBM is what is measured):

  c2 (default)  3840x2160, 4x4 blocks, matrix.txt, RLE: a batch of independent images
  c3            3840x2160, 8x8 blocks, matrix8_1.txt, RLE
  c4            1920x1080 gop=1 video batch, 4x4: frames sharded over ranks, ONE stream
                assembled on rank 0 by an RCCL gather (encode + gather are both timed)
  c5            3840x2160, 4x4, Huffman post-pass on every image (device histogram + host
                tree build + device re-encode)

For N>1 run under torch.distributed.run: one process per GPU, each rank encodes its own batch
(weak scaling); rank 0 prints one JSON line.  value = all pixels encoded by all ranks / max-over-
ranks wall time of the K timed steps (inputs already resident, outputs left in HBM).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    "c2": dict(w=3840, h=2160, n=4, matrix="matrix.txt", batch=16, resident=64, gen="U", huffman=False),
    "c3": dict(w=3840, h=2160, n=8, matrix="matrix8_1.txt", batch=16, resident=64, gen="U", huffman=False),
    "c4": dict(w=1920, h=1080, n=4, matrix="matrix.txt", batch=64, resident=128, gen="U", huffman=False),
    "c5": dict(w=3840, h=2160, n=4, matrix="matrix.txt", batch=16, resident=64, gen="U", huffman=True),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    p.add_argument("--mode", default="fast", choices=["fast", "exact"])
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--cpu-iters", type=int, default=4)
    p.add_argument("--no-decode", action="store_true", help="skip the one-image decode timing (inverse path)")
    p.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) timing")
    p.add_argument("--batch", type=int, default=None, help="frames per launch (default: the workload's)")
    p.add_argument("--resident", type=int, default=None, help="distinct resident frames (default: the workload's)")
    p.add_argument("--no-single-frame", dest="single_frame", action="store_false",
                   help="skip timing one-image launches (configs[1] taken literally: one 4K frame per launch)")
    return p.parse_args()


def cpu_baseline(cfg, frame: np.ndarray) -> dict | None:
    """The reference encoder itself (oracle/_ref/ref_harness, compiled from the reference sources
    with OpenMP) timed on this host on a bounded sample: cfg-sized frames, --cpu-iters passes.
    Falls back to the oracle restatement (kind "port") if the reference build is absent."""
    from tests import oracle_lib as O

    threads = min(16, os.cpu_count() or 1)
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    w, h = cfg["w"], cfg["h"]
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness_huff" if cfg["huffman"] else "ref_harness")
    iters = ARGS.cpu_iters
    if cfg["n"] == 4 and os.path.exists(harness):
        with tempfile.TemporaryDirectory() as d:
            raw = os.path.join(d, "in.raw")
            frame.tofile(raw)
            # the reference opens the matrix with std::fstream(in|out): it needs a writable copy
            mat = os.path.join(d, cfg["matrix"])
            shutil.copyfile(os.path.join(ROOT, "tests", "golden", cfg["matrix"]), mat)
            os.chmod(mat, 0o644)
            r = subprocess.run([harness, "time4", raw, str(w), str(h), "1", mat, str(iters)],
                               env=env, capture_output=True, text=True, timeout=600)
            line = [ln for ln in r.stderr.splitlines() if ln.startswith("{")]
            why = f"ref_harness rc={r.returncode}: {r.stderr.strip()[-200:]}"
            if r.returncode == 0 and line:
                res = json.loads(line[-1])
                return dict(value=round(w * h / (res["mean_ms"] * 1e3), 3), unit="Mpx/s", cores=threads,
                            kind="reference",
                            sample=f"{iters} x {w}x{h} {cfg['gen']} frame, reference ImageEncoder::process "
                                   f"(OpenMP{', Huffman' if cfg['huffman'] else ''}) via oracle/_ref/ref_harness, "
                                   f"{threads} threads, mean {res['mean_ms']:.1f} ms/frame")
    if cfg["n"] != 4:
        why = ("the reference fixes its block size at compile time (Block.hpp:13, BlockSize = 4u): an 8x8 "
               "reference build would mean editing its sources, so the 8x8 baseline is the oracle port")
    # port: the oracle restatement (single image encode, OpenMP transform, serial emission)
    oracle = O.load()
    q = O.read_matrix(cfg["matrix"], cfg["n"])
    t0 = time.perf_counter()
    for _ in range(iters):
        oracle.encode_image(frame, cfg["n"], q, rle=True, huffman=cfg["huffman"])
    dt = (time.perf_counter() - t0) / iters
    return dict(value=round(w * h / (dt * 1e6), 3), unit="Mpx/s", cores=threads, kind="port",
                sample=f"{iters} x {w}x{h} {cfg['gen']} frame, oracle restatement, {threads} threads",
                reference_unavailable=locals().get("why", "oracle/_ref not built"))


class Timer:
    """K timed steps bracketed by barrier + synchronize; HIP events on the encoder's stream for
    the per-launch device time of the dominant kernel."""

    def __init__(self, torch, dist, dev, stream, world):
        self.torch, self.dist, self.dev, self.stream, self.world = torch, dist, dev, stream, world

    def run(self, step, warmup, steps, drain=None):
        """drain (pipelined steps): completes the work the last step left in flight -- once after
        the warmup (outside the timed region) and once after the K timed steps (inside it)."""
        torch, dist = self.torch, self.dist
        for i in range(warmup):
            step(i)
        if drain:
            drain()
        torch.cuda.synchronize(self.dev)
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize(self.dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(self.stream)
        for i in range(steps):
            step(warmup + i)
        if drain:
            drain()
        ev1.record(self.stream)
        torch.cuda.synchronize(self.dev)
        wall = time.perf_counter() - t0
        if self.world > 1:
            dist.barrier()
        # gloo (rehearsal backend) reduces host tensors; RCCL device tensors
        t = torch.tensor([wall], dtype=torch.float64,
                         device="cpu" if self.world > 1 and dist.get_backend() == "gloo" else self.dev)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()), ev0.elapsed_time(ev1) / 1e3


def main():
    global ARGS
    ARGS = args = parse()
    cfg = WORKLOADS[args.workload]
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    from imageencoder_amd import MODE_EXACT, MODE_FAST, Codec, stream_bound, synth, write_header
    from imageencoder_amd import dist as D
    from tests import oracle_lib as O

    # IE_BENCH_BACKEND=gloo with ranks sharing the visible GPUs (local % device_count) rehearses the
    # multi-rank control flow on a box with fewer GPUs than ranks; the real run is RCCL, one GPU each
    backend = os.environ.get("IE_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    w, h, n, B, R = cfg["w"], cfg["h"], cfg["n"], cfg["batch"], cfg["resident"]
    B = args.batch or B
    R = max(args.resident or R, B)
    q = O.read_matrix(cfg["matrix"], n)
    codec = Codec(local, q, n)
    # a dedicated stream: the encoder's launches and the timing events share it (the default
    # stream's handle is NULL, which ie_set_stream reads as "the context's own stream")
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    codec.set_stream(stream.cuda_stream)
    mode = MODE_EXACT if args.mode == "exact" else MODE_FAST
    timer = Timer(torch, dist, dev, stream, world)

    # resident synthetic frames, distinct per rank (seed offset), generated on the host once
    seed = synth.DEFAULT_SEED + 1000 * rank
    frames = torch.empty((R, h, w), dtype=torch.uint8, device=dev)
    for i in range(R):
        frames[i].copy_(torch.from_numpy(synth.frame(cfg["gen"], w, h, seed + i)))
    nslots = R // B
    extra = {}

    if args.workload in ("c2", "c3", "c5"):
        hdr_bits = write_header(n, q, True, w, h, huffman=cfg["huffman"])[1]
        pitch = (stream_bound(w, h, n, 1, hdr_bits) + 255) // 256 * 256
        # two output buffers in turn (the pipelined Huffman step needs both; see step below)
        outs = [torch.zeros(pitch * B, dtype=torch.uint8, device=dev) for _ in range(2)]
        # sizes for the algorithmic byte count (deterministic per frame)
        ends_per_slot = []
        for slot in range(nslots):
            ends_per_slot.append(codec.encode_images(frames[slot * B:(slot + 1) * B], w, h, outs[0],
                                                     out_pitch=pitch, nframes=B, start_bit=hdr_bits, mode=mode))
        out_bytes_per_launch = sum(int(sum((int(e) - hdr_bits + 7) // 8 for e in ends))
                                   for ends in ends_per_slot) / nslots
        fallbacks = codec.last_fallbacks()

        if not cfg["huffman"]:
            def step(i):
                slot = i % nslots
                codec.encode_images(frames[slot * B:(slot + 1) * B], w, h, outs[i % len(outs)], out_pitch=pitch,
                                    nframes=B, start_bit=hdr_bits, mode=mode, want_sizes=False)
        else:
            hpitch = 2 * pitch  # >= 32-bit codes x payload bytes
            houts = torch.zeros(hpitch * B, dtype=torch.uint8, device=dev)
            hsizes = []
            pending = []  # the batch whose trees + pack are still to do: (output buffer, slot)

            def finish():
                if pending:
                    out, hslot = pending.pop()
                    hsizes[:] = codec.huffman_finish_after_encode(out, pitch, B, hslot, houts, hpitch)

            def step(i):
                # a batch's Huffman pass: the byte counts (from the encoder), the first positions
                # (lengths from the encoder's end bits on the device), host tree builds, one pack
                # launch.  Pipelined: batch i's encode
                # and histogram are issued before batch i-1's trees, so the host builds those
                # while the device encodes (two output buffers alternate, so batch i never
                # overwrites the bytes batch i-1's pack still reads)
                slot = i % nslots
                out = outs[i % len(outs)]
                # the encoder also counts the bytes it stores (the histogram of the Huffman pass)
                codec.encode_images(frames[slot * B:(slot + 1) * B], w, h, out, out_pitch=pitch,
                                    nframes=B, start_bit=hdr_bits, mode=mode, want_sizes=False, count_bytes=True)
                codec.huffman_begin_after_encode(out, pitch, B, i % 2)
                finish()
                pending.append((out, i % 2))
        wall, gpu_s = timer.run(step, args.warmup, args.steps, drain=finish if cfg["huffman"] else None)
        px_total = world * args.steps * B * w * h
        in_bytes_per_launch = B * w * h
        # dominant kernel alone: the block encoder's launch time on its stream
        enc_s = gpu_s / args.steps
        if cfg["huffman"]:
            def enc_only(i):
                slot = i % nslots
                codec.encode_images(frames[slot * B:(slot + 1) * B], w, h, outs[i % len(outs)], out_pitch=pitch,
                                    nframes=B, start_bit=hdr_bits, mode=mode, want_sizes=False)
            _, g2 = timer.run(enc_only, 1, args.steps)
            enc_s = g2 / args.steps
            extra["huffman_bytes_per_image"] = int(sum(hsizes) / max(len(hsizes), 1))
        if args.single_frame:  # one 4K frame per launch: the latency of the single-image configuration
            one = outs[0][:pitch]

            def single(i):
                f = i % R
                codec.encode_images(frames[f:f + 1], w, h, one, out_pitch=pitch, nframes=1, start_bit=hdr_bits,
                                    mode=mode, want_sizes=False)
            _, g1 = timer.run(single, 2, 4 * B)
            extra["single_frame"] = {"us_per_frame": round(g1 / (4 * B) * 1e6, 2),
                                     "Mpx_s": round(w * h / (g1 / (4 * B)) / 1e6, 1)}
        if not cfg["huffman"] and not args.no_e2e:
            # end to end from HOST buffers (reported separately, never `value`): pageable
            # numpy frames in, the library stages them over PCIe, encodes, copies the streams back
            yh = frames[:B].cpu().numpy()
            oh = np.zeros(pitch * B, dtype=np.uint8)
            codec.encode_images(yh, w, h, oh, out_pitch=pitch, nframes=B, start_bit=hdr_bits, mode=mode)
            ke = 3
            t0 = time.perf_counter()
            for _ in range(ke):
                codec.encode_images(yh, w, h, oh, out_pitch=pitch, nframes=B, start_bit=hdr_bits, mode=mode)
            te = (time.perf_counter() - t0) / ke
            extra["e2e_host_buffers"] = {"ms_per_batch": round(te * 1e3, 2), "Mpx_s": round(B * w * h / te / 1e6, 1),
                                         "note": "pageable host frames in, host streams out (PCIe both ways)"}
        if not cfg["huffman"] and not args.no_decode:
            # the inverse path: one image's stream decoded back to pixels on the
            # device (chunked record walk + index scan + FP64 IDCT), wall time per call incl. syncs
            ends0 = codec.encode_images(frames[:B], w, h, outs[0], out_pitch=pitch, nframes=B, start_bit=hdr_bits,
                                        mode=mode)
            nb0 = (int(ends0[0]) + 7) // 8
            pix = torch.empty((h, w), dtype=torch.uint8, device=dev)
            one = outs[0][:nb0]
            codec.decode_frames(one, w, h, pix, start_bit=hdr_bits, length=nb0)
            torch.cuda.synchronize(dev)
            kd = 10
            t0 = time.perf_counter()
            for _ in range(kd):
                codec.decode_frames(one, w, h, pix, start_bit=hdr_bits, length=nb0)
            torch.cuda.synchronize(dev)
            td = (time.perf_counter() - t0) / kd
            extra["decode_one_image"] = {"us": round(td * 1e6, 1), "Mpx_s": round(w * h / td / 1e6, 1)}
        workload = (f"{args.workload}: {w}x{h} {n}x{n} {cfg['matrix']} RLE"
                    f"{' +Huffman' if cfg['huffman'] else ''}, batch of {B} independent images per step, "
                    f"{R} distinct resident frames per GPU ({R * w * h / 2**20:.0f} MiB)")
        parallelism = f"independent images sharded x{world} (no collective)"
    else:  # c4: one gop=1 video stream, frames sharded over ranks, RCCL gather to rank 0
        F = B * world
        f0, f1 = D.frame_range(F, rank, world)
        nloc = f1 - f0
        hdr, hb = write_header(n, q, True, w, h, video=True, frames=F, gop=1, merange=16)
        root_cap = stream_bound(w, h, n, F, hb) + 64
        out_root = torch.zeros(root_cap if rank == 0 else 8, dtype=torch.uint8, device=dev)
        if rank == 0:
            out_root[:hdr.size].copy_(torch.from_numpy(hdr))
        seg_cap = stream_bound(w, h, n, max(nloc, 1), 0) + 64
        seg = torch.zeros(seg_cap, dtype=torch.uint8, device=dev)
        shifted = torch.zeros(seg_cap + 8, dtype=torch.uint8, device=dev)

        def shift(src, nbytes, start):
            shifted[:8].zero_()
            codec.bitcopy(src[:nbytes], shifted, start)
            return shifted

        def new_bytes(k):
            return torch.zeros(k, dtype=torch.uint8, device=dev)

        stats = {}

        def encode_local(i, sizes=True):
            slot = (i * nloc) % max(R - nloc + 1, 1)
            y = frames[slot:slot + nloc]
            dst, sb = (out_root, hb) if rank == 0 else (seg, 0)
            r = codec.encode_frames(y, w, h, dst, start_bit=sb, nframes=nloc, mode=mode, want_sizes=sizes)
            if not sizes:
                return None, None
            return (None if rank == 0 else seg), r[1] - sb

        def step(i):
            if world == 1:  # the stream is complete after the launch: no host round trip per step
                encode_local(i, sizes=False)
                return
            sg, bits = encode_local(i)
            stats["total_bits"] = D.gather_stream(dist, rank, world, sg, bits, hb, out_root, shift, new_bytes)

        wall, gpu_s = timer.run(step, args.warmup, args.steps)
        if world == 1:
            stats["total_bits"] = hb + encode_local(0)[1]
        # the encoder launch alone (asynchronous: no size read-back between launches)
        wall_enc, gpu_enc = timer.run(lambda i: encode_local(i, sizes=False), 1, args.steps)
        px_total = world * args.steps * nloc * w * h
        extra["encode_only_Mpx_s"] = round(px_total / wall_enc / 1e6, 2)
        extra["stream_bytes"] = (stats["total_bits"] + 7) // 8
        in_bytes_per_launch = nloc * w * h
        out_bytes_per_launch = extra["stream_bytes"] / world
        enc_s = gpu_enc / args.steps
        fallbacks = codec.last_fallbacks()
        B = nloc
        workload = (f"c4: {F} x {w}x{h} gop=1 video ({nloc} frames per GPU), {n}x{n} {cfg['matrix']} RLE, "
                    f"ONE stream assembled on rank 0 (all_gather of sizes + bit re-shift + P2P gather)")
        parallelism = f"frame-sharded x{world} + RCCL gather"

    value = px_total / wall / 1e6
    alg_bytes = in_bytes_per_launch + out_bytes_per_launch
    achieved = alg_bytes / enc_s / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(cfg, synth.frame(cfg["gen"], w, h, seed))

    if rank == 0:
        traffic = None
        tf = os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
        if os.path.exists(tf):
            traffic = json.load(open(tf)).get("hbm_bytes_per_launch")
        line = {
            "metric": "Mpixels/s encode (DCT+quant+RLE), 4K grayscale, 1/2/4/8 GPU + CPU ref",
            "value": round(value, 2),
            "unit": "Mpx/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (splitmix64 uniform 8-bit frames, seeded per rank)",
            "config": {"workload": workload, "block": n, "frames_per_step_per_gpu": B, "mode": args.mode,
                       "parallelism": parallelism},
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "encode_kernel",
                "alg_bytes_per_launch": int(alg_bytes),
                "launch_us": round(enc_s * 1e6, 2),
                "read_only_frac": round(in_bytes_per_launch / enc_s / 1e9 / HBM_PEAK_GBS, 4),
            },
            "cpu_baseline": cpu,
            "fallback_coefs_per_launch": fallbacks,
            "arith": "FP32 separable DCT + FP64 re-evaluation of near-tie coefficients (bit-exact)",
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
