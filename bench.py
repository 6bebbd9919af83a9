#!/usr/bin/env python3
"""Benchmark: Mpixels/s of the ImageEncoder encode hot path (DCT + quant + zig-zag RLE pack) on
MI355X, with the reference's own OpenMP CPU encoder timed beside it.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|c5]

A "step" is one pass of the encoder over one batch of distinct synthetic frames resident in HBM
(a rotating set larger than the 256 MiB Infinity Cache, so HBM is what is measured):

  c2 (default at N=1)  3840x2160, 4x4 blocks, matrix.txt, RLE: a batch of independent images
  c3                   3840x2160, 8x8 blocks, matrix8_1.txt, RLE
  c4 (default at N>1)  1920x1080 gop=1 video, 4x4: 64 frames per GPU (512 at N=8), sharded over
                       the ranks and assembled into ONE stream on rank 0 (all_gather of the bit
                       counts, per-rank bit re-shift, RCCL point-to-point gather); encode and
                       gather are both timed.  At N>1 each rank's frames go in K=2 sub-batches so
                       that the gather of the first overlaps the encode of the second
                       (imageencoder_amd/dist.py PipelinedGather); at N=1 there is nothing to
                       gather and the 64 frames are one launch (K=1)
  c5                   3840x2160, 4x4, Huffman post-pass on every image (device histogram +
                       host tree build + device re-encode)

--gpus N > 1 without a torch.distributed environment re-launches itself as
``python -m torch.distributed.run --nproc-per-node N`` (this parent never touches a GPU) and
relays rank 0's line.  One process per GPU; value = all pixels encoded by all ranks / max-over-
ranks wall time of the K timed steps (inputs already resident, outputs left in HBM).

After the timed steps every run checks its own output (``bit_exact``): the reference golden md5
of the 4K synthetic image (c2/c3/c5: image 0 of the batch is that golden's frame) or, for c4, the
golden 3-frame 1080p gop=1 stream plus the assembled N-rank stream against a single-GPU encode of
the same frames; asynchronous launches are checked for look-back timeouts (ie_sync).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")  # data files (matrices, manifest of md5s)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ROUND = "r06"  # profiles/<ROUND>_traffic_<workload>.json: this round's counter passes (tools/gpu_traffic.sh)
# the dominant kernel of each workload's timed launch (launch_encode: 4x4 FAST over whole 16-byte
# groups runs encode4p_kernel; 8x8 runs encode_kernel<8>)
KERNEL = {"c2": "encode4p_kernel<false>", "c3": "encode_kernel<8,false>", "c4": "encode4p_kernel<false>",
          "c5": "encode4p_kernel<true>"}

WORKLOADS = {
    "c2": dict(w=3840, h=2160, n=4, matrix="matrix.txt", batch=16, resident=64, gen="U", huffman=False,
               golden="synU4k_4x4"),
    "c3": dict(w=3840, h=2160, n=8, matrix="matrix8_1.txt", batch=16, resident=64, gen="U", huffman=False,
               golden="synU4k_8x8"),
    # c4: batch = frames per GPU per step, split into `chunks` pipelined sub-batches: None = 1 at one
    # GPU (one launch of 64 1080p frames, 8 128 tiles: 0.260 of HBM against 0.234 for two 32-frame
    # launches, round 4) and 2 above, where the first sub-batch's gather overlaps the second's encode
    # (rank 0's ingress of the other ranks' streams, not the encode, sets the multi-GPU step)
    "c4": dict(w=1920, h=1080, n=4, matrix="matrix.txt", batch=64, resident=256, gen="U", huffman=False,
               chunks=None, golden="vidU1080x3_4x4"),
    "c5": dict(w=3840, h=2160, n=4, matrix="matrix.txt", batch=16, resident=64, gen="U", huffman=True,
               golden="synU4k_4x4_huff"),
}
METRIC = "Mpixels/s encode (DCT+quant+RLE), 4K grayscale, 1/2/4/8 GPU + CPU ref"
ARITH = "FP32 separable DCT + FP64 re-evaluation of near-tie coefficients (bit-exact vs the FP64 reference)"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                   help="default: c2 at one GPU, c4 (the multi-GPU configuration) above")
    p.add_argument("--mode", default="fast", choices=["fast", "exact"])
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--cpu-iters", type=int, default=2)
    p.add_argument("--no-decode", action="store_true", help="skip the one-image decode timing (inverse path)")
    p.add_argument("--no-gop", action="store_true", help="skip the P-frame video timing (gop > 1)")
    p.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) timing")
    p.add_argument("--no-check", action="store_true", help="skip the output self-check")
    p.add_argument("--batch", type=int, default=None, help="frames per launch (default: the workload's)")
    p.add_argument("--resident", type=int, default=None, help="distinct resident frames (default: the workload's)")
    p.add_argument("--chunks", type=int, default=None,
                   help="C4: pipelined sub-batches per step (default: 1 at one GPU, 2 at more)")
    p.add_argument("--no-single-frame", dest="single_frame", action="store_false",
                   help="skip timing one-image launches (configs[1] taken literally: one 4K frame per launch)")
    return p.parse_args()


def launch_ranks(args) -> int:
    """--gpus N outside torch.distributed: start N ranks (this process never initialises HIP)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def host_info() -> dict:
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "nproc": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": quota}


def cpu_baseline(cfg, frame: np.ndarray) -> dict | None:
    """The reference encoder itself (oracle/_ref/ref_harness, compiled from the reference sources
    with OpenMP) timed on this host on a bounded sample, OMP_NUM_THREADS = the CPUs this process
    may use (nproc, or the cgroup quota when lower): time4 runs the
    reference's ImageEncoder::process, time8 the same loop over its Block<8>.  Falls back to the
    oracle restatement (kind "port") only if the reference build is absent."""
    info = host_info()
    # every CPU this process may use: nproc, bounded by the cgroup's CPU quota where one is set
    # (the GPU box: nproc 256, quota 16 -- 256 OpenMP threads on 16 CPUs measured 8x slower)
    threads = min(info["nproc"], int(info["cgroup_cpu_quota"])) if info["cgroup_cpu_quota"] else info["nproc"]
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    w, h, n = cfg["w"], cfg["h"], cfg["n"]
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness_huff" if cfg["huffman"] else "ref_harness")
    iters = ARGS.cpu_iters
    why = "oracle/_ref not built"
    if os.path.exists(harness) and not (n == 8 and cfg["huffman"]):
        with tempfile.TemporaryDirectory() as d:
            raw = os.path.join(d, "in.raw")
            frame.tofile(raw)
            # the reference opens the matrix with std::fstream(in|out): it needs a writable copy
            mat = os.path.join(d, cfg["matrix"])
            shutil.copyfile(os.path.join(GOLDEN, cfg["matrix"]), mat)
            os.chmod(mat, 0o644)
            mode = "time4" if n == 4 else "time8"
            r = subprocess.run([harness, mode, raw, str(w), str(h), "1", mat, str(iters)],
                               env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, timeout=900)
            line = [ln for ln in r.stderr.splitlines() if ln.startswith("{")]
            why = f"ref_harness rc={r.returncode}: {r.stderr.strip()[-200:]}"
            if r.returncode == 0 and line:
                res = json.loads(line[-1])
                what = ("ImageEncoder::process" if n == 4 else
                        "ImageEncoder::process loop over its Block<8> (ImageEncoder.cpp:52-147)")
                return dict(value=round(w * h / (res["mean_ms"] * 1e3), 3), unit="Mpx/s", cores=threads,
                            kind="reference",
                            sample=f"{iters} x {w}x{h} {cfg['gen']} frame, reference {what} "
                                   f"(OpenMP{', Huffman' if cfg['huffman'] else ''}) via oracle/_ref/ref_harness "
                                   f"{mode}, OMP_NUM_THREADS={threads}, mean {res['mean_ms']:.1f} ms/frame",
                            host=info)
    # port: the oracle restatement (test infrastructure, allowed in this leg only)
    from tests import oracle_lib as O
    oracle = O.load()
    from imageencoder_amd import read_matrix
    q = read_matrix(os.path.join(GOLDEN, cfg["matrix"]), n)
    t0 = time.perf_counter()
    for _ in range(iters):
        oracle.encode_image(frame, n, q, rle=True, huffman=cfg["huffman"])
    dt = (time.perf_counter() - t0) / iters
    return dict(value=round(w * h / (dt * 1e6), 3), unit="Mpx/s", cores=threads, kind="port",
                sample=f"{iters} x {w}x{h} {cfg['gen']} frame, oracle restatement, {threads} threads",
                reference_unavailable=why, host=info)


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


def golden(name: str) -> dict:
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return {c["name"]: c for c in json.load(f)}[name]


def md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


def main():
    global ARGS
    ARGS = args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    wl = args.workload or ("c2" if world == 1 else "c4")
    cfg = WORKLOADS[wl]

    import torch
    import torch.distributed as dist

    from imageencoder_amd import (MODE_EXACT, MODE_FAST, Codec, read_matrix, stream_bound, synth,
                                  write_header)
    from imageencoder_amd import dist as D

    # IE_BENCH_BACKEND=gloo with ranks sharing the visible GPUs (local % device_count) rehearses the
    # multi-rank control flow on a box with fewer GPUs than ranks; the real run is RCCL, one GPU each
    backend = os.environ.get("IE_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
        # ranks share a GPU: concurrent look-back kernels of different processes could hold each
        # other's predecessor tiles off the CUs -- order tiles by atomic ticket (deadlock-free)
        os.environ["IE_FORCE_TICKET"] = "1"
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
    q = read_matrix(os.path.join(GOLDEN, cfg["matrix"]), n)
    codec = Codec(local, q, n)
    # a dedicated stream: the encoder's launches and the timing events share it (the default
    # stream's handle is NULL, which ie_set_stream reads as "the context's own stream")
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    codec.set_stream(stream.cuda_stream)
    mode = MODE_EXACT if args.mode == "exact" else MODE_FAST
    timer = Timer(torch, dist, dev, stream, world)
    extra = {}
    check = {}

    if wl in ("c2", "c3", "c5"):
        # resident synthetic frames, distinct per rank (seed offset), generated on the device;
        # rank 0's frame 0 is the golden synU4k frame (seed DEFAULT_SEED)
        seed = synth.DEFAULT_SEED + 1000 * rank
        frames = synth.uniform_device(w, h, R, seed, dev, torch)
        nslots = R // B
        hdr, hdr_bits = write_header(n, q, True, w, h, huffman=cfg["huffman"])
        pitch = (stream_bound(w, h, n, 1, hdr_bits) + 255) // 256 * 256
        # two output buffers in turn (the pipelined Huffman step needs both); every image's region
        # starts with its settings header (the encoder keeps the bits before start_bit)
        outs = [torch.zeros(pitch * B, dtype=torch.uint8, device=dev) for _ in range(2)]
        hdr_t = torch.from_numpy(hdr).to(dev)
        for o in outs:
            o.view(B, pitch)[:, : hdr.size].copy_(hdr_t)
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
            drain = None
        else:
            hpitch = 2 * pitch  # >= 32-bit codes x payload bytes
            houts = torch.zeros(hpitch * B, dtype=torch.uint8, device=dev)
            hsizes = []
            pending = []  # the batch whose trees + pack are still to do: (output buffer, slot)

            def drain():
                if pending:
                    out, hslot = pending.pop()
                    hsizes[:] = codec.huffman_finish_after_encode(out, pitch, B, hslot, houts, hpitch)

            def step(i):
                # a batch's Huffman pass: the byte counts (from the encoder), the first positions
                # (lengths from the encoder's end bits on the device), host tree builds, one pack
                # launch.  Pipelined: batch i's encode and histogram are issued before batch i-1's
                # trees, so the host builds those while the device encodes (two output buffers
                # alternate, so batch i never overwrites the bytes batch i-1's pack still reads)
                slot = i % nslots
                out = outs[i % len(outs)]
                # the encoder also counts the bytes it stores (the histogram of the Huffman pass)
                codec.encode_images(frames[slot * B:(slot + 1) * B], w, h, out, out_pitch=pitch,
                                    nframes=B, start_bit=hdr_bits, mode=mode, want_sizes=False, count_bytes=True)
                codec.huffman_begin_after_encode(out, pitch, B, i % 2)
                drain()
                pending.append((out, i % 2))
        wall, gpu_s = timer.run(step, args.warmup, args.steps, drain=drain)
        codec.sync()  # raises if any asynchronous launch of the timed region timed out
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
            # the Huffman pass's own kernels, timed by HIP events inside the library around its
            # launches (ie_last_stage_ms): the first-occurrence / histogram stage (the byte counts
            # themselves come from the counting encoder) and the pack; algorithmic bytes = the
            # payload bytes the pack reads + the Huffman bytes it writes
            th, tp, nin, nout = [], [], 0, 0
            codec.set_stage_timing(True)  # (outside the timed region: the events cost the step time)
            for i in range(5):
                slot = i % nslots
                codec.encode_images(frames[slot * B:(slot + 1) * B], w, h, outs[0], out_pitch=pitch, nframes=B,
                                    start_bit=hdr_bits, mode=mode, want_sizes=False, count_bytes=True)
                codec.huffman_begin_after_encode(outs[0], pitch, B, 0)
                th.append(codec.last_stage_ms(0))
                hs = codec.huffman_finish_after_encode(outs[0], pitch, B, 0, houts, hpitch)
                tp.append(codec.last_stage_ms(1))
                eb = ends_per_slot[slot]
                nin += sum((int(e) + 7) // 8 for e in eb)
                nout += sum(int(x) for x in hs)
            codec.set_stage_timing(False)
            t_h, t_p = float(np.median(th)) / 1e3, float(np.median(tp)) / 1e3
            hbytes = (nin + nout) / 5
            # the counting encoder the step really runs (encode_kernel<4,HIST>: it also counts the
            # bytes it stores), timed alone on the same stream
            def enc_counted(i):
                slot = i % nslots
                codec.encode_images(frames[slot * B:(slot + 1) * B], w, h, outs[i % len(outs)], out_pitch=pitch,
                                    nframes=B, start_bit=hdr_bits, mode=mode, want_sizes=False, count_bytes=True)
            _, g3 = timer.run(enc_counted, 1, args.steps)
            t_cnt = g3 / args.steps
            # the roofline prices the launch the step runs (the counting encoder); the plain encoder
            # (same kernel without the byte counts) is reported beside it
            extra["plain_encode"] = {"kernel": "encode4p_kernel<false>", "launch_us": round(enc_s * 1e6, 2),
                                     "frac": round((B * w * h + out_bytes_per_launch) / enc_s / 1e9 / HBM_PEAK_GBS, 4)}
            enc_s = t_cnt
            extra["huffman_roofline"] = {
                "bound": "hbm", "achieved": round(hbytes / (t_h + t_p) / 1e9, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(hbytes / (t_h + t_p) / 1e9 / HBM_PEAK_GBS, 4),
                "kernels": "first-occurrence/histogram stage + pack_kernel", "alg_bytes_per_batch": int(hbytes),
                "hist_us": round(t_h * 1e6, 2), "pack_us": round(t_p * 1e6, 2),
                "note": "payload bytes read by the pack + Huffman bytes written, per 16-image batch; the byte "
                        "counts are taken by the encoder as it stores (its launch is the line's roofline)"}
            # the inverse of the Huffman pass: image 0's Huffman stream decoded back
            # to payload bytes, device-resident (ie_huffman_decode: table walk + composition + count +
            # emit kernels), wall time per call incl. its host sync
            hs0 = codec.huffman_encode_after_encode(outs[0], pitch, B, houts, hpitch)
            henc = houts[: hs0[0]].cpu().numpy().tobytes()
            tab = codec.huffman_table(henc)
            if tab is not None:
                lut, hsb = tab
                dlut = torch.from_numpy(lut.view(np.int16).copy()).to(dev)
                denc = houts[: hs0[0]]
                dsym = torch.zeros(8 * len(henc) + 64, dtype=torch.uint8, device=dev)
                nsym = codec.huffman_decode_device(denc, len(henc), dlut, hsb, dsym)
                torch.cuda.synchronize(dev)
                kh = 10
                t0 = time.perf_counter()
                for _ in range(kh):
                    codec.huffman_decode_device(denc, len(henc), dlut, hsb, dsym)
                torch.cuda.synchronize(dev)
                thd = (time.perf_counter() - t0) / kh
                hb_dec = len(henc) + nsym
                extra["huffman_decode"] = {"us": round(thd * 1e6, 1), "symbols": nsym, "stream_bytes": len(henc),
                                           "achieved_GBps": round(hb_dec / thd / 1e9, 1),
                                           "frac": round(hb_dec / thd / 1e9 / HBM_PEAK_GBS, 4),
                                           "note": "Huffman stream read + symbols written per call, wall time incl. "
                                                   "its one host sync (device output: the emit is bounded by the "
                                                   "output size, then the total and flags are read back together)"}
        if args.single_frame:  # one 4K frame per launch: the latency of the single-image configuration
            one = outs[0][:pitch]

            def single(i):
                f = i % R
                codec.encode_images(frames[f:f + 1], w, h, one, out_pitch=pitch, nframes=1, start_bit=hdr_bits,
                                    mode=mode, want_sizes=False)
            _, g1 = timer.run(single, 2, 4 * B)
            extra["single_frame"] = {"us_per_frame": round(g1 / (4 * B) * 1e6, 2),
                                     "Mpx_s": round(w * h / (g1 / (4 * B)) / 1e6, 1)}
        codec.sync()
        if not args.no_check and rank == 0:
            # image 0 of slot 0 is the reference's golden 4K frame: its file md5
            g = golden(cfg["golden"])
            out = outs[0]
            ends = codec.encode_images(frames[:B], w, h, out, out_pitch=pitch, nframes=B, start_bit=hdr_bits,
                                       mode=mode)
            if cfg["huffman"]:
                sizes = codec.huffman_encode_after_encode(out, pitch, B, houts, hpitch)
                got = houts[: sizes[0]].cpu().numpy().tobytes()
            else:
                got = out[: (int(ends[0]) + 7) // 8].cpu().numpy().tobytes()
            check = {"golden": cfg["golden"], "md5": md5(got), "expected_md5": g["md5"],
                     "bit_exact": md5(got) == g["md5"] and len(got) == g["size"]}
        if not cfg["huffman"] and not args.no_e2e:
            # end to end from HOST buffers (reported separately, never `value`): host frames
            # in, host streams out, through the streamed path (chunks in flight on three HIP
            # streams, PCIe full duplex).  Pageable numpy buffers go through the library's pinned
            # slots; pinned ones (ie_host_alloc) are DMA'd directly.  Each variant's streams are
            # checked against the device-resident batch above.
            yh = frames[:B].cpu().numpy()
            dref = codec.encode_images(frames[:B], w, h, outs[0], out_pitch=pitch, nframes=B, start_bit=hdr_bits,
                                       mode=mode)
            ref0 = outs[0][: (int(dref[0]) + 7) // 8].cpu().numpy()
            e2e = {}
            for kind in ("pageable", "pinned"):
                if kind == "pinned":
                    yk = codec.host_array(yh.size)
                    yk[:] = yh.ravel()
                    ok = codec.host_array(pitch * B)
                    ok[:] = 0
                else:
                    yk, ok = yh, np.zeros(pitch * B, dtype=np.uint8)
                ok.reshape(B, pitch)[:, : hdr.size] = hdr  # each image's settings header
                ends_h = codec.encode_images(yk, w, h, ok, out_pitch=pitch, nframes=B, start_bit=hdr_bits, mode=mode)
                same = list(ends_h) == list(dref) and bytes(ok[: ref0.size]) == ref0.tobytes()
                ke = 5
                t0 = time.perf_counter()
                for _ in range(ke):
                    codec.encode_images(yk, w, h, ok, out_pitch=pitch, nframes=B, start_bit=hdr_bits, mode=mode)
                te = (time.perf_counter() - t0) / ke
                e2e[kind] = {"ms_per_batch": round(te * 1e3, 2), "Mpx_s": round(B * w * h / te / 1e6, 1),
                             "host_GBps": round((yh.nbytes + sum((int(e) + 7) // 8 for e in ends_h)) / te / 1e9, 1),
                             "same_as_device": same}
            extra["e2e_host_buffers"] = dict(e2e, note="host frames in, host streams out: streamed path (H2D, "
                                                       "encode, D2H of consecutive chunks concurrent); "
                                                       "PCIe-inclusive, never `value`")
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
            chunks, groups = codec.last_decode_info()
            dec_bytes = nb0 + w * h  # the stream read + the pixels written
            extra["decode_one_image"] = {"us": round(td * 1e6, 1), "Mpx_s": round(w * h / td / 1e6, 1),
                                         "achieved_GBps": round(dec_bytes / td / 1e9, 1),
                                         "frac": round(dec_bytes / td / 1e9 / HBM_PEAK_GBS, 4),
                                         "path": f"exact parse: {chunks} chunk transfer tables composed in "
                                                 f"{groups} level(s), then count and decode launches; "
                                                 "one host sync at the end (device-resident stream and pixels)"}
        if n == 4 and not cfg["huffman"] and not args.no_gop:
            # P-frames: 8 resident frames as one video, gop = 1 against gop = 8
            # (one I-frame + 7 P-frames: macroblock search + coded error + reconstruction), merange 16
            F, mer = 8, 16
            vf = frames[:F]
            vcap = codec.gop_stream_bound(w, h, F, mer, 0)
            vout = torch.zeros(vcap, dtype=torch.uint8, device=dev)
            tv = {}
            for gop in (1, F):
                codec.encode_gop(vf, w, h, vout, gop, mer, nframes=F, mode=mode)
                torch.cuda.synchronize(dev)
                kv = 5
                t0 = time.perf_counter()
                for _ in range(kv):
                    vout.zero_()
                    codec.encode_gop(vf, w, h, vout, gop, mer, nframes=F, mode=mode)
                torch.cuda.synchronize(dev)
                tv[gop] = (time.perf_counter() - t0) / kv
            tp = max(tv[F] - tv[1] / F, 0.0) / (F - 1)
            extra["video_gop"] = {"frames": F, "gop": F, "merange": mer, "ms_gop1": round(tv[1] * 1e3, 3),
                                  "ms_gop": round(tv[F] * 1e3, 3), "us_per_pframe": round(tp * 1e6, 1),
                                  "pframe_Mpx_s": round(w * h / tp / 1e6, 1) if tp else None,
                                  "note": "ie_encode_gop, device-resident frames and stream, one host sync per "
                                          "call (stream zeroing included)"}
        workload = (f"{wl}: {w}x{h} {n}x{n} {cfg['matrix']} RLE"
                    f"{' +Huffman' if cfg['huffman'] else ''}, batch of {B} independent images per step, "
                    f"{R} distinct resident frames per GPU ({R * w * h / 2**20:.0f} MiB)")
        parallelism = f"independent images sharded x{world} (no collective)"
        cpu_frame = frames[0].cpu().numpy() if rank == 0 else None
    else:  # c4: one gop=1 video stream, frames sharded over ranks, RCCL gather to rank 0
        K = args.chunks or cfg["chunks"] or (1 if world == 1 else 2)
        m = max(B // K, 1)  # frames per rank per chunk
        nloc = m * K
        F = nloc * world
        nsets = max(R // nloc, 1)  # distinct resident batches per rank
        # resident frames: set p, global frame g of the batch -> seed DEFAULT_SEED + p*F + g
        frames = torch.empty((nsets, nloc, h, w), dtype=torch.uint8, device=dev)
        for p in range(nsets):
            for k in range(K):
                fr = D.chunk_frames(k, rank, world, F, K)
                frames[p, k * m:(k + 1) * m].copy_(
                    synth.uniform_device(w, h, m, synth.DEFAULT_SEED + p * F + fr.start, dev, torch))
        hdr, hb = write_header(n, q, True, w, h, video=True, frames=F, gop=1, merange=16)
        root_cap = stream_bound(w, h, n, F, hb) + 64
        seg_cap = stream_bound(w, h, n, m, 0) + 64
        comm = torch.cuda.Stream(dev)
        shifter = Codec(local, q, n)  # its own context: the bit copies run beside the encodes
        shifter.set_stream(comm.cuda_stream)
        gloo = world > 1 and dist.get_backend() == "gloo"

        def encode(k, i, seg, bits):
            codec.encode_frames(frames[i % nsets, k * m:(k + 1) * m], w, h, seg, start_bit=0, nframes=m,
                                mode=mode, want_sizes=False)
            codec.end_bits_into(bits)

        def shift(src, nbytes, start, dst):
            shifter.bitcopy(src[:nbytes], dst, start)

        if world > 1:
            G = D.PipelinedGather(dist, rank, world, F, K, hdr, hb, seg_cap, root_cap, encode, shift, dev,
                                  comm_dev="cpu" if gloo else None, enc_stream=stream, comm_stream=comm)
            wall, _ = timer.run(G.step, args.warmup, args.steps)
            total_bits = G.total
            segs = G.segs
        else:  # one GPU: the whole batch in one launch straight after the header (nothing to gather)
            out_root = torch.zeros(root_cap, dtype=torch.uint8, device=dev)
            out_root[: hdr.size].copy_(torch.from_numpy(hdr).to(dev))
            segs = [torch.zeros(seg_cap, dtype=torch.uint8, device=dev) for _ in range(K)]
            wall, _ = timer.run(lambda i: codec.encode_frames(frames[i % nsets].view(nloc, h, w), w, h, out_root,
                                                              start_bit=hb, nframes=nloc, mode=mode,
                                                              want_sizes=False), args.warmup, args.steps)
            total_bits = codec.encode_frames(frames[0], w, h, out_root, start_bit=hb, nframes=nloc, mode=mode)[1]
        codec.sync()
        shifter.sync()
        # the encoder launches alone (no gather): the dominant kernel's time
        def enc_only(i):
            for k in range(K):
                codec.encode_frames(frames[i % nsets, k * m:(k + 1) * m], w, h, segs[k], start_bit=0, nframes=m,
                                    mode=mode, want_sizes=False)
        wall_enc, gpu_enc = timer.run(enc_only, 1, args.steps)
        codec.sync()
        px_total = world * args.steps * nloc * w * h
        extra["encode_only_Mpx_s"] = round(px_total / wall_enc / 1e6, 2)
        extra["stream_bytes"] = (total_bits + 7) // 8
        extra["world_size_backend"] = {"world": dist.get_world_size() if world > 1 else 1,
                                       "backend": dist.get_backend() if world > 1 else None}
        in_bytes_per_launch = m * w * h
        out_bytes_per_launch = extra["stream_bytes"] / (world * K)
        enc_s = gpu_enc / (args.steps * K)
        fallbacks = codec.last_fallbacks()
        if not args.no_check:
            ok = True
            if world > 1:
                # the assembled stream of the last step vs ONE device encoding the same F frames
                last = (args.warmup + args.steps - 1) % nsets
                G.step(last)
                torch.cuda.synchronize(dev)
                if rank == 0:
                    allf = synth.uniform_device(w, h, F, synth.DEFAULT_SEED + last * F, dev, torch)
                    ref = torch.zeros(root_cap, dtype=torch.uint8, device=dev)
                    ref[: hdr.size].copy_(torch.from_numpy(hdr).to(dev))
                    _, end = codec.encode_frames(allf, w, h, ref, start_bit=hb, nframes=F, mode=mode)
                    nbytes = (end + 7) // 8
                    ok = end == G.total and torch.equal(ref[:nbytes], G.out[:nbytes])
                    check["gathered_equals_single_gpu"] = bool(ok)
                    del allf, ref
            if rank == 0:
                # the golden gop=1 stream (3 x 1080p YUV420 frames) through the same encoder
                g = golden(cfg["golden"])
                gy = torch.from_numpy(synth.frames("U", w, h, 3, seed=g["input"]["seed"])).to(dev)
                ghdr, ghb = write_header(n, q, True, w, h, video=True, frames=3, gop=1, merange=16)
                gout = torch.zeros(stream_bound(w, h, n, 3, ghb) + 64, dtype=torch.uint8, device=dev)
                gout[: ghdr.size].copy_(torch.from_numpy(ghdr).to(dev))
                _, gend = codec.encode_frames(gy, w, h, gout, start_bit=ghb, nframes=3, mode=mode)
                got = gout[: (gend + 7) // 8].cpu().numpy().tobytes()
                check.update({"golden": cfg["golden"], "md5": md5(got), "expected_md5": g["md5"]})
                check["bit_exact"] = bool(ok and md5(got) == g["md5"])
        B = nloc
        if world > 1:
            workload = (f"c4: {F} x {w}x{h} gop=1 video ({nloc} frames per GPU in {K} sub-batches of {m}), "
                        f"{n}x{n} {cfg['matrix']} RLE, ONE stream assembled on rank 0 (all_gather of sizes + bit "
                        f"re-shift + P2P gather" + (", each sub-batch's gather overlapped with the next one's encode)"
                                                   if K > 1 else ", after the encode: one sub-batch, no overlap)"))
        else:
            workload = (f"c4: {F} x {w}x{h} gop=1 video, {n}x{n} {cfg['matrix']} RLE, ONE stream: all {nloc} frames "
                        f"in {'one launch' if K == 1 else f'{K} launches'} on one GPU (nothing to gather)")
        parallelism = (f"frame-sharded x{world} + {'RCCL' if not gloo else 'gloo (rehearsal)'} gather" if world > 1
                       else "one GPU, whole batch in one launch (no collective)")
        cpu_frame = frames[0, 0].cpu().numpy() if rank == 0 else None

    value = px_total / wall / 1e6
    alg_bytes = in_bytes_per_launch + out_bytes_per_launch
    achieved = alg_bytes / enc_s / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(cfg, cpu_frame)

    if rank == 0:
        traffic = None
        tf = os.path.join(ROOT, "profiles", f"{ROUND}_traffic_{wl}.json")  # this round's passes only
        if os.path.exists(tf):
            traffic = json.load(open(tf)).get("hbm_bytes_per_launch")
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mpx/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8->int16 (FP32 DCT + FP64 near-tie fix-up)" if mode == MODE_FAST else "u8->int16 (FP64 DCT)",
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
                "traffic_file": os.path.relpath(tf, ROOT) if traffic is not None else None,
                "kernel": KERNEL[wl],
                "alg_bytes_per_launch": int(alg_bytes),
                "launch_us": round(enc_s * 1e6, 2),
                "read_only_frac": round(in_bytes_per_launch / enc_s / 1e9 / HBM_PEAK_GBS, 4),
            },
            "cpu_baseline": cpu,
            "bit_exact": check.get("bit_exact"),
            "check": check,
            "fallback_coefs_per_launch": fallbacks,
            "arith": ARITH,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
