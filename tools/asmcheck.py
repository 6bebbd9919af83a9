#!/usr/bin/env python3
"""Guard for SURVEY Appendix C.4 ("no FMA and no re-association in exact mode"): scan the gfx950
assembly of the encode / decode kernels and fail if any FP64 fused multiply-add was emitted.

The reference evaluates every FP64 product and sum with its own rounding (algo.cpp:314-325,
:348-358); hipcc contracts a*b+c into v_fma_f64 by default, which changes results at exact
rounding ties.  The kernels are built with -ffp-contract=off; this check proves it held.  It also
reports each kernel's VGPR count, scratch size and occupancy so register spills show up in the
CPU build.

    python3 tools/asmcheck.py build/asm/ie_encode.s [build/asm/ie_decode.s ...] [csrc/*.hip ...]

It also rejects 64-bit LDS atomics in the ISA and 64/96/128-bit DS instructions in the inline asm
of the given source files (DS_ATOMIC64 below).
"""
import re
import sys

FORBIDDEN = ("v_fma_f64", "v_fmac_f64", "v_fma_mix", "v_pk_fma_f64")

# LDS atomics on 64-bit data need an 8-byte aligned address; at a 4-byte aligned one the SQ raises a
# memory violation and the whole queue aborts (round 5: one `ds_or_b64` at a word-aligned bit-image
# address -- HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION on the first launch, twice; gone with the
# same field as two `ds_or_b32`).  The kernels need none, so the rule is absolute: no 64-bit DS
# atomic in any kernel's ISA, and no 64/96/128-bit DS mnemonic in hand-written inline asm, whose
# addresses the compiler cannot check (compiler-generated wide DS reads/writes come from naturally
# aligned types; a misaligned one is replayed, not faulted -- SQ_LDS_UNALIGNED_STALL, profiled).
DS_ATOMIC64 = re.compile(r"^ds_(add|sub|rsub|inc|dec|min|max|and|or|xor|mskor|wrxchg|wrxchg2|wrxchg2st64|cmpst|"
                         r"cmpswap|condxchg32|wrap|append|consume)(_rtn)?_(u64|i64|b64|f64)\b")
DS_WIDE = re.compile(r"\bds_\w+_(b64|b96|b128|u64|i64|f64)\b")


def inline_asm_wide_ds(paths):
    """(file, line, text) of every inline-asm string in the given sources naming a 64/96/128-bit DS
    instruction."""
    hits = []
    for path in paths:
        for i, ln in enumerate(open(path), 1):
            code = ln.split("//", 1)[0]
            if "asm" in code and DS_WIDE.search(code):
                hits.append((path, i, ln.strip()))
    return hits


def _regs(operands):
    """Register names of an instruction's operands (modifiers stripped): 'v[16:17]', 's[22:23]'."""
    out = []
    for o in operands:
        o = o.strip().lstrip("-").strip("|")
        if re.match(r"^[vs](\[\d+:\d+\]|\d+)$", o):
            out.append(o)
    return out


# A correctly rounded FP64 division on gfx950 is v_div_scale_f64 x2, v_rcp_f64, two Newton
# rounds on the reciprocal (v_fma_f64 error + v_fmac_f64 update each), v_mul_f64, one residual
# v_fma_f64, v_div_fmas_f64, v_div_fixup_f64: its five fused ops are part of ONE IEEE-rounded
# operation, as the reference's `/`, and are exempt -- but only those:
DIV_FMAS = 5


def scan(path):
    bad = []
    kernels = {}
    cur = None
    for ln in open(path):
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            scales = fixups = 0   # v_div_scale_f64 / v_div_fixup_f64 seen (two scales per division)
            exempt = 0            # FMAs accepted as division steps so far in this kernel
            taint = set()         # registers written by an open division's scale / rcp / steps
            continue
        s = ln.strip()
        op = s.split(None, 1)[0] if s and not s.startswith((";", ".")) else ""
        if op and DS_ATOMIC64.match(op):
            bad.append((cur, "64-bit LDS atomic: " + s))
        args = s.split(None, 1)[1].split(",") if op and len(s.split(None, 1)) > 1 else []
        regs = _regs(args)
        fused = op in FORBIDDEN or any(op.startswith(f + "_") for f in FORBIDDEN)
        # "inside a division": some division whose scales were seen has not reached its fixup yet
        # (the scheduler may interleave several).  An FMA there is a division step only if it reads
        # a register the division's own scale / rcp / earlier steps wrote, and no division may
        # carry more than its DIV_FMAS steps: a contracted a*b+c scheduled into the window is not.
        if op.startswith(("v_div_scale_f64", "v_rcp_f64")) and regs:
            scales += op.startswith("v_div_scale_f64")
            taint.add(regs[0])
        elif op.startswith("v_div_fixup_f64"):
            fixups += 1
            if (scales + 1) // 2 <= fixups:
                taint.clear()
        elif fused:
            inside = (scales + 1) // 2 > fixups
            step = inside and any(r in taint for r in regs[1:]) and exempt < DIV_FMAS * ((scales + 1) // 2)
            if step:
                exempt += 1
                taint.add(regs[0])
            else:
                bad.append((cur, s))
        if cur:
            for key in ("NumVgprs", "ScratchSize", "Occupancy"):
                m = re.match(rf"^; {key}: (\d+)", s)
                if m:
                    kernels[cur][key] = int(m.group(1))
    return bad, kernels


def static_lds(path):
    """{kernel: group_segment_fixed_size} from the code object metadata."""
    txt = open(path).read()
    k = txt.find("amdhsa.kernels")
    out = {}
    for ent in txt[k:].split("\n  - ")[1:] if k >= 0 else []:
        m = re.search(r"\.name:\s+(\S+)", ent)
        g = re.search(r"\.group_segment_fixed_size:\s+(\d+)", ent)
        if m and g:
            out[m.group(1)] = int(g.group(1))
    return out


# Register budgets of the hot kernels (occupancy >= waves per SIMD, scratch bytes <= limit): a
# change that makes the compiler spill or drop a wave shows up in the CPU build, not only on a GPU
# (an unguarded profiling branch once took the 8x8 kernel from 68 to 308 B of scratch, 2x slower).
BUDGETS = {
    "_ZN2ie13encode_kernelILi4ELb0ELb0ELi4EEEvNS_7EncArgsEPKNS_9EncTablesE": (5, 0),
    "_ZN2ie13encode_kernelILi8ELb0ELb0ELi1EEEvNS_7EncArgsEPKNS_9EncTablesE": (4, 0),
    "_ZN2ie15encode4w_kernelILb0EEEvNS_7EncArgsEPKNS_9EncTablesE": (6, 0),
    "_ZN2ie15encode4w_kernelILb1EEEvNS_7EncArgsEPKNS_9EncTablesE": (6, 0),
    "_ZN2ie15encode4p_kernelILb0EEEvNS_7EncArgsEPKNS_9EncTablesE": (6, 0),
    "_ZN2ie15encode4p_kernelILb1EEEvNS_7EncArgsEPKNS_9EncTablesE": (6, 0),
}
def main(paths):
    rc = 0
    srcs = [a for a in paths if a.endswith((".hip", ".h", ".hpp", ".cpp"))]
    paths = [a for a in paths if a not in srcs]
    for f, i, t in inline_asm_wide_ds(srcs):
        rc = 1
        print(f"{f}:{i}: 64/96/128-bit DS instruction in inline asm (alignment unchecked): {t}", file=sys.stderr)
    if srcs and rc == 0:
        print(f"{len(srcs)} source files: no wide DS instruction in inline asm")
    for p in paths:
        # the encoder's bit image is addressed from LDS byte 0 (scatter_bits' inline ds_or): its
        # kernels must allocate no static LDS, so the dynamic area starts there
        for name, size in static_lds(p).items():
            if ("encode_kernel" in name or "encode4w_kernel" in name or "encode4p_kernel" in name) and size != 0:
                rc = 1
                print(f"{p}: {name} allocates {size} B of static LDS (scatter_bits assumes 0)", file=sys.stderr)
        bad, kernels = scan(p)
        if "encode" in p and not any(k in kernels for k in BUDGETS):
            rc = 1
            print(f"{p}: none of the budgeted encode kernels found (renamed? update BUDGETS)", file=sys.stderr)
        for name, (waves, scratch) in BUDGETS.items():
            info = kernels.get(name)
            if info and (info.get("Occupancy", 0) < waves or info.get("ScratchSize", 0) > scratch):
                rc = 1
                print(f"{p}: {name[:60]} over budget: occupancy {info.get('Occupancy')} (>= {waves}), "
                      f"scratch {info.get('ScratchSize')} B (<= {scratch})", file=sys.stderr)
        for name, info in kernels.items():
            if info:
                print(f"{p}: {name[:70]:70s} vgpr={info.get('NumVgprs')} scratch={info.get('ScratchSize')} "
                      f"occupancy={info.get('Occupancy')}")
        if bad:
            rc = 1
            for k, s in bad[:20]:
                print(f"{p}: {'' if s.startswith('64-bit LDS') else 'FP64 FMA '}in {k}: {s}", file=sys.stderr)
            print(f"{p}: {len(bad)} forbidden instructions (fused FP64: reference order violated; 64-bit "
                  f"LDS atomics: alignment faults)", file=sys.stderr)
        else:
            print(f"{p}: no fused FP64 instructions")
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
