#!/usr/bin/env python3
"""Guard for SURVEY Appendix C.4 ("no FMA and no re-association in exact mode"): scan the gfx950
assembly of the encode / decode kernels and fail if any FP64 fused multiply-add was emitted.

The reference evaluates every FP64 product and sum with its own rounding (algo.cpp:314-325,
:348-358); hipcc contracts a*b+c into v_fma_f64 by default, which changes results at exact
rounding ties.  The kernels are built with -ffp-contract=off; this check proves it held.  It also
reports each kernel's VGPR count, scratch size and occupancy so register spills show up in the
CPU build.

    python3 tools/asmcheck.py build/asm/ie_encode.s [build/asm/ie_decode.s ...]
"""
import re
import sys

FORBIDDEN = ("v_fma_f64", "v_fmac_f64", "v_fma_mix", "v_pk_fma_f64")


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
    "_ZN2ie15encode4p_kernelILb0ELi4EEEvNS_7EncArgsEPKNS_9EncTablesE": (6, 0),
    "_ZN2ie15encode4p_kernelILb1ELi4EEEvNS_7EncArgsEPKNS_9EncTablesE": (6, 0),
    "_ZN2ie15encode4p_kernelILb0ELi8EEEvNS_7EncArgsEPKNS_9EncTablesE": (6, 0),
    "_ZN2ie15encode4q_kernelENS_7EncArgsEPKNS_9EncTablesE": (4, 0),
}
# Persistent kernels: the host sizes the grid as (workgroups per CU) x CUs with workgroups per CU
# = min(occupancy API, PERSIST[name]); every one of them must be resident at once (static tile
# order), so the SGPR admission rule (MI355X_MICROARCH.md, Residency: 256-thread blocks per CU <=
# floor(800 / (ceil(sgpr / 16) * 16 + 16))) must admit at least that many.
PERSIST = {
    "_ZN2ie15encode4p_kernelILb0ELi4EEEvNS_7EncArgsEPKNS_9EncTablesE": 6,
    "_ZN2ie15encode4p_kernelILb1ELi4EEEvNS_7EncArgsEPKNS_9EncTablesE": 6,
    "_ZN2ie15encode4q_kernelENS_7EncArgsEPKNS_9EncTablesE": 4,
}


def sgpr_counts(path):
    """{kernel: .sgpr_count} from the code object metadata."""
    txt = open(path).read()
    k = txt.find("amdhsa.kernels")
    out = {}
    for ent in txt[k:].split("\n  - ")[1:] if k >= 0 else []:
        m = re.search(r"\.name:\s+(\S+)", ent)
        g = re.search(r"\.sgpr_count:\s+(\d+)", ent)
        if m and g:
            out[m.group(1)] = int(g.group(1))
    return out


def main(paths):
    rc = 0
    for p in paths:
        # the encoder's bit image is addressed from LDS byte 0 (scatter_bits' inline ds_or): its
        # kernels must allocate no static LDS, so the dynamic area starts there
        for name, size in static_lds(p).items():
            if ("encode_kernel" in name or "encode4w_kernel" in name or "encode4p_kernel" in name or "encode4q_kernel" in name) and size != 0:
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
        sg = sgpr_counts(p)
        for name, per_cu in PERSIST.items():
            if name in sg:
                admit = 800 // ((sg[name] + 15) // 16 * 16 + 16)
                if admit < per_cu:
                    rc = 1
                    print(f"{p}: {name[:60]} sgpr_count {sg[name]} admits {admit} workgroups per CU "
                          f"< {per_cu} (the persistent grid would not be resident)", file=sys.stderr)
        for name, info in kernels.items():
            if info:
                print(f"{p}: {name[:70]:70s} vgpr={info.get('NumVgprs')} scratch={info.get('ScratchSize')} "
                      f"occupancy={info.get('Occupancy')}")
        if bad:
            rc = 1
            for k, s in bad[:20]:
                print(f"{p}: FP64 FMA in {k}: {s}", file=sys.stderr)
            print(f"{p}: {len(bad)} fused FP64 instructions (reference order violated)", file=sys.stderr)
        else:
            print(f"{p}: no fused FP64 instructions")
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
