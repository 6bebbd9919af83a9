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


def scan(path):
    bad = []
    kernels = {}
    cur = None
    scales = fixups = 0  # v_div_scale_f64 / v_div_fixup_f64 seen in this kernel (two scales per division)
    for ln in open(path):
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            scales = fixups = 0
            continue
        s = ln.strip()
        op = s.split(None, 1)[0] if s and not s.startswith((";", ".")) else ""
        # The correctly rounded FP64 division (v_div_scale, v_rcp, Newton steps as FMAs,
        # v_div_fmas, v_div_fixup) returns the IEEE quotient: its FMAs are part of ONE rounded
        # operation, as in the reference's `/`, and are exempt.
        # The scheduler may interleave several divisions, so "inside" means: some division whose
        # scales were seen has not reached its fixup yet.
        if op.startswith("v_div_scale_f64"):
            scales += 1
        elif op.startswith("v_div_fixup_f64"):
            fixups += 1
        elif (op in FORBIDDEN or any(op.startswith(f + "_") for f in FORBIDDEN)) and (scales + 1) // 2 <= fixups:
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


def main(paths):
    rc = 0
    for p in paths:
        # the encoder's bit image is addressed from LDS byte 0 (scatter_bits' inline ds_or): its
        # kernels must allocate no static LDS, so the dynamic area starts there
        for name, size in static_lds(p).items():
            if "encode_kernel" in name and size != 0:
                rc = 1
                print(f"{p}: {name} allocates {size} B of static LDS (scatter_bits assumes 0)", file=sys.stderr)
        bad, kernels = scan(p)
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
