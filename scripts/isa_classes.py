#!/usr/bin/env python3
"""Issue-cost classes of a kernel's VALU instructions, from its ISA.

The PMC counters split a launch's VALU instructions into f64 add/mul/fma, int64, cvt,
transcendentals, f32 add/mul/fma and int32, plus an unnamed rest (moves, selects, compares,
logic, lane moves).  The microbenchmark (scripts/microbench/valu_ceiling.hip,
profiles/r05/valu_ceiling_summary.json) measured that only all-VGPR v_fma/add/mul_f32,
v_add_u32, v_and_b32 and v_mov_b32 pair (~2.3 cycles per wave instruction at >= 2 waves per
SIMD); v_cndmask, v_cmp, v_max, v_med3, v_bfe, v_lshl_add, v_add_co, v_mul_lo, any op with an
SGPR operand, packed f32, f64, cvt take a quad-cycle (~4.2); transcendentals 2 / 4.  This script
reads the kernel's instructions in the hot loops (basic blocks LLVM marks as inside a loop,
`; in Loop:` / `Loop Header`), classifies every VALU instruction into the PMC's classes and
into measured-pairable / measured-unpaired / unmeasured, and writes, per PMC class, the share
of its instructions that pair.  bench.py applies those shares to the profile's dynamic class
counts: the class-priced peak ("exact": the mix at the measured costs) beside the optimistic one
(every instruction outside the f64 / int64 / cvt / transcendental classes priced as pairable).
Unmeasured 32-bit mnemonics (v_sub_f32, v_fmac_f32, v_or/xor_b32, v_lshlrev_b32, ...) are
counted both ways: `pair_share` prices them unpaired (the exact peak is at most this
optimistic), `pair_share_if_vop2_pairs` pairs the VOP2-encoded ones.

usage: scripts/isa_classes.py <kernel.s> <kernel symbol> <out.json>
  (kernel.s: hipcc --offload-arch=gfx950 ... --cuda-device-only -S csrc/rtx_park.hip)
"""
import collections
import json
import re
import sys

PAIRABLE = {"v_fma_f32", "v_add_f32", "v_mul_f32", "v_add_u32", "v_and_b32", "v_mov_b32"}
MEASURED_UNPAIRED = {"v_cndmask_b32", "v_mul_lo_u32", "v_mad_u64_u32", "v_pk_fma_f32", "v_cmp", "v_max_f32",
                     "v_med3_f32", "v_add_co_u32", "v_lshl_add_u32", "v_bfe_u32", "v_mul_u32_u24"}
F64 = re.compile(r"^v_(add|mul|fma|fmac)_f64$")
TRANS = re.compile(r"^v_(rcp|rsq|sqrt|sin|cos|exp|log|rcp_iflag)_")
INT64 = re.compile(r"^v_(lshl_add_u64|lshlrev_b64|lshrrev_b64|ashrrev_i64|mov_b64|mad_u64_u32|mad_i64_i32|add_u64)")
F32 = re.compile(r"^v_(add|sub|subrev|mul|fma|fmac|mad|fmaak|fmamk)_f32$")
INT32 = re.compile(r"^v_(add|sub|subrev|add3|mul_lo|mul_hi|mul|lshl_add|add_lshl|lshl_or|and_or|lshlrev|lshrrev|ashrrev|"
                   r"and|or|xor|or3|xad|bfe|bfi|bitop3|not|add_co|sub_co|subrev_co|addc_co|subb_co|subbrev_co|alignbit|"
                   r"perm|min|max)_(u32|i32|b32|u16|i16)")
INLINE_F = {"0.5", "-0.5", "1.0", "-1.0", "2.0", "-2.0", "4.0", "-4.0", "0.15915494"}


def base(mn):
    return re.sub(r"_e(32|64|64_dpp|32_dpp|64_sdwa|32_sdwa)$", "", mn)


def pmc_class(b):
    if F64.match(b):
        return "f64"
    if b.startswith("v_cvt_"):
        return "cvt"
    if TRANS.match(b):
        return "trans64" if b.endswith("f64") else "trans32"
    if INT64.match(b):
        return "int64"
    if F32.match(b):
        return "f32"
    if INT32.match(b):
        return "int32"
    return "other"


def operands_plain(ops):
    """True when every source operand is a VGPR or an inline constant (no SGPR, vcc, literal)."""
    for o in ops[1:]:
        o = o.strip()
        if re.match(r"^-?\|?v(\d+|\[\d+:\d+\])\|?$", o):
            continue
        if re.match(r"^-?\d+$", o) and -16 <= int(o) <= 64:
            continue
        if o in INLINE_F:
            continue
        return False
    return True


def main():
    src, sym, out = sys.argv[1:4]
    lines = open(src).read().splitlines()
    try:
        start = next(i for i, line in enumerate(lines) if line.startswith(sym + ":"))
    except StopIteration:
        sys.exit(f"{sym} not found")
    in_loop = False
    counts = {k: collections.Counter() for k in ("all", "loop")}
    for line in lines[start + 1:]:
        if line.startswith(".Lfunc_end"):
            break
        s = line.strip()
        if s.startswith(".LBB") or s.startswith("; %bb"):
            in_loop = "in Loop:" in line or "Loop Header" in line
            continue
        if not s.startswith("v_"):
            continue
        mn, _, rest = s.partition(" ")
        b = base(mn)
        if b in ("v_readlane_b32", "v_writelane_b32", "v_readfirstlane_b32", "v_nop"):
            kind = "unpaired_lane"
        else:
            ops = [o for o in rest.split("//")[0].split(",") if o.strip()]
            plain = operands_plain(ops)
            if b in PAIRABLE and plain:
                kind = "pairable"
            elif b in PAIRABLE or b in MEASURED_UNPAIRED or b.startswith("v_cmp") or pmc_class(b) != "other" and \
                    pmc_class(b) not in ("f32", "int32"):
                kind = "unpaired"
            elif mn.endswith("_e32") and plain:
                kind = "unmeasured_vop2"
            else:
                kind = "unmeasured_other"
        c = pmc_class(b)
        for k in ("all",) + (("loop",) if in_loop else ()):
            counts[k][(c, kind)] += 1
    res = {"source": src, "kernel": sym, "note": __doc__.split("\n\n")[1].replace("\n", " ")}
    for k, cnt in counts.items():
        per = collections.defaultdict(collections.Counter)
        for (c, kind), n in cnt.items():
            per[c][kind] += n
        res[k] = {c: {"static": sum(v.values()), **v,
                      "pair_share": v["pairable"] / sum(v.values()),
                      "pair_share_if_vop2_pairs": (v["pairable"] + v["unmeasured_vop2"]) / sum(v.values())}
                  for c, v in sorted(per.items())}
    json.dump(res, open(out, "w"), indent=1)
    for c, v in res["loop"].items():
        print(f"{c:8s} static {v['static']:5d} pair share {v['pair_share']:.3f} (if VOP2 pairs "
              f"{v['pair_share_if_vop2_pairs']:.3f})  {dict((k, n) for k, n in v.items() if isinstance(n, int))}")


if __name__ == "__main__":
    main()
