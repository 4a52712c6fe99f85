#!/usr/bin/env python3
"""Instruction-class histogram of a kernel's loops and a mix-weighted issue
ceiling.

Each VALU opcode is priced in "units": the SIMD's issue time of one wave64
v_add_u32_e32 at full occupancy, from tools/ubench_isa.hip
(profiles/r02_ubench_isa.txt: 62.4 T lane-ops/s over 256 CUs x 4 SIMDs, i.e.
1 unit = 1.05 ns per SIMD).  Classes:
  mad    v_mad_u64_u32                                  1.84
  vop3   64-bit shifts/adds, mul_lo, 3-operand and      ~1.65 (per opcode below)
         lshl-class ops, alignbit, perm, cndmask_e64
  fast   add/sub/and/or/xor/lshr/ashr/mov (VOP2)        0.86-1.00
  vcc    v_cndmask_b32_e32 (reads VCC)                   8.37
SALU, branches, waitcnt, s_nop and memory instructions are listed but not
priced (they issue on other ports; s_nop holds only its own wave).

python tools/isa_mix.py FILE.s KERNEL_SUBSTRING [--min 100] [--trips SPEC]
  SPEC: comma list of MADS=TRIPS, e.g. "527=128.4,909=66.2": loops whose body
  holds exactly MADS v_mad_u64_u32 are weighted by TRIPS executions per lane
  (per verification); the weighted sum gives units per verification.
"""
import argparse
import collections
import re

UNIT_NS = 1.05  # ns per unit per SIMD (62.4 T v_add_u32 lane-ops/s on 1024 SIMDs)

COST = {
    "v_mad_u64_u32": 1.84,
    "v_add_u32_e32": 1.00, "v_sub_u32_e32": 0.99, "v_and_b32_e32": 0.94, "v_or_b32_e32": 0.93,
    "v_xor_b32_e32": 0.92, "v_lshrrev_b32_e32": 0.87, "v_ashrrev_i32_e32": 0.88, "v_mov_b32_e32": 0.86,
    "v_lshlrev_b32_e32": 1.61, "v_mul_lo_u32": 1.68, "v_mul_u32_u24_e32": 1.61, "v_mad_u32_u24": 1.65,
    "v_lshl_or_b32": 1.63, "v_lshl_add_u32": 1.64, "v_add_lshl_u32": 1.63, "v_and_or_b32": 1.64,
    "v_or3_b32": 1.64, "v_add3_u32": 1.66, "v_bfe_u32": 1.61, "v_bfi_b32": 1.64, "v_alignbit_b32": 1.63,
    "v_perm_b32": 1.67, "v_cndmask_b32_e32": 8.37, "v_cndmask_b32_e64": 1.70, "v_lshrrev_b64": 1.65,
    "v_lshl_add_u64": 1.72, "v_mov_b64_e32": 1.61,
}


def klass(op):
    if op == "v_mad_u64_u32":
        return "mad"
    if op == "v_cndmask_b32_e32":
        return "vcc"
    if op.startswith("v_"):
        c = COST.get(op)
        if c is None:
            return "valu?"
        return "fast" if c < 1.2 else "vop3"
    if op == "s_nop":
        return "s_nop"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_", "ds_")):
        return "mem"
    return "salu"


def units(op):
    if op.startswith("v_"):
        return COST.get(op, 1.65)
    return 0.0


def kernel_body(lines, want):
    st = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and want in l)
    en = st + next(i for i, l in enumerate(lines[st:]) if "s_endpgm" in l)
    return lines[st:en + 1]


def loops(body):
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    res = []
    for i, l in enumerate(body):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            res.append((labels[m.group(1)], i))
    return res


def histogram(lines):
    ops = [l.split()[0] for l in lines if re.match(r"^\s+[vsgdb][a-z_0-9]+", l)]
    return collections.Counter(ops)


def summarize(c):
    by = collections.Counter()
    u = 0.0
    for op, n in c.items():
        by[klass(op)] += n
        u += units(op) * n
    return by, u


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--min", type=int, default=100)
    ap.add_argument("--trips", default="")
    a = ap.parse_args()
    body = kernel_body(open(a.asm).read().split("\n"), a.kernel)
    spec = {int(k): float(v) for k, v in (x.split("=") for x in a.trips.split(",") if x)}
    whole = histogram(body)
    by, u = summarize(whole)
    print(f"kernel {a.kernel}: {sum(whole.values())} static instructions; classes {dict(by)}; {u:.0f} units")
    total_units, seen = 0.0, set()
    for lo, hi in sorted(loops(body), key=lambda x: x[0]):
        c = histogram(body[lo:hi + 1])
        n = sum(c.values())
        if n < a.min:
            continue
        by, u = summarize(c)
        mads = c.get("v_mad_u64_u32", 0)
        share = 100.0 * c.get("v_mad_u64_u32", 0) * COST["v_mad_u64_u32"] / u if u else 0.0
        top = ", ".join(f"{op} {k}" for op, k in c.most_common(8))
        print(f"loop lines {lo}-{hi}: {n} instrs, {mads} mad, classes {dict(by)}, {u:.0f} units "
              f"({share:.0f}% in mad)\n    {top}")
        if mads in spec and mads not in seen:
            seen.add(mads)
            total_units += spec[mads] * u
            print(f"    x {spec[mads]} trips per verification -> {spec[mads] * u:.0f} units")
    if spec:
        print(f"weighted loops: {total_units:.0f} units per verification lane = {total_units * UNIT_NS / 1e3:.1f} us "
              f"of SIMD issue per 64-lane wave")


if __name__ == "__main__":
    main()
