#!/usr/bin/env python3
"""Bit-exact model of the lane-split field product (csrc/hsv_fe16x16.hpp,
fl_mul): 16 lanes of a DPP row, radix 2^16, 2^256 = 38 (mod p), with the
bounds every instruction relies on checked on each call:

  * the rotated partner limb g' feeds v_mul_u32_u24: its input < 2^24;
  * the 64-bit column sums do not overflow, and pass 1's carry fits 32 bits
    (v_alignbit_b32), also after lane 15's factor 38;
  * pass 2's carry feeds v_mul_u32_u24: < 2^24.

run() drives chains of products from worst-case and random limbs, including
operands with limbs up to 2^18 (a sum such as yy + (p - 1) fed straight into a
product), and returns the largest output limb: the bound is a fixed point of
the two carry passes (<= 2^16.05 once inputs are <= 2^16.05).

python tools/lanesplit_model.py
"""
import math
import random

P = 2**255 - 19


def value(limbs):
    return sum(x << (16 * k) for k, x in enumerate(limbs))


def limbs_of(v):
    return [(v >> (16 * k)) & 0xFFFF for k in range(16)]


def fl_mul(f, g, stats=None):
    """One product as the device computes it; asserts the instruction bounds."""
    acc = [0] * 16
    gr = list(g)
    for i in range(16):
        if i:
            src = [gr[(k - 1) % 16] for k in range(16)]  # DPP row_ror:1
            assert max(src) < 2**24, "v_mul_u32_u24 input"
            gr = [x * (38 if k == 0 else 1) for k, x in enumerate(src)]
        fi = f[i]  # DPP row_newbcast:i
        for k in range(16):
            acc[k] += fi * gr[k]
    assert max(acc) < 2**64
    lo = [a & 0xFFFF for a in acc]
    t = [a >> 16 for a in acc]
    assert max(t) < 2**32, "pass-1 carry (v_alignbit_b32)"
    t = [x * (38 if k == 15 else 1) for k, x in enumerate(t)]
    assert max(t) < 2**32, "pass-1 carry times 38"
    x = [lo[k] + t[(k - 1) % 16] for k in range(16)]
    lo = [a & 0xFFFF for a in x]
    t = [a >> 16 for a in x]
    assert max(t) < 2**24, "pass-2 carry (v_mul_u32_u24)"
    t = [v * (38 if k == 15 else 1) for k, v in enumerate(t)]
    out = [lo[k] + t[(k - 1) % 16] for k in range(16)]
    assert value(out) % P == value(f) * value(g) % P
    if stats is not None:
        stats["out"] = max(stats.get("out", 0), max(out))
        stats["acc"] = max(stats.get("acc", 0), max(acc))
    return out


def run(trials=400, seed=1):
    rnd = random.Random(seed)
    st = {}
    hi = int(2**16.05)

    def rand_limbs(top):
        return [rnd.choice([0xFFFF, rnd.randrange(2**16), rnd.randrange(top + 1), top]) for _ in range(16)]

    for _ in range(trials):
        f, g = rand_limbs(hi), rand_limbs(hi)
        x = fl_mul(f, g, st)
        for _ in range(4):
            x = fl_mul(x, x, st)
    # all limbs at the bound, and operands up to 2^18 (an unreduced sum)
    x = [hi] * 16
    for _ in range(4):
        x = fl_mul(x, x, st)
    for top in (2**17, int(2**17.1), 2**18 - 1):
        for _ in range(trials // 4):
            y = fl_mul(rand_limbs(top), rand_limbs(hi), st)
            assert max(y) <= int(2**16.3)
            y = fl_mul(y, y, st)
    return st


if __name__ == "__main__":
    st = run()
    print({k: round(math.log2(v), 4) for k, v in st.items()})
