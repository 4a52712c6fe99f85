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


def fl2_mul(f, g, stats=None):
    """The two-row product (hsv_fe16x16.hpp, fl2_mul): the even row steps
    0..7 from (f, g), the odd row steps 8..15 from f and g turned by 8 lanes
    (g's wrapped half times 38); each row splits its half column sums at bit
    16 and the pair adds the halves (v_permlane16_swap) before the carry
    passes.  Asserts the same instruction bounds as fl_mul."""
    def half(fr, gr):
        acc = [0] * 16
        for i in range(8):
            if i:
                src = [gr[(k - 1) % 16] for k in range(16)]  # DPP row_ror:1
                assert max(src) < 2**24, "v_mul_u32_u24 input"
                gr = [x * (38 if k == 0 else 1) for k, x in enumerate(src)]
            for k in range(16):
                acc[k] += fr[i] * gr[k]
        assert max(acc) < 2**64
        t = [a >> 16 for a in acc]
        assert max(t) < 2**32, "half carry (v_alignbit_b32)"
        return [a & 0xFFFF for a in acc], t
    g8 = [g[(k - 8) % 16] for k in range(16)]  # row_ror:8 on the odd row
    assert max(g8) < 2**24, "v_mul_u32_u24 input (odd row start)"
    g8 = [x * (38 if k < 8 else 1) for k, x in enumerate(g8)]
    lo_e, t_e = half(list(f), list(g))
    lo_o, t_o = half([f[(i + 8) % 16] for i in range(16)], g8)
    t = [a + b for a, b in zip(t_e, t_o)]
    t = [x * (38 if k == 15 else 1) for k, x in enumerate(t)]
    assert max(t) < 2**32, "summed carry times 38"
    x = [lo_e[k] + lo_o[k] + t[(k - 1) % 16] for k in range(16)]
    assert max(x) < 2**32
    lo = [a & 0xFFFF for a in x]
    c = [a >> 16 for a in x]
    assert max(c) < 2**24, "pass-2 carry (v_mul_u32_u24)"
    c = [v * (38 if k == 15 else 1) for k, v in enumerate(c)]
    out = [lo[k] + c[(k - 1) % 16] for k in range(16)]
    assert value(out) % P == value(f) * value(g) % P
    if stats is not None:
        stats["out"] = max(stats.get("out", 0), max(out))
    return out


def run_two_row(trials=200, seed=5):
    """fl2_mul on the operands run() and run_points() feed fl_mul: limbs up
    to 2^16.05 (product outputs) and up to 2^18.4 (sums and differences, the
    largest operand hsv_rowpoint.hpp forms).  Its limbs equal fl_mul's, so
    every bound of the one-row model carries over."""
    rnd = random.Random(seed)
    st = {}
    for top in (int(2**16.05), 2**17, int(2**18.4)):
        for _ in range(trials // 4):
            f = [rnd.choice([0, 0xFFFF, rnd.randrange(top + 1), top]) for _ in range(16)]
            g = [rnd.choice([0, 0xFFFF, rnd.randrange(top + 1), top]) for _ in range(16)]
            y = fl2_mul(f, g, st)
            assert y == fl_mul(f, g), "two-row and one-row products differ"
            for _ in range(3):
                y = fl2_mul(y, y, st)
    x = [int(2**18.4)] * 16
    fl2_mul(x, x, st)
    return st


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



# ---- the row-form point formulas (csrc/hsv_rowpoint.hpp), bounds only ----
FOURP = [0x1FFB4] + [0x1FFFE] * 15
assert value(FOURP) == 4 * P


def fl_add(a, b):
    return [x + y for x, y in zip(a, b)]


def fl_sub(a, b):
    assert all(y <= q for y, q in zip(b, FOURP)), "fl_sub subtrahend above 4p's limbs"
    return [x + q - y for x, y, q in zip(a, b, FOURP)]


def fl_carry(x):
    assert max(x) < 2**24
    lo = [a & 0xFFFF for a in x]
    t = [(a >> 16) * (38 if k == 15 else 1) for k, a in enumerate(x)]
    return [lo[k] + t[(k - 1) % 16] for k in range(16)]


def rp_finish(E, F, G, H, st):
    return (fl_mul(E, F, st), fl_mul(G, H, st), fl_mul(F, G, st), fl_mul(E, H, st))


def rp_dbl(p, st):
    X, Y, Z, _ = p
    A, B, C, S = fl_mul(X, X, st), fl_mul(Y, Y, st), fl_mul(Z, Z, st), fl_mul(fl_add(X, Y), fl_add(X, Y), st)
    H = fl_add(A, B)
    E = fl_sub(H, S)
    G = fl_sub(A, B)
    F = fl_carry(fl_add(fl_add(C, C), G))
    return rp_finish(E, F, G, H, st)


def rp_add_cached(p, q, st):
    X, Y, Z, T = p
    YpX, YmX, Z2, T2d = q
    A = fl_mul(fl_sub(Y, X), YmX, st)
    B = fl_mul(fl_add(Y, X), YpX, st)
    C = fl_mul(T, T2d, st)
    D = fl_mul(Z, Z2, st)
    return rp_finish(fl_sub(B, A), fl_sub(D, C), fl_add(D, C), fl_add(B, A), st)


def rp_add_niels(p, n, st):
    X, Y, Z, T = p
    ypx, ymx, xy2d = n
    A = fl_mul(fl_sub(Y, X), ymx, st)
    B = fl_mul(fl_add(Y, X), ypx, st)
    C = fl_mul(T, xy2d, st)
    D = fl_add(Z, Z)
    return rp_finish(fl_sub(B, A), fl_sub(D, C), fl_add(D, C), fl_add(B, A), st)


def rp_to_cached(p, d2, st):
    X, Y, Z, T = p
    return (fl_add(Y, X), fl_sub(Y, X), fl_add(Z, Z), fl_mul(T, d2, st))


def run_points(trials=60, seed=3):
    """Doublings, cached and Niels additions, negated entries and table
    builds on worst-case and random limbs: every fl_mul / fl_sub bound holds."""
    rnd = random.Random(seed)
    st = {}
    top = 0x1A000  # a product output's lane-0 limb can reach ~2^16.7

    def elem(hi=0xFFFF):
        return [rnd.choice([0, hi, rnd.randrange(hi + 1)]) for _ in range(16)]

    def prod():  # a product output (worst case: large lane-0 limb)
        x = elem()
        x[0] = rnd.choice([x[0], top])
        return x

    d2 = limbs_of(2 * (-121665 * pow(121666, P - 2, P)) % P)
    for _ in range(trials):
        p = (prod(), prod(), prod(), prod())
        for _ in range(4):
            p = rp_dbl(p, st)
        c = (fl_add(prod(), prod()), fl_sub(prod(), prod()), fl_add(prod(), prod()), prod())
        p = rp_add_cached(p, c, st)
        neg = (c[1], c[0], c[2], fl_sub([0] * 16, c[3]))
        p = rp_add_cached(p, neg, st)
        n = (elem(), elem(), elem())
        p = rp_add_niels(p, n, st)
        p = rp_add_niels(p, (n[1], n[0], fl_sub([0] * 16, n[2])), st)
        p = rp_add_cached(p, rp_to_cached(p, d2, st), st)
        for _ in range(2):
            p = rp_dbl(p, st)
    return st


if __name__ == "__main__":
    st = run()
    print("products", {k: round(math.log2(v), 4) for k, v in st.items()})
    st = run_points()
    print("point formulas", {k: round(math.log2(v), 4) for k, v in st.items()})
    st = run_two_row()
    print("two-row products", {k: round(math.log2(v), 4) for k, v in st.items()})
