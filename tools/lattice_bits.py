#!/usr/bin/env python3
"""Bit lengths of the lattice-reduced scalar pairs (c0, c1) for random
challenges k < l, per item and per 64-lane wave (the largest of the wave's
128 scalars sets how many Straus windows the wave runs: csrc/hsv_verify_hc.hpp
straus_vt).  Uses the host build of the kernel core (tests/native/core_host,
built by tests/test_kernel_host.py into build/core_host).

python tools/lattice_bits.py [N]
"""
import collections
import os
import random
import subprocess
import sys

L = 2**252 + 27742317777372353535851937790883648493
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    rnd = random.Random(3)
    ks = [rnd.randrange(L) for _ in range(n)]
    out = subprocess.run([os.path.join(ROOT, "build", "core_host"), "--lattice"],
                         input="\n".join(f"{k:064x}" for k in ks) + "\n",
                         capture_output=True, text=True, check=True).stdout.split()
    per_item, bits = collections.Counter(), []
    for i in range(n):
        ok, c0, c1 = int(out[4 * i]), int(out[4 * i + 2], 16), int(out[4 * i + 3], 16)
        if not ok:
            per_item["fallback"] += 1
            continue
        b = max(c0.bit_length(), c1.bit_length())
        per_item[b] += 1
        bits.append(b)
    print("items: max(bits(c0), bits(c1)) ->", dict(sorted((k, v) for k, v in per_item.items() if k != "fallback")),
          "fallback:", per_item["fallback"])
    waves = collections.Counter(max(bits[i:i + 64]) for i in range(0, len(bits) - 63, 64))
    tot = sum(waves.values())
    print("waves of 64: largest bit length ->", dict(sorted(waves.items())))
    print("share of waves with every scalar < 2^131 (top 4-bit window zero): %.3f"
          % (sum(v for k, v in waves.items() if k <= 131) / tot))


if __name__ == "__main__":
    main()
