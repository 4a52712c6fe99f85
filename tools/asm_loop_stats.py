#!/usr/bin/env python3
"""Instruction mix of the longest loop of a kernel in a hipcc -S output.

python tools/asm_loop_stats.py file.s kernel_substring
"""
import collections
import re
import sys


def main():
    path, want = sys.argv[1], sys.argv[2]
    L = open(path).read().split("\n")
    start = [i for i, l in enumerate(L) if re.match(r"^_Z\S*:", l) and want in l][0]
    end = start + [i for i, l in enumerate(L[start:]) if "s_endpgm" in l][0]
    K = L[start:end + 1]
    labels = {m.group(1): i for i, l in enumerate(K) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    is_ins = lambda l: re.match(r"^\s+[vsdgb][a-z_0-9]+", l) is not None
    back = []
    for i, l in enumerate(K):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            back.append((labels[m.group(1)], i))
    lo, hi = max(back, key=lambda x: x[1] - x[0])
    c = collections.Counter(l.split()[0] for l in K[lo:hi + 1] if is_ins(l))
    print(f"kernel instrs {sum(is_ins(l) for l in K)}  main loop instrs {sum(c.values())}")
    body = K[lo:hi + 1]
    print("  in main loop: scratch ops %d, global loads %d, ds_read %d; whole kernel scratch ops %d" % (
        sum("scratch_" in l for l in body), sum("global_load" in l for l in body),
        sum("ds_read" in l for l in body), sum("scratch_" in l for l in K)))
    for k, v in c.most_common(14):
        print(f"  {k:28s} {v}")


if __name__ == "__main__":
    main()
