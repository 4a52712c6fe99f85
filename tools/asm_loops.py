#!/usr/bin/env python3
"""Every loop (back edge) of one kernel in a hipcc -S output: size, nesting
span and instruction mix, to find where a kernel's instructions go.

python tools/asm_loops.py file.s kernel_substring [min_instrs]
"""
import collections
import re
import sys


def main():
    path, want = sys.argv[1], sys.argv[2]
    min_n = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    L = open(path).read().split("\n")
    start = [i for i, l in enumerate(L) if re.match(r"^_Z\S*:", l) and want in l][0]
    end = start + [i for i, l in enumerate(L[start:]) if "s_endpgm" in l][0]
    K = L[start:end + 1]
    labels = {m.group(1): i for i, l in enumerate(K) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    is_ins = lambda l: re.match(r"^\s+[vsdgb][a-z_0-9]+", l) is not None
    loops = []
    for i, l in enumerate(K):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    print(f"kernel instrs {sum(is_ins(l) for l in K)}")
    for lo, hi in sorted(set(loops)):
        body = [l.split()[0] for l in K[lo:hi + 1] if is_ins(l)]
        if len(body) < min_n:
            continue
        c = collections.Counter(body)
        mad = c.get("v_mad_u64_u32", 0)
        top = ", ".join(f"{k} {v}" for k, v in c.most_common(14))
        print(f"lines {lo}-{hi}: {len(body)} instrs, mad {mad}\n    {top}")


if __name__ == "__main__":
    main()
