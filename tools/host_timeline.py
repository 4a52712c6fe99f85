#!/usr/bin/env python3
"""Timeline of one host-buffer hsv_verify call (2^20 triples) from a rocprofv3
kernel + memory-copy trace (CSV): copies and kernels of the last call, in
microseconds from its first copy.

rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o run -- \\
    python tools/host_api_probe.py
python tools/host_timeline.py DIR
"""
import csv
import glob
import os
import sys


def rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d = sys.argv[1]
    ev = []
    for r in rows(d, "*kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:40]))
    for r in rows(d, "*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   "C " + r.get("Direction", "?") + " " + r.get("Size", "?")))
    ev.sort()
    # the last call: from the last run of H2D copies that follows a gap > 2 ms
    starts = [i for i in range(1, len(ev)) if ev[i][0] - ev[i - 1][1] > 2_000_000]
    first = starts[-1] if starts else 0
    t0 = ev[first][0]
    for s, e, name in ev[first:]:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name}")


if __name__ == "__main__":
    main()
