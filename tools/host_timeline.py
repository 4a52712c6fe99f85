#!/usr/bin/env python3
"""Timeline of the last host-buffer hsv_verify call from a rocprofv3 kernel +
memory-copy trace (CSV): copies and kernels with their stream ids and grid
sizes, in microseconds from the call's first event (the last call = the
events after the last gap of more than 1.5 ms).

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
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:34]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   f"K s{r['Stream_Id']} {name} grid={int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}"))
    for r in rows(d, "*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   f"C s{r['Stream_Id']} {r['Direction'].replace('MEMORY_COPY_', '')}"))
    ev.sort()
    end = ev[0][1]
    starts = [0]
    for i in range(1, len(ev)):
        if ev[i][0] - end > 1_500_000:
            starts.append(i)
        end = max(end, ev[i][1])
    first = starts[-1]
    t0 = ev[first][0]
    for s, e, name in ev[first:]:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name}")


if __name__ == "__main__":
    main()
