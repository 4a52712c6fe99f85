#!/usr/bin/env python3
"""Per-kernel mean counter values of rocprofv3 --pmc passes.

python tools/pmc_table.py DIR [kernel-substring ...]
DIR holds pass subdirectories with p_counter_collection.csv (tools/pmc_*.sh).
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d, want):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "*", "p_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if want and not any(w in k for w in want):
                continue
            key = k.split("(")[0]
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(key, f, r["Counter_Name"])].add(r["Dispatch_Id"])
    out = {}
    for key, cs in agg.items():
        out[key] = {}
        for c, v in cs.items():
            n = max(len(ds) for (k2, f, c2), ds in disp.items() if k2 == key and c2 == c)
            out[key][c] = v / n
    return out


if __name__ == "__main__":
    res = load(sys.argv[1], sys.argv[2:])
    print(json.dumps(res, indent=1, sort_keys=True))
