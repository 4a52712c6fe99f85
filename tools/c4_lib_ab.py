#!/usr/bin/env python3
"""Same-box A/B of the C4 line (bench.py --no-qc --no-cpu-baseline) between
library builds in hsverify/ (HSV_LIB), alternating fresh processes; prints
each run's verif/s, ms per step and one-launch time, then the medians.
python tools/c4_lib_ab.py [--rounds 3] LIB[@VAR=VALUE] [LIB[@VAR=VALUE] ...]
(LIB@VAR=VALUE runs that library with one more environment variable)"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    res = {lib: [] for lib in a.libs}
    for _ in range(a.rounds):
        for lib in a.libs:
            name, _, kv = lib.partition("@")
            env = dict(os.environ, HSV_LIB=name)
            if kv:
                k, _, v = kv.partition("=")
                env[k] = v
            r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-qc", "--no-cpu-baseline"],
                               capture_output=True, text=True, timeout=300, env=env)
            if r.returncode != 0:
                print(lib, "rc", r.returncode, r.stderr[-1500:])
                return r.returncode
            d = json.loads(r.stdout.strip().splitlines()[-1])
            row = (d["value"] / 1e6, d["ms_per_step"], d["roofline"]["isolated_launch_ms"])
            res[lib].append(row)
            print(lib, json.dumps({"M_verif_s": round(row[0], 2), "ms_per_step": round(row[1], 4),
                                   "one_launch_ms": round(row[2], 4)}), flush=True)
    for lib, v in res.items():
        print("median", lib, round(statistics.median(x[0] for x in v), 2), "M verif/s,",
              round(statistics.median(x[1] for x in v), 4), "ms per step,",
              round(statistics.median(x[2] for x in v), 4), "ms one launch")
    return 0


if __name__ == "__main__":
    sys.exit(main())
