#!/usr/bin/env python3
"""Drop-in QC / verify_strict latency with the resident service
(HSV_QC_RESIDENT=1) against launches, alternating fresh processes; prints
each run's p50s (bench.qc_latency) and the medians.
python tools/qc_resident_ab.py [--rounds 3] [--reps 300]"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys
sys.path.insert(0, {root!r}); sys.path.insert(0, {root!r} + "/hotstuff-digital-signature-benchmarking_amd")
import bench
import time
import numpy as np
from hsverify import synth
r = bench.qc_latency({reps}, auto=True)
out = {{k: v["p50_ms"] for k, v in r.items() if isinstance(v, dict) and "p50_ms" in v}}
lib = bench._oracle()   # the dalek port's single verify_strict, same process and box
w = synth.qc_votes(4, seed=4)
ts = bench._timed(lambda: lib.oracle_verify_flags(bytes(w.pk[0]), bytes(w.sig[0]), bytes(w.msg), 32), 200, warm=5)
out["cpu_port_single_verify_strict"] = float(np.median(ts) * 1e3)
print(json.dumps(out))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=300)
    a = ap.parse_args()
    res = {"launch": [], "resident": []}
    for _ in range(a.rounds):
        for mode in res:
            env = dict(os.environ)
            if mode == "resident":
                env["HSV_QC_RESIDENT"] = "1"
            r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, reps=a.reps)], capture_output=True,
                               text=True, timeout=300, env=env)
            if r.returncode != 0:
                print(mode, "rc", r.returncode, r.stderr[-1500:])
                return r.returncode
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res[mode].append(d)
            print(mode, json.dumps(d), flush=True)
    for mode, runs in res.items():
        print("median", mode, json.dumps({k: round(statistics.median(x[k] for x in runs), 4) for k in runs[0]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
