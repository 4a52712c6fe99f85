#!/usr/bin/env python3
"""A/B of QC latency between kernel builds: each library named on the command
line (files in hsverify/, selected with HSV_LIB) runs bench.qc_latency in a
fresh process, alternating A, B, A, B; prints the p50s per run and the
medians per library.

python tools/qc_ab.py [--rounds 2] [--reps 200] LIB [LIB ...]
"""
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
r = bench.qc_latency({reps}, auto={auto})
print(json.dumps({{k: v["p50_ms"] for k, v in r.items() if isinstance(v, dict) and "p50_ms" in v}}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--generic", action="store_true", help="committee cache off: the generic kernels")
    ap.add_argument("--env", action="append", default=[],
                    help="NAME=VALUE for every child (repeatable); a LIB argument of the form "
                         "lib.so:NAME=VALUE sets NAME for that run only")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    res = {lib: [] for lib in a.libs}
    for _ in range(a.rounds):
        for lib in a.libs:
            name, _, extra = lib.partition(":")
            env = dict(os.environ, HSV_LIB=name)
            for kv in a.env + ([extra] if extra else []):
                k, _, v = kv.partition("=")
                env[k] = v
            r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, reps=a.reps, auto=not a.generic)],
                               capture_output=True, text=True, timeout=300, env=env)
            if r.returncode != 0:
                print(r.stdout, r.stderr[-2000:])
                return r.returncode
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res[lib].append(d)
            print(lib, json.dumps({k: round(v, 4) for k, v in d.items()}), flush=True)
    for lib, runs in res.items():
        print("median", lib, json.dumps({k: round(statistics.median(r[k] for r in runs), 4) for k in runs[0]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
