#!/usr/bin/env python3
"""Same-box A/B of whole bench.py lines between library builds in hsverify/
(HSV_LIB), alternating fresh processes: prints, per run, the C4 line, the
mempool line and its ratio to C4, the host-buffer call and the cached C3 QC
p50, then the medians per library.
python tools/bench_lib_ab.py [--rounds 2] LIB[@VAR=VALUE] [LIB[@VAR=VALUE] ...]
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
    ap.add_argument("--rounds", type=int, default=2)
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
            r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-launched"],
                               capture_output=True, text=True, timeout=600, env=env)
            if r.returncode != 0:
                print(lib, "failed", r.stderr[-2000:])
                return r.returncode
            d = json.loads(r.stdout.strip().splitlines()[-1])
            row = {"c4_ms": d["ms_per_step"], "mempool_ms": d["mempool_tx"]["ms_per_step"],
                   "vs_c4": d["mempool_tx"]["vs_c4"], "host_ms": d["host_api"]["ms"],
                   "c3_p50": d["latency"]["qc_c3_667votes"]["gpu"][0]}
            res[lib].append(row)
            print(lib, json.dumps(row), flush=True)
    for lib, rows in res.items():
        print("median", lib, json.dumps({k: round(statistics.median(r[k] for r in rows), 4) for k in rows[0]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
