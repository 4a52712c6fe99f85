#!/usr/bin/env python3
"""A/B of the mempool line (bench.mempool_bench: 2^20 transactions of 512 B
in HBM, record + prepass + point pass) between library builds, alternating
fresh processes; HSV_LIB selects each build (files in hsverify/).

python tools/mempool_ab.py [--rounds 3] LIB[@VAR=VALUE] [LIB[@VAR=VALUE] ...]
(LIB@VAR=VALUE runs that library with one more environment variable, e.g.
libhsv.so@HSV_TX_FUSED=0)
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
import torch, bench
r = bench.mempool_bench(torch.device("cuda", 0), cpu_sample=0)
print(json.dumps({{"ms": r["ms_per_step"], "ok": r["honest_all_accepted"] and r["corrupted_all_rejected"]}}))
"""


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
            r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], capture_output=True, text=True,
                               timeout=300, env=env)
            if r.returncode != 0:
                print(r.stdout, r.stderr[-2000:])
                return r.returncode
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res[lib].append(d["ms"])
            print(lib, json.dumps(d), flush=True)
    for lib, v in res.items():
        print("median", lib, round(statistics.median(v), 4), "ms per 2^20")
    return 0


if __name__ == "__main__":
    sys.exit(main())
