#!/usr/bin/env python3
"""A/B of the host-buffer call (hsv_verify from numpy arrays at 2^20 items,
PCIe-inclusive) between environment settings, alternating fresh processes:
by default the chunked copy pipeline against the same chunk schedule with
the pack and the copies skipped on repeat calls (HSV_PIPE_NOCOPY=1 here makes
the child load libhsv_test.so and set hsv_test_pipe_nocopy: its GPU time
alone); HSV_HOST_PIPE=streamed selects the streamed launch.  Prints each
run's median of 5 calls and the median per setting.

python tools/host_api_ab.py [--rounds 3] [SETTING ...]   (SETTING: NAME=VALUE,... or "default")
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, os, sys, time
import numpy as np
sys.path.insert(0, {root!r} + "/hotstuff-digital-signature-benchmarking_amd")
from hsverify import _testing, synth, verifier
n = 1 << 20
w = synth.independent_triples(n, seed=5, corrupt_frac=0.05)
if os.environ.get("HSV_PIPE_NOCOPY") == "1":  # the test library's no-copy hook
    _ctx = _testing.test_library()
    _ctx.__enter__()
    _testing.pipe_nocopy(True)
verifier.verify_flags(w.pk, w.sig, w.msg)
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    f = verifier.verify_flags(w.pk, w.sig, w.msg)
    ts.append(time.perf_counter() - t0)
ok = bool((f[w.accept] & 1).all()) and not bool((f[~w.accept] & 1).any())
print(json.dumps({{"ms": float(np.median(ts) * 1e3), "ok": ok, "marks": _testing.host_call_marks()[:8],
                  "pack_ms": _testing.host_call_stats()["pack_ms"]}}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("settings", nargs="*", default=["default", "HSV_PIPE_NOCOPY=1"])
    a = ap.parse_args()
    res = {s: [] for s in a.settings}
    for _ in range(a.rounds):
        for st in a.settings:
            env = dict(os.environ)
            if st != "default":
                for kv in st.split(","):
                    k, _, v = kv.partition("=")
                    env[k] = v
            r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], capture_output=True, text=True,
                               timeout=300, env=env)
            if r.returncode != 0:
                print(r.stdout, r.stderr[-2000:])
                return r.returncode
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res[st].append(d["ms"])
            print(st, json.dumps(d), flush=True)
    for st, v in res.items():
        print("median", st, round(statistics.median(v), 3), "ms", round((1 << 20) / statistics.median(v) / 1e3, 1),
              "M verif/s")
    return 0


if __name__ == "__main__":
    sys.exit(main())
