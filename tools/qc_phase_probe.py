#!/usr/bin/env python3
"""Which wave sets the committee QC latency (hsv_comb_verify_quad_fused_kernel):
p50 of the drop-in call for C1 / C3 / one strict verify under each library
named (hsverify/, via HSV_LIB), one fresh process each, no verdict checks --
the timing-stub builds (-DHSV_TIMING_STUB_RWAVE: quad path alone,
-DHSV_TIMING_STUB_QUADPATH: R waves alone) give wrong flags.

python tools/qc_phase_probe.py [--reps 300] LIB [LIB ...]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys, time
import numpy as np
sys.path.insert(0, {root!r} + "/hotstuff-digital-signature-benchmarking_amd")
from hsverify import _lib, synth
lib = _lib.load()
lib.hsv_set_auto_committee(1)
out = {{}}
for committee in (4, 1000):
    w = synth.qc_votes(committee, seed=committee)
    packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
    d = bytes(w.msg)
    for _ in range(3):
        lib.hsv_verify_batch_packed(d, packed, w.n)
    lib.hsv_auto_committee_wait(60000)
    ts = []
    for i in range({reps} + 20):
        t0 = time.perf_counter()
        lib.hsv_verify_batch_packed(d, packed, w.n)
        if i >= 20:
            ts.append(time.perf_counter() - t0)
    out[f"n{{committee}}_votes{{w.n}}"] = round(float(np.median(ts)) * 1e3, 4)
print(json.dumps(out))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    for _ in range(a.rounds):
        for lib in a.libs:
            r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, reps=a.reps)], capture_output=True,
                               text=True, timeout=300, env=dict(os.environ, HSV_LIB=lib))
            line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else f"rc={r.returncode} {r.stderr[-500:]}"
            print(lib, line, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
