#!/usr/bin/env python3
"""The drop-in QC call (automatic committee cache) against the explicit
committee handle on the same votes, alternating in one process: p50 and the
library's median host phases (bench._timed_lib).  Both run the committee
latency kernel; the difference is what each path does around it.

python tools/qc_dropin_vs_explicit.py [--reps 500] [--rounds 3]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=500)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import bench
    from hsverify import _lib, committee, synth
    lib = _lib.load()
    lib.hsv_set_auto_committee(1)
    for size in (100, 1000):
        w = synth.qc_votes(size, seed=size)
        packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
        d = bytes(w.msg)
        dropin = lambda: lib.hsv_verify_batch_packed(d, packed, w.n)
        for _ in range(3):
            assert dropin() == 1
        lib.hsv_auto_committee_wait(60000)
        c = committee.Committee(w.pk)
        h = c._h
        explicit = lambda: lib.hsv_committee_verify_batch_packed(h, d, packed, w.n)
        assert explicit() == 1
        for r in range(a.rounds):
            for name, fn in (("dropin", dropin), ("explicit", explicit)):
                t = bench._timed_lib(fn, a.reps)
                print(json.dumps({"votes": w.n, "round": r, "path": name, "p50_ms": round(t["p50_ms"], 4),
                                  "p99_ms": round(t["p99_ms"], 4), "phases": t.get("median_phases_ms")}), flush=True)
        c.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
