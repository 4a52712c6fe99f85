#!/usr/bin/env python3
"""Where the C3 QC's extra time comes from: p50 of the drop-in
verify_batch with the committee cache warm for
  * C3: 667 votes by 667 distinct keys (the bench case),
  * C3 one key: the first vote repeated 667 times (one key's table, one R),
  * C1: 3 votes,
so the difference between the first two is what 667 distinct keys' comb
tables and R values cost beyond the vote count.

python tools/qc_c3_keys_probe.py [--reps 300]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))

from hsverify import _lib, synth  # noqa: E402


def p50(lib, digest, packed, n, reps):
    for _ in range(5):
        lib.hsv_verify_batch_packed(digest, packed, n)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        rc = lib.hsv_verify_batch_packed(digest, packed, n)
        ts.append(time.perf_counter() - t0)
        assert rc == 1, rc
    return round(float(np.median(ts)) * 1e3, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    a = ap.parse_args()
    lib = _lib.load()
    lib.hsv_set_auto_committee(1)
    w = synth.qc_votes(1000, seed=1000)
    rows = np.concatenate([w.pk, w.sig], axis=1)
    digest = bytes(w.msg)
    for _ in range(3):
        lib.hsv_verify_batch_packed(digest, rows.tobytes(), w.n)
    lib.hsv_auto_committee_wait(60000)
    same = np.repeat(rows[:1], w.n, axis=0)
    out = {}
    for rnd in range(2):
        out[f"c3_distinct_{rnd}"] = p50(lib, digest, rows.tobytes(), w.n, a.reps)
        out[f"c3_one_key_{rnd}"] = p50(lib, digest, same.tobytes(), w.n, a.reps)
        out[f"c1_{rnd}"] = p50(lib, digest, rows[:3].tobytes(), 3, a.reps)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
