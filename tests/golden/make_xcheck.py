#!/usr/bin/env python3
"""Commit the independent verdict columns that pin the oracle (round 4).

For every record set of tests/xcheck.py `datasets` (the 2193 golden records,
the lattice-fallback records, the reference's fixture records, the
transaction vectors, the C3 QC and TC vectors and 2^15 random records) this
runs OpenSSL 3.0.2's Ed25519 verify and libsodium 1.0.18's, classifies every
record against the oracle's flags (xcheck.classify_openssl / classify_sodium)
and writes tests/golden/xcheck_verdicts.json:

  {set: {"n", "records_sha256", "openssl": packed verdict bits (hex, bit i =
   record i, little-endian), "sodium": same, "openssl_divergent": {i: class},
   "sodium_divergent": {i: class}}}

The generator aborts on any unclassified divergence.  tests/test_xcheck.py
re-runs both libraries and compares with the committed columns; the columns
also let a box without either library check the classification.

Run from the repo root:  python tests/golden/make_xcheck.py
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))
import xcheck  # noqa: E402


def c_oracle():
    import subprocess
    so = os.path.join(ROOT, "oracle", "_build", "libhsv_oracle.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s"], cwd=os.path.join(ROOT, "oracle"), check=True)
    lib = ctypes.CDLL(so)
    lib.oracle_verify_many.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                                               ctypes.c_int]

    def flags(pk, sig, msg):
        pk, sig, msg = (np.ascontiguousarray(a, np.uint8) for a in (pk, sig, msg))
        out = np.zeros(pk.shape[0], np.uint8)
        lib.oracle_verify_many(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, 32, pk.shape[0],
                               out.ctypes.data, min(16, os.cpu_count() or 1))
        return out
    return flags


def main():
    ossl, sodium = xcheck.OpenSSL(), xcheck.Sodium()
    out = {"generator": "tests/golden/make_xcheck.py", "openssl": ossl.version, "libsodium": sodium.version,
           "sets": {}}
    for name, (pk, sig, msg, flags) in xcheck.datasets(c_oracle()).items():
        vo = xcheck.run(ossl, pk, sig, msg)
        vs = xcheck.run(sodium, pk, sig, msg)
        cls = xcheck.classify_all(flags, pk, sig, vo, vs)
        bad = [(i, c) for k in cls for i, c in enumerate(cls[k]) if c.startswith("unclassified")]
        if bad:
            raise SystemExit(f"{name}: unclassified divergences {bad[:5]}")
        out["sets"][name] = {
            "n": int(pk.shape[0]),
            "records_sha256": xcheck.records_digest(pk, sig, msg),
            "openssl": xcheck.pack_verdicts(vo),
            "sodium": xcheck.pack_verdicts(vs),
            "openssl_divergent": {str(i): c for i, c in enumerate(cls["openssl"]) if c != "agree"},
            "sodium_divergent": {str(i): c for i, c in enumerate(cls["sodium"]) if c != "agree"},
        }
        s = out["sets"][name]
        print(f"{name}: n={s['n']} openssl accepts {int(vo.sum())}, divergent {len(s['openssl_divergent'])}; "
              f"sodium accepts {int(vs.sum())}, divergent {len(s['sodium_divergent'])}")
    with open(os.path.join(HERE, "xcheck_verdicts.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
