#!/usr/bin/env python3
"""Time share of the verification phases: the same kernel variant built with
one phase replaced by a stub (tools/build_phase_libs.sh, -DHSV_TIMING_STUB_*).
Stub builds give WRONG flags; only their launch times are reported.

Round 2 measured the shares with tools/build_ab_libs.sh (st_sqrt, st_straus,
st_tables, st_comb, st_lattice, st_sha: -DHSV_TIMING_STUB_<PHASE>) and
tools/ab_probe.py, which alternates the builds on one box
(profiles/r02_ab_log.txt).  This script does the same for the default variant.

python tools/phase_probe.py [--variant 21] [--n 1048576]
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd")


def child(lib_path, variant, n, reps):
    code = f"""
import sys, numpy as np, torch
sys.path.insert(0, {PKG!r})
from hsverify import _lib
_lib.LIB_PATH = {lib_path!r}
from hsverify import verifier, synth
verifier.set_variant({variant})
w = synth.independent_triples({n}, seed=77, corrupt_frac=0.05, nthreads=16)
dev = torch.device('cuda:0')
pk, sig, msg = (torch.from_numpy(a).to(dev) for a in (w.pk, w.sig, w.msg))
flags = torch.zeros({n}, dtype=torch.uint8, device=dev)
verifier.verify_device(pk, sig, msg, flags); torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range({reps}): verifier.verify_device(pk, sig, msg, flags)
e1.record(); torch.cuda.synchronize()
print('%.4f' % (e0.elapsed_time(e1) / {reps}))
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-2000:])
    return float(r.stdout.strip().split()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=21)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default=None,
                    help="time only this build: full, lattice, sqrt, sha, straus, tables or comb")
    a = ap.parse_args()
    if a.only:
        lib = os.path.join(PKG, "hsverify", "libhsv.so") if a.only == "full" else \
            os.path.join(PKG, f"build_stub_{a.only}", "libhsv.so")
        print(f"{a.only}: {child(lib, a.variant, a.n, a.reps):.3f} ms", flush=True)
        return
    base = child(os.path.join(PKG, "hsverify", "libhsv.so"), a.variant, a.n, a.reps)
    print(f"variant {a.variant}  full kernel {base:.3f} ms", flush=True)
    for name in ("lattice", "sqrt", "sha", "straus", "tables", "comb"):
        t = child(os.path.join(PKG, f"build_stub_{name}", "libhsv.so"), a.variant, a.n, a.reps)
        print(f"  without {name:8s} {t:.3f} ms   share {100 * (base - t) / base:5.1f} %", flush=True)


if __name__ == "__main__":
    main()
