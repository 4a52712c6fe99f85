#!/usr/bin/env python3
"""Workspace pool bookkeeping: device memory left after
2^20-item launches each on a fresh stream that is then dropped (blocks freed
on a stream are reused only on that stream), and the cross-stream event
pipeline's outputs (tests/test_device_model.py's chain) for the library in
use (HSV_LIB).

python tools/pool_strand_probe.py [--streams 12]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=12)
    a = ap.parse_args()
    import torch
    from hsverify import synth, verifier
    dev = torch.device("cuda", 0)
    n = 1 << 20
    w = synth.independent_triples(n, seed=5, corrupt_frac=0.05, nthreads=16)
    pk, sig, msg = (torch.from_numpy(x).to(dev) for x in (w.pk, w.sig, w.msg))
    f = torch.zeros(n, dtype=torch.uint8, device=dev)
    verifier.verify_device(pk, sig, msg, f)
    torch.cuda.synchronize(dev)
    free0 = torch.cuda.mem_get_info(dev)[0]
    rows = []
    for i in range(a.streams):
        s = torch.cuda.Stream(dev)
        verifier.verify_device(pk, sig, msg, f, stream=s.cuda_stream)
        torch.cuda.synchronize(dev)
        del s
        rows.append(round((free0 - torch.cuda.mem_get_info(dev)[0]) / 2**20, 1))
    # torch hands out streams from a fixed pool of its own; raw streams are
    # new every time
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    raw = []
    for i in range(a.streams * 2):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        verifier.verify_device(pk, sig, msg, f, stream=h.value)
        torch.cuda.synchronize(dev)
        assert hip.hipStreamDestroy(h) == 0
        raw.append(round((free0 - torch.cuda.mem_get_info(dev)[0]) / 2**20, 1))
    print(json.dumps({"lib": os.environ.get("HSV_LIB", "libhsv.so"), "mib_held_after_each_fresh_stream": rows,
                      "mib_held_after_each_raw_stream": raw}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
