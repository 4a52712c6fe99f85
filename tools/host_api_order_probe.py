#!/usr/bin/env python3
"""Why bench.py's host_api reads slower than a fresh-process probe: the same
2^20 host-buffer call (hsv_verify from numpy arrays) timed at each point of
bench.py's order -- fresh, after the C4 launches on three streams, after the
mad peak probe -- with the library's per-chunk host marks each time.

    python tools/host_api_order_probe.py
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from hsverify import _lib, _testing, synth, verifier  # noqa: E402

n = 1 << 20
dev = torch.device("cuda", 0)
lib = _lib.load()
if os.environ.get("PROBE_BIND", "1") == "1":
    verifier.bind_device(0)
w = synth.independent_triples(n, seed=0xC4 * 1000, corrupt_frac=0.05, nthreads=16)


def host_calls(tag, reps=7):
    verifier.verify_flags(w.pk, w.sig, w.msg)
    ts, st = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        f = verifier.verify_flags(w.pk, w.sig, w.msg)
        ts.append((time.perf_counter() - t0) * 1e3)
        st.append(_testing.host_call_stats())
    marks = (ctypes.c_double * 256)()
    cnt = lib.hsv_host_call_marks(marks, 256)
    last = [round(marks[k], 3) for k in range(cnt)]
    ok = bool((f[w.accept] & 1).all()) and not bool((f[~w.accept] & 1).any())
    print(json.dumps({"tag": tag, "ms": sorted(round(t, 3) for t in ts), "median_ms": float(np.median(ts)),
                      "pack_ms": [round(s["pack_ms"], 3) for s in st], "call_ms": [round(s["call_ms"], 3) for s in st],
                      "last_marks_launch_enqueued": last[3::4], "ok": ok}), flush=True)


host_calls("fresh")
pk, sig, msg = (torch.from_numpy(x).to(dev) for x in (w.pk, w.sig, w.msg))
streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(2)]
outs = [(torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros((n + 31) // 32, dtype=torch.int32, device=dev))
        for _ in range(3)]
torch.cuda.synchronize(dev)
t0 = time.perf_counter()
for i in range(12):
    o = outs[i % 3]
    verifier.verify_device(pk, sig, msg, o[0], o[1], stream=streams[i % 3].cuda_stream)
torch.cuda.synchronize(dev)
print(json.dumps({"tag": "c4_device", "ms_per_step": (time.perf_counter() - t0) / 12 * 1e3}), flush=True)
host_calls("after_c4")
probe = verifier.measure_mad_peak()
print(json.dumps({"tag": "mad_peak", "T": probe / 1e12}), flush=True)
host_calls("after_mad_peak")
time.sleep(2.0)
host_calls("after_2s_idle")
# bench.py's own host_api leg in this process (its reps, median and marks)
sys.path.insert(0, ROOT)
import bench  # noqa: E402
r = bench.host_api_bench(w, dev)
print(json.dumps({"tag": "bench_host_api_bench", "ms": r["ms"], "rep_ms": r["rep_ms"], "call_ms": r["call_ms"],
                  "pack_ms": r["pack_ms"], "last_launch_enqueued_ms": r["median_call_last_launch_enqueued_ms"]}),
      flush=True)
