#!/usr/bin/env python3
"""Does the calling thread's NUMA node change the QC latency?  Prints the
host's NUMA nodes (CPU lists), the GPU's node, then runs the drop-in C1 / C3
QC p50 (bench._timed_lib, automatic committee cache) in child processes
pinned (sched_setaffinity before any GPU call) to CPUs of each node.

python tools/qc_numa_probe.py [--reps 300]
"""
import argparse
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, json
os.sched_setaffinity(0, {cpus!r})  # where the library allocates its slots (the warm-up calls)
sys.path.insert(0, {root!r}); sys.path.insert(0, {root!r} + "/hotstuff-digital-signature-benchmarking_amd")
import numpy as np
import bench
from hsverify import _lib, synth
lib = _lib.load()
lib.hsv_set_auto_committee(1)
out = {{}}
for size in (4, 1000):
    w = synth.qc_votes(size, seed=size)
    p = np.concatenate([w.pk, w.sig], 1).tobytes(); d = bytes(w.msg)
    call = lambda: lib.hsv_verify_batch_packed(d, p, w.n)
    for _ in range(3): call()
    lib.hsv_auto_committee_wait(60000)
    os.sched_setaffinity(0, {run_cpus!r})  # where the timed calls run
    t = bench._timed_lib(call, {reps})
    os.sched_setaffinity(0, {cpus!r})
    out[f"votes{{w.n}}"] = [round(t["p50_ms"], 4), (t.get("median_phases_ms") or {{}}).get("sync")]
print(json.dumps(out))
"""


def cpulist(s):
    cpus = []
    for part in s.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus += range(int(a), int(b) + 1)
        elif part:
            cpus.append(int(part))
    return cpus


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    a = ap.parse_args()
    nodes = {}
    for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        nodes[int(d.rsplit("node", 1)[1])] = cpulist(open(d + "/cpulist").read())
    allowed = os.sched_getaffinity(0)
    gpu_nodes = set()
    for f in glob.glob("/sys/class/drm/card*/device/numa_node"):
        try:
            gpu_nodes.add(int(open(f).read()))
        except (OSError, ValueError):
            pass
    print(json.dumps({"nodes": {k: [v[0], v[-1], len(v)] for k, v in nodes.items()}, "allowed": len(allowed),
                      "gpu_numa_nodes": sorted(gpu_nodes), "visible": os.environ.get("HIP_VISIBLE_DEVICES")}),
          flush=True)
    picks = {node: [c for c in cpus if c in allowed][:8] for node, cpus in nodes.items()}
    picks = {k: v for k, v in picks.items() if v}
    for rnd in range(2):
        for init_node, init_cpus in picks.items():
            for run_node, run_cpus in picks.items():
                r = subprocess.run([sys.executable, "-c", CHILD.format(cpus=set(init_cpus), run_cpus=set(run_cpus),
                                                                      root=ROOT, reps=a.reps)],
                                   capture_output=True, text=True, timeout=300)
                line = (r.stdout.strip().splitlines()[-1] if r.returncode == 0
                        else f"rc={r.returncode} {r.stderr[-300:]}")
                print(json.dumps({"round": rnd, "init_node": init_node, "run_node": run_node, "result": line}),
                      flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
