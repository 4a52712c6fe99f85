#!/usr/bin/env python3
"""Writes a C3 TC (667 timeouts, 5 % corrupted member votes) and a C3 QC as
bincode bytes to /tmp/tc.bin and /tmp/qc.bin for tools/wire_parse_bench.cpp
(the same certificates bench.py's tc_latency / qc_latency legs verify)."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))
import bench  # noqa: E402
from hsverify import synth, wire  # noqa: E402

w = bench.member_corrupted(synth.tc_votes, 1000, seed=1000, frac=0.05)
hqc = bench.tc_hqc(1000, 1000)
open("/tmp/tc.bin", "wb").write(wire.encode_tc(1000, [(bytes(p), bytes(s), int(h)) for p, s, h in zip(w.pk, w.sig, hqc)]))
q = synth.qc_votes(1000, seed=1000)
bh = hashlib.sha512(b"block" + (1000).to_bytes(4, "little")).digest()[:32]
open("/tmp/qc.bin", "wb").write(wire.encode_qc(bh, 1, [(bytes(p), bytes(s)) for p, s in zip(q.pk, q.sig)]))
