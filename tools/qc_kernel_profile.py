#!/usr/bin/env python3
"""Latency kernels under rocprofv3 --kernel-trace --stats: the C3 QC (667
votes) through the drop-in verify_batch, 200 calls with the committee cache
warm (hsv_comb_verify_quad_fused_kernel) and 200 with it off
(hsv_verify_row_kernel), so the kernel durations stand beside the host-side
p50s of bench.py.

cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o qc -- \\
    python3 /root/repo/tools/qc_kernel_profile.py [VOTES]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))

from hsverify import _lib, synth  # noqa: E402

# argv[1]: votes per QC (default 667, C3; 3 for C1), from a committee of 1000
votes = int(sys.argv[1]) if len(sys.argv) > 1 else 667
lib = _lib.load()
w = synth.qc_votes(1000, seed=1000)
rows = np.concatenate([w.pk, w.sig], axis=1)
lib.hsv_set_auto_committee(1)
for _ in range(3):
    lib.hsv_verify_batch_packed(bytes(w.msg), rows.tobytes(), w.n)
lib.hsv_auto_committee_wait(60000)
packed = rows[:votes].tobytes()
digest = bytes(w.msg)
ok = all(lib.hsv_verify_batch_packed(digest, packed, votes) == 1 for _ in range(200))
lib.hsv_set_auto_committee(0)
ok &= all(lib.hsv_verify_batch_packed(digest, packed, votes) == 1 for _ in range(200))
lib.hsv_set_auto_committee(1)
print("all accepted" if ok else "VERDICT MISMATCH", flush=True)
sys.exit(0 if ok else 1)
