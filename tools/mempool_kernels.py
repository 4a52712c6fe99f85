#!/usr/bin/env python3
"""The mempool line's kernels one at a time (one stream, a sync after every
step), for a kernel trace whose durations are the kernels' own:

cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o mk -- python3 tools/mempool_kernels.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def main():
    import torch
    from hsverify import mempool, synth, verifier
    dev = torch.device("cuda:0")
    n = 1 << 20
    w = synth.transactions(n, tx_size=512, seed=9)
    d = torch.from_numpy(w.txs.reshape(-1)).to(dev)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    t = synth.independent_triples(n, seed=5, corrupt_frac=0.05)
    pk, sig, msg = (torch.from_numpy(x).to(dev) for x in (t.pk, t.sig, t.msg))
    for _ in range(6):
        mempool.verify_transactions_device(d, None, tx_size=512, n=n, flags=flags)
        torch.cuda.synchronize()
        verifier.verify_device(pk, sig, msg, flags)
        torch.cuda.synchronize()
    print("ok", int((flags.cpu().numpy() & 1).sum()))


if __name__ == "__main__":
    main()
