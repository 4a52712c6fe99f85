import sys, os, time, numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hotstuff-digital-signature-benchmarking_amd"))
from hsverify import verifier, synth
dev = torch.device("cuda:0")
for n in (1000, 64, 1024, 4096):
    for use_bits in (False, True):
        w = synth.independent_triples(n, seed=5, corrupt_frac=0.05)
        pk, sig, msg = (torch.from_numpy(a).to(dev) for a in (w.pk, w.sig, w.msg))
        flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        bits = torch.zeros((n + 31) // 32, dtype=torch.int32, device=dev) if use_bits else None
        t = time.time()
        print("launch", n, use_bits, flush=True)
        verifier.verify_device(pk, sig, msg, flags, bits)
        torch.cuda.synchronize()
        print("  done %.3fs ok=%s" % (time.time() - t, bool((flags.cpu().numpy()[w.honest] & 1).all())), flush=True)
