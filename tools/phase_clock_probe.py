#!/usr/bin/env python3
"""Per-batch phase durations of the point pass from a -DHSV_PHASE_CLOCKS build
(tools/build_ab_libs.sh clk "-DHSV_PHASE_CLOCKS"; never shipped).

Every 64-item batch of hsv_verify_hp_kernel records wall-clock stamps (100 MHz)
at its start, after the two root chains, after the two table builds, after the
window loop and at its end.  Batches are ranked by start time and grouped into
rounds of the persistent grid (3 waves x 1024 SIMDs); the table prints each
phase's mean duration per round, so a phase that slows down when every wave of
the chip runs it at once (round 0) shows up against the later, drifted rounds.

HSV_LIB=libhsv_clk.so python tools/phase_clock_probe.py [--json out.json]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))
CACHE = "/tmp/hsv_ab_c4.npz"
TICK_US = 0.01  # s_memrealtime: 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    ap.add_argument("--slots", type=int, default=3072)
    ap.add_argument("--raw")
    a = ap.parse_args()
    import torch
    from hsverify import _lib, synth, verifier
    lib = _lib.load()
    rd = lib.hsv_phase_clocks_read
    rd.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    rd.restype = ctypes.c_int
    if os.path.exists(CACHE):
        z = np.load(CACHE)
        P, S, M = z["pk"], z["sig"], z["msg"]
    else:
        w = synth.independent_triples(1 << 20, seed=0xC4 * 1000, corrupt_frac=0.05, nthreads=16)
        P, S, M = w.pk, w.sig, w.msg
        np.savez(CACHE, pk=P, sig=S, msg=M)
    dev = torch.device("cuda:0")
    tp, ts, tm = (torch.from_numpy(x).to(dev) for x in (P, S, M))
    fl = torch.zeros(P.shape[0], dtype=torch.uint8, device=dev)
    bits = torch.zeros(P.shape[0] // 32, dtype=torch.int32, device=dev)
    nb = P.shape[0] // 64
    buf = np.zeros(nb * 8, dtype=np.uint64)
    runs = []
    for r in range(4):
        torch.cuda.synchronize()
        assert rd(buf.ctypes.data, buf.size, 1) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        verifier.verify_device(tp, ts, tm, fl, bits)
        e1.record()
        torch.cuda.synchronize()
        assert rd(buf.ctypes.data, buf.size, 0) == 0
        runs.append((e0.elapsed_time(e1), buf.reshape(nb, 8).copy()))
    ms, rec = runs[-1]
    assert (((rec[:, 7] >> 8) & 0xff) == 1).all(), "batches without a record"
    cyc = (rec[:, 7] >> 16).astype(np.int64)
    xcc = (rec[:, 7] & 15).astype(np.int64)
    seq = (rec[:, 6] & 255).astype(np.int64)
    t = rec[:, :5].astype(np.int64)
    t -= t[:, 0].min()
    order = np.argsort(t[:, 0], kind="stable")
    rnd = np.empty(nb, dtype=np.int64)
    rnd[order] = np.arange(nb) // a.slots
    names = ["roots", "tables", "straus", "comb+rest"]
    d = np.diff(t, axis=1) * TICK_US
    out = {"launch_ms": ms, "all_launch_ms": [r[0] for r in runs], "span_us": float(t[:, 4].max() * TICK_US),
           "rounds": []}
    print(f"launch {ms:.3f} ms (HIP events), batch stamps span {t[:, 4].max() * TICK_US:.0f} us")
    print("round  batches  start_us(min..max)   " + "  ".join(f"{n:>10s}" for n in names) + "   total_us")
    for r in range(int(rnd.max()) + 1):
        sel = rnd == r
        dd = d[sel].mean(axis=0)
        st = t[sel, 0] * TICK_US
        row = {"round": r, "batches": int(sel.sum()), "start_min_us": float(st.min()), "start_max_us": float(st.max()),
               "phase_us": {n: float(v) for n, v in zip(names, dd)}, "total_us": float(d[sel].sum(axis=1).mean())}
        out["rounds"].append(row)
        print(f"{r:5d}  {sel.sum():7d}  {st.min():8.0f}..{st.max():8.0f}   " +
              "  ".join(f"{v:10.1f}" for v in dd) + f"   {row['total_us']:8.1f}")
    # per XCC (each has its own real-time counter): first batch of a wave vs later ones
    out["xcc"] = []
    print("xcc  batches  span_us   first-batch phases (us)                    later-batch phases (us)")
    for x in range(int(xcc.max()) + 1):
        sx = xcc == x
        if not sx.any():
            continue
        tx = t[sx]
        span = float((tx[:, 4].max() - tx[:, 0].min()) * TICK_US)
        f1 = d[sx & (seq == 1)].mean(axis=0)
        fl_ = d[sx & (seq > 1)].mean(axis=0)
        out["xcc"].append({"xcc": x, "batches": int(sx.sum()), "span_us": span, "first": f1.tolist(), "later": fl_.tolist()})
        mhz = float(cyc[sx].sum() / ((t[sx, 4] - t[sx, 0]).sum() * TICK_US))
        out["xcc"][-1]["shader_mhz"] = mhz
        print(f"{x:3d}  {sx.sum():7d}  {span:7.0f}   " + " ".join(f"{v:7.1f}" for v in f1) + "     " +
              " ".join(f"{v:7.1f}" for v in fl_) + f"   {mhz:6.0f} MHz")
    for k in range(1, int(seq.max()) + 1):
        sk = seq == k
        print(f"wave batch #{k}: {sk.sum()} batches, mean phases " + " ".join(f"{v:7.1f}" for v in d[sk].mean(axis=0)))
    # per SIMD: waves active over time (a wave spans its first batch start .. last batch end)
    hw = rec[:, 5].astype(np.int64)
    simd = (xcc << 16) | (((hw >> 8) & 0xff) << 4) | ((hw >> 4) & 3)  # XCC | SE/SH/CU bits | SIMD
    wave = hw & 15  # HW_ID.WAVE_ID: the wave slot of its SIMD (persistent waves keep it)
    key = simd * 100000 + wave
    alone = []; two = []; end_spread = []
    for sid in np.unique(simd):
        m = simd == sid
        ws = {}
        for kk, a0, a1 in zip(key[m], t[m, 0], t[m, 4]):
            lo, hi = ws.get(kk, (a0, a1))
            ws[kk] = (min(lo, a0), max(hi, a1))
        ends = sorted(v[1] for v in ws.values())
        if len(ends) >= 3:
            alone.append((ends[-1] - ends[-2]) * TICK_US)
            two.append((ends[-2] - ends[-3]) * TICK_US)
        end_spread.append((ends[-1] - ends[0]) * TICK_US)
    out["simd_alone_us_mean"] = float(np.mean(alone)) if alone else None
    out["simd_two_us_mean"] = float(np.mean(two)) if two else None
    print(f"SIMDs {len(end_spread)}: last wave alone {np.mean(alone):.0f} us (mean), two waves left {np.mean(two):.0f} us, "
          f"first-to-last wave exit {np.mean(end_spread):.0f} us; kernel span {t[:, 4].max() * TICK_US:.0f} us")
    if a.raw:
        np.save(a.raw, rec)
    # concurrency of the table phase: how many batches are in it at each moment
    ev = np.concatenate([np.stack([t[:, 1], np.ones(nb)], 1), np.stack([t[:, 2], -np.ones(nb)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    conc = np.cumsum(ev[:, 1])
    out["table_phase_max_concurrency"] = int(conc.max())
    print(f"batches in the table phase at once: max {int(conc.max())}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
