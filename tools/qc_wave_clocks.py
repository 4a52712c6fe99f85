#!/usr/bin/env python3
"""Where the committee QC kernel spends its time, wave by wave
(hsv_comb_verify_quad_fused_kernel built with -DHSV_QC_WAVE_CLOCKS:
tools/build_ab_libs.sh qcclk "-DHSV_QC_WAVE_CLOCKS").

Each wave's lane 0 stamps the 100 MHz constant clock (s_memrealtime) at
0 entry, 1 past the entry barrier, 2 its own work done (comb wave: the s
half; R waves: the decompression; hash wave: the hash), 3 the comb wave past
the k handover (R and hash waves: their first loads landed), 4 at the final
barrier, 5 exit; plus its place (XCC, SE, SH,
CU, SIMD) and the shader clock at entry and exit.  A -DHSV_QC_WAVE_CLOCKS_TWICE
build decompresses R twice (slot 9 between the passes): the second pass runs
with the code already in the instruction cache.  For the drop-in C1 (3 votes,
1 block) and C3 (667 votes, 167 blocks) calls this reports, as medians over the
reps: the spread of wave entries (dispatch ramp), every role's phase lengths,
and the kernel span (first entry to last exit).

HSV_LIB=libhsv_qcclk.so python tools/qc_wave_clocks.py [--reps 200]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))

TICK_US = 0.01  # 100 MHz
SLOTS = 10


def analyse(clk, nblocks, wpb):
    raw = clk[: nblocks * wpb].reshape(nblocks, wpb, SLOTS)
    place = raw[:, :, 6].astype(np.uint64)
    sclk0, sclk1 = raw[:, :, 7].astype(np.int64), raw[:, :, 8].astype(np.int64)
    c = raw[:, :, :6].astype(np.int64)
    t0 = c[:, :, 0].min()
    c = c - t0
    life_rt = np.maximum(c[:, :, 5] - c[:, :, 0], 1)
    hw = place & np.uint64(0xffffffff)
    xcc = (place >> np.uint64(32)) & np.uint64(0xf)
    simd_key = (xcc << np.uint64(16)) | (((hw >> np.uint64(13)) & np.uint64(7)) << np.uint64(8)) | \
        (((hw >> np.uint64(12)) & np.uint64(1)) << np.uint64(7)) | (((hw >> np.uint64(8)) & np.uint64(15)) << np.uint64(2)) | \
        ((hw >> np.uint64(4)) & np.uint64(3))
    cu_key = simd_key >> np.uint64(2)
    _, simd_counts = np.unique(simd_key.ravel(), return_counts=True)
    _, cu_counts = np.unique(cu_key[:, 0], return_counts=True)
    entry = c[:, :, 0]
    comb, r, hashw = c[:, 0, :], c[:, 1:wpb - 1, :], c[:, wpb - 1, :]
    out = {
        "entry_spread_us": float(entry.max()) * TICK_US,
        "block_entry_spread_us": float((entry.max(axis=1) - entry.min(axis=1)).max()) * TICK_US,
        "span_us": float(c[:, :, 5].max()) * TICK_US,
        "comb_s_half_us": float(np.median(comb[:, 2] - comb[:, 0])) * TICK_US,
        "comb_wait_k_us": float(np.median(comb[:, 3] - comb[:, 2])) * TICK_US,
        "comb_k_half_swaps_us": float(np.median(comb[:, 4] - comb[:, 3])) * TICK_US,
        "comb_barrier_wait_us": float(np.median(np.maximum(r[:, :, 4].max(axis=1), comb[:, 4]) - comb[:, 4])) * TICK_US,
        "comb_tail_us": float(np.median(comb[:, 5] - np.maximum(r[:, :, 4].max(axis=1), comb[:, 4]))) * TICK_US,
        "r_decompress_us": float(np.median(r[:, :, 2] - r[:, :, 0])) * TICK_US,
        "hash_us": float(np.median(hashw[:, 2] - hashw[:, 1])) * TICK_US,
        "r_load_us": float(np.median(r[:, :, 3] - r[:, :, 0])) * TICK_US,
        "r_alu_us": float(np.median(r[:, :, 2] - r[:, :, 3])) * TICK_US,
        "r_first_pass_us": float(np.median(raw[:, 1:wpb - 1, 9].astype(np.int64) - t0 - r[:, :, 3])) * TICK_US
        if raw[:, 1:wpb - 1, 9].any() else None,
        "r_second_pass_us": float(np.median(r[:, :, 2] - (raw[:, 1:wpb - 1, 9].astype(np.int64) - t0))) * TICK_US
        if raw[:, 1:wpb - 1, 9].any() else None,
        "hash_load_us": float(np.median(hashw[:, 3] - hashw[:, 1])) * TICK_US,
        "hash_alu_us": float(np.median(hashw[:, 2] - hashw[:, 3])) * TICK_US,
        "comb_life_us": float(np.median(comb[:, 5] - comb[:, 0])) * TICK_US,
        "comb_life_max_us": float((comb[:, 5] - comb[:, 0]).max()) * TICK_US,
        "last_exit_block": int(c[:, 0, 5].argmax()),
        "last_exit_block_entry_us": float(entry[c[:, 0, 5].argmax()].min()) * TICK_US,
        "shader_clock_mhz": float(np.median((sclk1 - sclk0) / (life_rt * TICK_US))),
        "max_waves_per_simd": int(simd_counts.max()),
        "max_blocks_per_cu": int(cu_counts.max()),
        "cus_used": int(len(cu_counts)),
        "xccs_used": int(len(np.unique(xcc))),
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    from hsverify import _lib, synth
    lib = _lib.load()
    fn = lib.hsv_qc_wave_clocks
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.hsv_set_auto_committee(1)
    res = {}
    for committee in (4, 100, 1000):
        w = synth.qc_votes(committee, seed=committee)
        packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
        d = bytes(w.msg)
        for _ in range(3):
            lib.hsv_verify_batch_packed(d, packed, w.n)
        lib.hsv_auto_committee_wait(60000)
        nblocks = (w.n + 3) // 4
        buf = np.zeros((4096, SLOTS), dtype=np.uint64)
        wpb = fn(None, 0)
        rows = []
        for i in range(a.reps + 10):
            rc = lib.hsv_verify_batch_packed(d, packed, w.n)
            assert rc in (0, 1), rc
            wpb = fn(buf.ctypes.data, nblocks * wpb)
            assert wpb > 0
            if i >= 10:
                rows.append(analyse(buf, nblocks, wpb))
        keys = rows[0].keys()
        res[f"n{committee}_votes{w.n}"] = {
            "blocks": nblocks, "waves_per_block": wpb,
            **{k: (round(float(np.median([r[k] for r in rows])), 3) if rows[0][k] is not None else None)
               for k in keys},
            "span_us_p90": round(float(np.percentile([r["span_us"] for r in rows], 90)), 3),
        }
        print(json.dumps({f"n{committee}_votes{w.n}": res[f"n{committee}_votes{w.n}"]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
