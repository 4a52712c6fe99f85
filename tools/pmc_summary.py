#!/usr/bin/env python3
"""Summarise tools/pmc_round.sh output for the verification launch of the
default variant (prepass + point pass): per-launch counter means per kernel,
VALU instructions per verification, VALU lane-issue rate against the int32
peak, and HBM bytes (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE).

    python tools/pmc_summary.py gpurun_out/<tag> > profiles/<tag>_summary.json
"""
import collections
import csv
import glob
import json
import os
import sys

PEAK_LANE_OPS = 256 * 4 * 16 * 2.4e9   # int32 VALU lane-ops/s (MI355X_MICROARCH.md chip table)
N = 1 << 20
KERNELS = ("hsv_prep_kernel", "hsv_verify_hp_kernel")


def load(pass_dir):
    f = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> counter -> sum
    dur = {}
    for r in csv.DictReader(open(f[0])):
        k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
        if k is None or int(r["Grid_Size"]) < 1024:
            continue
        key = (k, r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            out[k][c].append(v)
        out[k]["_seconds"].append(dur[(k, _)])
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in out.items()}


def main():
    root = sys.argv[1]
    merged = collections.defaultdict(dict)
    for p in ("pass_valu", "pass_mem", "pass_fetch", "pass_write"):
        for k, cs in load(os.path.join(root, p)).items():
            for c, v in cs.items():
                if c == "_seconds":
                    merged[k].setdefault("_seconds_by_pass", {})[p] = v
                else:
                    merged[k][c] = v
    res = {"items": N, "per_launch_mean": merged}
    tot_valu = sum(merged[k].get("SQ_INSTS_VALU", 0.0) for k in KERNELS)
    tot_s = sum(merged[k].get("_seconds_by_pass", {}).get("pass_valu", 0.0) for k in KERNELS)
    res["valu_instr_per_verify"] = tot_valu * 64 / N
    if tot_s:
        res["kernel_ms_under_pmc"] = tot_s * 1e3
        res["valu_lane_instr_per_s_T"] = tot_valu * 64 / tot_s / 1e12
        res["valu_issue_frac_of_int32_peak"] = tot_valu * 64 / tot_s / PEAK_LANE_OPS
    for k in KERNELS:
        m = merged.get(k, {})
        if m.get("SQ_BUSY_CYCLES") and m.get("SQ_ACTIVE_INST_VALU") is not None and m.get("SQ_WAVE_CYCLES"):
            res.setdefault("per_kernel", {})[k] = {
                "valu_instr_per_verify": m.get("SQ_INSTS_VALU", 0) * 64 / N,
                "vmem_rd_instr_per_verify": m.get("SQ_INSTS_VMEM_RD", 0) * 64 / N,
                "valu_share_of_issued": m.get("SQ_ACTIVE_INST_VALU", 0) / max(1.0, m.get("SQ_ACTIVE_INST_ANY", 0) or 1.0),
                "wait_share_of_wave_cycles": m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"],
            }
    fetch = sum(merged[k].get("FETCH_SIZE", 0.0) for k in KERNELS) * 1024
    write = sum(merged[k].get("WRITE_SIZE", 0.0) for k in KERNELS) * 1024
    res["hbm_bytes_per_launch"] = 2 * fetch + write
    res["hbm_bytes_per_verify"] = (2 * fetch + write) / N
    res["algorithmic_bytes_per_verify"] = 129
    json.dump(res, sys.stdout, indent=1, default=float)
    print()


if __name__ == "__main__":
    main()
