#!/usr/bin/env python3
"""Summarise tools/pmc_r04.sh: per-dispatch counter means per kernel.

  python tools/pmc_r04_summary.py gpurun_out/TAG [out_prefix]
writes OUT_pmc_mix.json (C4 point pass + prepass) and OUT_qc_pmc.json
(committee and generic QC kernels at C1 and C3); out_prefix defaults to
profiles/TAG.
"""
import collections
import csv
import glob
import json
import os
import sys

N = 1 << 20
PEAK_LANE_OPS = 256 * 4 * 16 * 2.4e9


def per_kernel(pass_dir, min_grid=0):
    f = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur, name = {}, {}
    for r in csv.DictReader(open(f[0])):
        if int(r["Grid_Size"]) < min_grid:
            continue
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
        key = (k, r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for key, cs in per.items():
        for c, v in cs.items():
            out[key[0]][c].append(v)
        out[key[0]]["_us"].append(dur[key] * 1e6)
    res = {}
    for k, cs in out.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["_dispatches"] = len(cs["_us"])
        res[k] = d
    return res


def main():
    root = sys.argv[1].rstrip("/")
    tag = os.path.basename(root)
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join("profiles", tag)
    mix = per_kernel(os.path.join(root, "mix"), min_grid=1024)
    pick = lambda d, name: next((v for k, v in d.items() if k.endswith(name)), {})
    hp = pick(mix, "hsv_verify_hp_kernel")
    pre = pick(mix, "hsv_prep_kernel")
    res = {"source": f"tools/pmc_r04.sh ({tag}/mix): rocprofv3 --kernel-trace --pmc over bench.py --steps 3 "
                     "--streams 1, C4 2^20 items per launch", "items": N, "per_dispatch_mean": mix}
    if hp:
        simds = 1024
        res["point_pass"] = {
            "valu_instr_per_wave_64_items": hp["SQ_INSTS_VALU"] / (N / 64),
            "valu_lane_instr_per_verify": hp["SQ_INSTS_VALU"] * 64 / N,
            "int64_share_of_valu": hp.get("SQ_INSTS_VALU_INT64", 0) / hp["SQ_INSTS_VALU"],
            "int32_share_of_valu": hp.get("SQ_INSTS_VALU_INT32", 0) / hp["SQ_INSTS_VALU"],
            "vmem_rd_instr_per_wave": hp.get("SQ_INSTS_VMEM_RD", 0) / (N / 64),
            # rocprof's VALUBusy: active VALU cycles x 4 / SIMDs / GPU busy cycles (per XCD)
            "valu_busy": hp["SQ_ACTIVE_INST_VALU"] * 4 / simds / (hp["GRBM_GUI_ACTIVE"] / 8)
            if hp.get("GRBM_GUI_ACTIVE") else None,
            "kernel_us_under_pmc": hp["_us"],
            "valu_lane_issue_frac_of_int32_peak": hp["SQ_INSTS_VALU"] * 64 / (hp["_us"] * 1e-6) / PEAK_LANE_OPS,
        }
    if pre:
        res["prepass"] = {"valu_lane_instr_per_verify": pre["SQ_INSTS_VALU"] * 64 / N, "kernel_us_under_pmc": pre["_us"]}
    with open(f"{out}_pmc_mix.json", "w") as f:
        json.dump(res, f, indent=1, default=float)
        f.write("\n")
    qc = {"source": f"tools/pmc_r04.sh ({tag}/qc3, qc667): tools/qc_kernel_profile.py under rocprofv3 --pmc, "
                    "200 drop-in verify_batch calls with the committee cache warm + 200 with it off"}
    for v in ("3", "667"):
        ks = per_kernel(os.path.join(root, f"qc{v}"))
        qc[f"votes_{v}"] = {k: d for k, d in ks.items() if "committee" in k or "comb_verify" in k or "row_kernel" in k}
    a = qc.get("votes_3", {})
    b = qc.get("votes_667", {})
    diff = {}
    for k in set(a) & set(b):
        diff[k] = {c: b[k][c] - a[k][c] for c in a[k] if c in b[k] and not c.startswith("_dispatches")}
    qc["c3_minus_c1"] = diff
    with open(f"{out}_qc_pmc.json", "w") as f:
        json.dump(qc, f, indent=1, default=float)
        f.write("\n")
    print(json.dumps({"point_pass": res.get("point_pass"), "c3_minus_c1": diff}, indent=1, default=float))


if __name__ == "__main__":
    main()
