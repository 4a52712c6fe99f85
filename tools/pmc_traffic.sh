#!/bin/bash
# HBM traffic of the default verify kernel: two rocprofv3 --pmc passes over a
# short bench run (FETCH_SIZE and WRITE_SIZE cannot share a pass), summarised
# into gpurun_out/pmc_traffic.json (copy it to profiles/latest_pmc_traffic.json).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/pmc_traffic_$c -o p -- \
    python3 $R/bench.py --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-qc > $OUT/pmc_traffic_$c.json 2> $OUT/pmc_traffic_$c.err || exit 1
done
cd $R && python3 - <<'PY'
import csv, glob, json, collections
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/pmc_traffic_{c}/**/*counter_collection.csv", recursive=True)[0]
    # one verify launch = its prepass (hsv_prep_kernel, two-pass variants) +
    # the verify kernel, summed per launch; the warm-up launch is dropped
    per, names = collections.OrderedDict(), {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "hsv_verify" not in k and "hsv_prep" not in k:
            continue
        names[r["Dispatch_Id"]] = k
        per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    launches, cur, name = [], 0.0, None
    for d in sorted(per, key=int):
        cur += per[d]
        if "hsv_verify" in names[d]:
            launches.append(cur)
            cur, name = 0.0, names[d]
    vals = launches[1:]
    out[c] = sum(vals) / len(vals) * 1024.0  # rocprofv3 reports kilobytes
    out["kernel"] = name + (" + hsv_prep_kernel" if any("hsv_prep" in v for v in names.values()) else "")
bench = json.load(open("gpurun_out/pmc_traffic_FETCH_SIZE.json"))
json.dump({"variant": bench["config"]["kernel_variant"], "n": bench["config"]["batch_per_gpu"],
           "fetch_bytes_per_launch": out["FETCH_SIZE"], "write_bytes_per_launch": out["WRITE_SIZE"],
           "kernel": out["kernel"], "source": "profiles/latest_pmc_traffic.json (tools/pmc_traffic.sh)"},
          open("gpurun_out/pmc_traffic.json", "w"), indent=1)
print(open("gpurun_out/pmc_traffic.json").read())
PY
