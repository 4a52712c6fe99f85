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
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-qc > $OUT/pmc_traffic_$c.json 2> $OUT/pmc_traffic_$c.err || exit 1
done
cd $R && python3 - <<'PY'
import csv, glob, json, collections
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/pmc_traffic_{c}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.OrderedDict()
    name = None
    for r in csv.DictReader(open(f)):
        if "hsv_verify" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"]
        per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    vals = list(per.values())[1:]  # drop the warm-up launch
    out[c] = sum(vals) / len(vals) * 1024.0  # rocprofv3 reports kilobytes
    out["kernel"] = name
bench = json.load(open("gpurun_out/pmc_traffic_FETCH_SIZE.json"))
json.dump({"variant": bench["config"]["kernel_variant"], "n": bench["config"]["batch_per_gpu"],
           "fetch_bytes_per_launch": out["FETCH_SIZE"], "write_bytes_per_launch": out["WRITE_SIZE"],
           "kernel": out["kernel"], "source": "profiles/latest_pmc_traffic.json (tools/pmc_traffic.sh)"},
          open("gpurun_out/pmc_traffic.json", "w"), indent=1)
print(open("gpurun_out/pmc_traffic.json").read())
PY
