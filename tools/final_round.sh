#!/bin/bash
# Full GPU round on the current tree: GPU suite, smoke, the default bench line, the C5
# line (2^24 on this GPU), the stream probe, and a rocprofv3 kernel trace of a
# one-stream bench (per-launch kernel averages).  TAG names the outputs; stops at the
# first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out; TAG=${TAG:-rfinal}; mkdir -p $OUT
step() { echo "== $1"; }
step pytest; timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_pytest_gpu.txt 2>&1; rc=$?
tail -2 $OUT/${TAG}_pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
step smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.txt 2>&1; rc=$?
tail -1 $OUT/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit $rc
step bench; timeout -k 10 600 python bench.py --detail $OUT/${TAG}_bench_detail.json > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err; rc=$?
[ $rc -eq 0 ] || { tail -5 $OUT/${TAG}_bench.err; exit $rc; }
python -c "import json; d=json.load(open('$OUT/${TAG}_bench.json')); r=d['roofline']; print(d['value']/1e6, d['ms_per_step'], r['frac'], r['isolated_launch_ms'], d['checks'])"
step c5; timeout -k 10 600 python bench.py --global-n 16777216 --steps 5 --warmup 1 --no-cpu-baseline --no-qc --detail $OUT/${TAG}_c5_detail.json > $OUT/${TAG}_c5_2p24_1gpu_bench.json 2> $OUT/${TAG}_c5.err; rc=$?
[ $rc -eq 0 ] || { tail -5 $OUT/${TAG}_c5.err; exit $rc; }
python -c "import json; d=json.load(open('$OUT/${TAG}_c5_2p24_1gpu_bench.json')); print(d['value']/1e6, d['ms_per_step'])"
step probe; timeout -k 10 300 python -u tools/pipeline_probe.py --rounds 5 > $OUT/${TAG}_pipeline_probe.txt 2>&1; rc=$?
tail -4 $OUT/${TAG}_pipeline_probe.txt; [ $rc -eq 0 ] || exit $rc
step rocprof; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o bench -- python3 $R/bench.py --steps 5 --warmup 1 --streams 1 --no-cpu-baseline --no-qc --detail $OUT/${TAG}_prof_detail.json > $OUT/${TAG}_prof_bench.json 2> $OUT/${TAG}_prof.err; rc=$?
[ $rc -eq 0 ] || { tail -5 $OUT/${TAG}_prof.err; exit $rc; }
f=$(find $OUT/${TAG}_prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/${TAG}_kernel_stats.csv
python -c "
import csv
for r in csv.DictReader(open('$OUT/${TAG}_kernel_stats.csv')): print(r['Name'][:44], r['Calls'], r['AverageNs'])" | head -4
