#!/bin/bash
# Round-3 GPU round: GPU suite, then the default bench line, then (STAGES) extra
# probes.  TAG names the outputs under gpurun_out/; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out; TAG=${TAG:-r03}; mkdir -p $OUT
step() { echo "== $1"; }
if [ -z "$NO_TESTS" ]; then
  step pytest; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest_gpu.txt 2>&1; rc=$?
  tail -2 $OUT/${TAG}_pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
fi
step bench; timeout -k 10 700 python bench.py $BENCH_ARGS > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err; rc=$?
[ $rc -eq 0 ] || { tail -5 $OUT/${TAG}_bench.err; exit $rc; }
python -c "
import json; d=json.load(open('$OUT/${TAG}_bench.json')); r=d['roofline']
print('C4', d['value']/1e6, d['ms_per_step'], r['frac'], r['isolated_launch_ms'], d['checks'])
for k in ('host_api', 'mempool_tx'):
    if k in d: print(k, json.dumps({a: b for a, b in d[k].items() if a != 'cpu_baseline'}))
"
if [ -n "$PROF" ]; then
  step rocprof; cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o bench -- python3 $R/bench.py --steps 5 --warmup 1 --streams 1 --no-cpu-baseline --no-qc > $OUT/${TAG}_prof_bench.json 2> $OUT/${TAG}_prof.err; rc=$?
  [ $rc -eq 0 ] || { tail -5 $OUT/${TAG}_prof.err; exit $rc; }
  f=$(find $OUT/${TAG}_prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/${TAG}_kernel_stats.csv; cut -d, -f1-4 $OUT/${TAG}_kernel_stats.csv | head -5
fi
