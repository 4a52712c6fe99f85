#!/bin/bash
# One GPU round: parity tests, smoke, bench, kernel-trace profile.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out
TAG=${1:-r01}
mkdir -p $OUT
echo "== pytest -m gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/${TAG}_pytest_gpu.txt 2>&1; rc=$?; tail -3 $OUT/${TAG}_pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.txt 2>&1; rc=$?; tail -2 $OUT/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 600 python bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err; rc=$?; cat $OUT/${TAG}_bench.json; [ $rc -eq 0 ] || { tail -20 $OUT/${TAG}_bench.err; exit $rc; }
echo "== rocprofv3 kernel trace" && cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o bench -- python3 $R/bench.py --steps 5 --warmup 1 --streams 1 --no-cpu-baseline --no-qc > $OUT/${TAG}_prof_bench.json 2> $OUT/${TAG}_prof.err; rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/${TAG}_prof.err; exit $rc; }
find $OUT/${TAG}_prof -name "*stats*" | head
echo done
