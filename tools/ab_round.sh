#!/bin/bash
# GPU suite, then an A/B timing of kernel builds (tools/ab_probe.py LIBS), then a
# rocprofv3 kernel-trace of a short bench.  TAG names the outputs; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out; TAG=${TAG:-ab}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_pytest_gpu.txt 2>&1; rc=$?
tail -2 $OUT/${TAG}_pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
if [ -n "$LIBS" ]; then
  timeout -k 10 500 python -u tools/ab_probe.py --rounds ${ROUNDS:-4} $LIBS > $OUT/${TAG}_ab.txt 2>&1; rc=$?
  tail -$(( $(echo $LIBS | wc -w) + 1 )) $OUT/${TAG}_ab.txt; [ $rc -eq 0 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o bench -- python3 $R/bench.py --steps 5 --warmup 1 --streams 1 --no-cpu-baseline --no-qc > $OUT/${TAG}_prof_bench.json 2> $OUT/${TAG}_prof.err; rc=$?
[ $rc -eq 0 ] || { tail -5 $OUT/${TAG}_prof.err; exit $rc; }
f=$(find $OUT/${TAG}_prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/${TAG}_kernel_stats.csv; cut -d, -f1-4 $OUT/${TAG}_kernel_stats.csv | head -4
