#!/bin/bash
# Round-4 GPU round.  STAGES (default "ubench pmc pytest bench") run in order;
# a test failure (exit 1) does not stop the later stages, a crash, abort or
# time limit (exit >= 124) does.  TAG names the outputs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out; TAG=${TAG:-r04}; mkdir -p $OUT
STAGES=${STAGES:-"ubench pmc pytest bench"}
fatal() { [ "$1" -ge 124 ] && { echo "stage $2 ended with $1: stopping"; exit "$1"; }; return 0; }
for st in $STAGES; do
  echo "== $st"
  case $st in
    ubench)
      timeout -k 10 120 ./tools/ubench_isa > $OUT/${TAG}_ubench_isa.txt 2>&1; rc=$?
      tail -8 $OUT/${TAG}_ubench_isa.txt; fatal $rc $st ;;
    pmc)
      timeout -k 10 600 bash tools/pmc_r04.sh ${TAG}_pmc > $OUT/${TAG}_pmc.log 2>&1; rc=$?
      tail -3 $OUT/${TAG}_pmc.log; fatal $rc $st ;;
    pytest)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > $OUT/${TAG}_pytest_gpu.txt 2>&1; rc=$?
      tail -4 $OUT/${TAG}_pytest_gpu.txt; fatal $rc $st ;;
    pysub)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYSUB" \
        > $OUT/${TAG}_pytest_sub.txt 2>&1; rc=$?
      tail -3 $OUT/${TAG}_pytest_sub.txt; fatal $rc $st ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.txt 2>&1; rc=$?
      tail -1 $OUT/${TAG}_smoke.txt; fatal $rc $st ;;
    bench)
      timeout -k 10 700 python bench.py $BENCH_ARGS > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err; rc=$?
      [ $rc -eq 0 ] || tail -5 $OUT/${TAG}_bench.err
      python -c "
import json; d=json.load(open('$OUT/${TAG}_bench.json')); r=d['roofline']
print('C4', d['value']/1e6, d['ms_per_step'], r['frac'], r['isolated_launch_ms'], d['checks'])
q=d.get('qc_latency', {})
for k, v in q.items():
    if isinstance(v, dict): print(k, v.get('p50_ms'), v.get('p99_ms'), v.get('max_ms'), v.get('tail', {}).get('phases_ms'))
" ; fatal $rc $st ;;
    qcab)
      timeout -k 10 600 python -u tools/qc_ab.py --rounds 3 --reps 300 libhsv.so libhsv.so:HSV_QC_SYNC=marker \
        > $OUT/${TAG}_qc_ab_marker.txt 2>&1; rc=$?
      tail -3 $OUT/${TAG}_qc_ab_marker.txt; fatal $rc $st ;;
    hostab)
      timeout -k 10 600 python -u tools/host_api_ab.py --rounds 3 > $OUT/${TAG}_host_api_ab.txt 2>&1; rc=$?
      tail -3 $OUT/${TAG}_host_api_ab.txt; fatal $rc $st ;;
    memab)
      timeout -k 10 600 python -u tools/mempool_ab.py --rounds 3 libhsv.so libhsv_b3.so \
        > $OUT/${TAG}_mempool_ab_bitop3.txt 2>&1; rc=$?
      tail -3 $OUT/${TAG}_mempool_ab_bitop3.txt; fatal $rc $st ;;
    streampmc)
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU \
        SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE \
        --output-format csv -d $OUT/${TAG}_streampmc -o p -- python3 $R/tools/host_api_probe.py \
        > $OUT/${TAG}_streampmc.txt 2>&1 ); rc=$?
      tail -2 $OUT/${TAG}_streampmc.txt; fatal $rc $st ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o bench -- \
        python3 $R/bench.py --steps 5 --warmup 1 --streams 1 --no-cpu-baseline --no-qc > $OUT/${TAG}_prof_bench.json \
        2> $OUT/${TAG}_prof.err; rc=$?
      f=$(find $OUT/${TAG}_prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/${TAG}_kernel_stats.csv
      cd $R; fatal $rc $st ;;
  esac
done
echo done
