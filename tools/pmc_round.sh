#!/bin/bash
# PMC passes over a short bench run (each pass separate: --pmc with --kernel-trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out; TAG=${1:-pmc}; VAR=${2:-0}
mkdir -p $OUT/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/$TAG/counters_list.txt 2>&1 || true
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$TAG/$name -o p -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-qc --variant $VAR > $OUT/$TAG/$name.json 2> $OUT/$TAG/$name.err
}
run pass_valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE && \
run pass_mem SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY && \
run pass_fetch FETCH_SIZE && \
run pass_write WRITE_SIZE
rc=$?
ls $OUT/$TAG
exit $rc
