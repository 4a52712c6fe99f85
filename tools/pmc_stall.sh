#!/bin/bash
# Stall / instruction-cache PMC passes of the default variant over a short
# bench run, one rocprofv3 --pmc pass each (--kernel-trace only):
# tools/pmc_stall.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out; TAG=${1:-pmc_stall}
mkdir -p $OUT/$TAG
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$TAG/$name -o p -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-qc > $OUT/$TAG/$name.json 2> $OUT/$TAG/$name.err
}
run pass_sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_INSTS SQ_BUSY_CYCLES && \
run pass_sqc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ && \
run pass_vmem SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_CYCLES
