#!/bin/bash
# Instruction-class PMC pass of the default variant over a short bench run
# (rocprofv3 --pmc with --kernel-trace only, one pass): tools/pmc_mix.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out; TAG=${1:-pmc_mix}
mkdir -p $OUT/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU \
  SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/$TAG/pass_mix -o p -- \
  python3 $R/bench.py --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-qc > $OUT/$TAG/pass_mix.json 2> $OUT/$TAG/pass_mix.err
