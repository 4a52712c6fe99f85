#!/bin/bash
# Round-4 counter passes (round-3 VERDICT item 5), one rocprofv3 --pmc run per
# pass, --kernel-trace only, each under its own time limit:
#   mix   the C4 launch (prepass + point pass, one stream): instruction mix and
#         VALU activity of hsv_verify_hp_kernel
#   qc1 / qc3   the committee QC kernel at C1 (3 votes) and C3 (667 votes):
#         L2 hits / misses, wait and busy cycles, instruction fetch
# tools/pmc_r04.sh TAG   -> gpurun_out/TAG/{mix,qc1,qc3}/...; summarise with
# python tools/pmc_r04_summary.py gpurun_out/TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out; TAG=${1:-r04_pmc}
mkdir -p $OUT/$TAG
cd /tmp && export TMPDIR=/tmp
echo "== pmc mix"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU \
  SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/$TAG/mix -o p -- \
  python3 $R/bench.py --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-qc > $OUT/$TAG/mix.json 2> $OUT/$TAG/mix.err || exit $?
for v in 3 667; do
  echo "== pmc qc $v"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES \
    SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_IFETCH GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/$TAG/qc$v -o p -- \
    python3 $R/tools/qc_kernel_profile.py $v > $OUT/$TAG/qc$v.txt 2> $OUT/$TAG/qc$v.err || exit $?
done
echo done
