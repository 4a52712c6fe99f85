#!/bin/bash
# Phase shares (tools/phase_probe.py) of one kernel variant, then one PMC pass
# per build (full and each stub build).  Usage (GPU box): bash tools/pmc_phase.sh [VARIANT]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
V=${1:-15}
timeout -k 10 500 python tools/phase_probe.py --variant $V > gpurun_out/phase_probe.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for b in full lattice sqrt sha; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_phase_$b -o p -- python3 $R/tools/phase_probe.py --reps 2 --variant $V --only $b > $R/gpurun_out/pmc_phase_$b.txt 2>&1 || exit 1
done
