#!/bin/bash
# One rocprofv3 --pmc pass over a short bench run: tools/pmc_pass.sh TAG VARIANT COUNTER...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out; TAG=$1; VAR=$2; shift 2
mkdir -p $OUT/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$TAG -o p -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-qc --variant $VAR > $OUT/$TAG.json 2> $OUT/$TAG.err
