#!/bin/bash
# The C4 line with its extra streams at normal and at high priority, one
# bench.py process each, two rounds (same box).
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
for r in 1 2; do for p in normal high; do
timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-qc --stream-priority $p > gpurun_out/sp_ab.json 2>/dev/null || exit 1
python -c "
import json; d=json.load(open('gpurun_out/sp_ab.json')); print('priority=$p', round(d['ms_per_step'],3), 'ms/step', round(d['value']/1e6,2), 'M verif/s')"
done; done
