#!/bin/bash
# C5 (2^24 triples on one GPU: four 2^22 launches alternating the caller's
# stream and a library side stream) with the library's streams at normal and
# at the greatest priority (HSV_PIPE_PRIO), one bench.py process each.
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
for r in 1 2; do for p in 0 1; do
HSV_PIPE_PRIO=$p timeout -k 10 300 python bench.py --global-n 16777216 --steps 5 --warmup 1 --no-cpu-baseline --no-qc > gpurun_out/c5_ab.json 2>/dev/null || exit 1
python -c "
import json; d=json.load(open('gpurun_out/c5_ab.json')); print('prio=$p C5', round(d['value']/1e6,2), 'M verif/s', round(d['ms_per_step'],2), 'ms')"
done; done
