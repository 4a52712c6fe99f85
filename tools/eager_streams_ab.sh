#!/bin/bash
# Host pipeline streams vs the application's C4 streams: the
# C4 line and the 2^20 host call under each setting of the switches
# HSV_EAGER_STREAMS (create the pipeline streams in hsv_init; measured in
# r03zm, since removed) and HSV_PIPE_PRIO (greatest stream priority, now the
# default), one bench.py process each.
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
for r in 1 2; do for cfg in "0 0" "1 0" "0 1" "1 1"; do
set -- $cfg
HSV_EAGER_STREAMS=$1 HSV_PIPE_PRIO=$2 timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --qc-reps 20 > gpurun_out/eager_ab.json 2>/dev/null || exit 1
python -c "
import json; d=json.load(open('gpurun_out/eager_ab.json')); h=d['host_api']
print('eager=$1 prio=$2 C4_ms_per_step', round(d['ms_per_step'],3), 'isolated', round(d['roofline']['isolated_launch_ms'],3), 'host_api_ms', round(h['ms'],3), 'qc_c3_p50', round(d['qc_latency']['n1000_votes667']['p50_ms'],4))"
done; done
