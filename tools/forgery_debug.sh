#!/bin/bash
# Runs the C++ mirror of the reference's crypto tests repeatedly (RUNS, default 16) under
# four builds/settings: the round-2 neutral-point check (a library built with
# -DHSV_NEUTRAL_NO_Z_CHECK in abdir_oldcheck/) or the fail-closed one, with launch
# workspaces from the default HIP memory pool (HSV_WS_POOL=default) or the library's own
# pool.  Prints failing runs' stderr and the failure count per mode.  Round-2 record
# (DESIGN.md section 6.2): the HSV_WS_POOL switch was a measurement-build knob, removed
# from the source in round 5, so the "default" rows need a library built from git history.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
AB=$(pwd)/hotstuff-digital-signature-benchmarking_amd/abdir_oldcheck
timeout -k 10 200 python -u -m pytest tests/test_cpp_mirror.py -x -q --timeout 120 --timeout-method thread > $OUT/fdbg_pytest.txt 2>&1; rc=$?
tail -1 $OUT/fdbg_pytest.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for check in old new; do
  for pool in default own; do
    fails=0
    for i in $(seq 1 ${RUNS:-16}); do
      if [ $check = old ]; then LP=$AB; else LP=; fi
      LD_LIBRARY_PATH=$LP HSV_WS_POOL=$pool timeout -k 10 60 build/crypto_tests > $OUT/fdbg_${check}_${pool}_$i.txt 2>&1; rc=$?
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
      if [ $rc -eq 1 ]; then fails=$((fails+1)); [ $fails -le 1 ] && { echo "check=$check pool=$pool run $i:"; cat $OUT/fdbg_${check}_${pool}_$i.txt; }; fi
    done
    echo "check=$check pool=$pool failed runs: $fails of ${RUNS:-16}"
  done
done
