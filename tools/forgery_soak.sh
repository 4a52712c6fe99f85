#!/bin/bash
# Soak of the round-2 forged-vote fix: RUNS fresh processes of the C++ port of the
# reference's crypto tests (each overlaps the automatic committee cache's first build)
# and the Python alternating honest/forged QC stress.  Stops on any exit status other
# than 0 (pass) or 1 (a failed check).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 200 python -u -m pytest tests/test_cpp_mirror.py -x -q --timeout 120 --timeout-method thread > $OUT/soak_pytest.txt 2>&1; rc=$?
tail -1 $OUT/soak_pytest.txt; ok $rc || exit $rc
fails=0
for i in $(seq 1 ${RUNS:-40}); do
  timeout -k 10 60 build/crypto_tests > $OUT/soak_cpp_$i.txt 2>&1; rc=$?
  ok $rc || exit $rc; [ $rc -eq 0 ] || fails=$((fails+1))
done
echo "crypto_tests failed runs: $fails of ${RUNS:-40}"
timeout -k 10 300 python -u tools/qc_forgery_stress.py --iters 300 > $OUT/soak_stress.txt 2>&1; rc=$?
tail -5 $OUT/soak_stress.txt; ok $rc || exit $rc
[ $fails -eq 0 ] && [ $rc -eq 0 ]
