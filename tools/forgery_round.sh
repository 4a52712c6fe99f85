#!/bin/bash
# GPU check of verdict independence between consecutive calls (tools/qc_forgery_stress.py)
# and repeated runs of the C++ mirror of the reference's crypto tests, with the
# zero-copy staging buffers coarse-grained (HSV_STAGING_COHERENT=0, the round-2 form)
# and fine-grained (default).  Stops on any exit status other than 0 (pass) or 1 (a
# wrong verdict / failed check).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 200 python -u -m pytest tests/test_cpp_mirror.py -x -q --timeout 120 --timeout-method thread > $OUT/forgery_cpp_pytest.txt 2>&1; rc=$?
tail -1 $OUT/forgery_cpp_pytest.txt; ok $rc || exit $rc
for coh in 0 1; do
  HSV_STAGING_COHERENT=$coh timeout -k 10 240 python -u tools/qc_forgery_stress.py --iters ${ITERS:-200} > $OUT/forgery_stress_c$coh.txt 2>&1; rc=$?
  echo "coherent=$coh"; tail -4 $OUT/forgery_stress_c$coh.txt; ok $rc || exit $rc
  fails=0
  for i in $(seq 1 ${RUNS:-8}); do
    HSV_STAGING_COHERENT=$coh timeout -k 10 60 build/crypto_tests > $OUT/forgery_cpp_c${coh}_$i.txt 2>&1; rc=$?
    ok $rc || exit $rc; [ $rc -eq 0 ] || fails=$((fails+1))
  done
  echo "coherent=$coh crypto_tests failed runs: $fails of ${RUNS:-8}"
done
exit 0
