#!/bin/bash
# Builds timing-stub variants of libhsv.so for tools/phase_probe.py (never shipped):
#   build_stub_<name>/libhsv.so with -DHSV_TIMING_STUB_<NAME>
set -e
cd "$(dirname "$0")/../hotstuff-digital-signature-benchmarking_amd"
for s in LATTICE SQRT SHA STRAUS TABLES COMB; do
  n=$(echo $s | tr A-Z a-z)
  make -j8 BUILD=build_stub_$n OUT=build_stub_$n/libhsv.so HSV_EXTRA_HIPFLAGS="-DHSV_TIMING_STUB_$s" > /dev/null
done
ls -la build_stub_*/libhsv.so
