#!/bin/bash
# A/B builds of libhsv.so under build-time switches, for tools/ab_probe.py
# (never shipped): tools/build_ab_libs.sh NAME "FLAGS" [NAME "FLAGS" ...]
# -> hsverify/libhsv_NAME.so built from build_ab_NAME/ with FLAGS added to both the
# hipcc and the g++ lines (HSV_EXTRA_HIPFLAGS, HSV_EXTRA_CXXFLAGS)
set -e
cd "$(dirname "$0")/../hotstuff-digital-signature-benchmarking_amd"
while [ $# -ge 2 ]; do
  make -j8 BUILD=build_ab_$1 OUT=hsverify/libhsv_$1.so OUT_TEST= HSV_EXTRA_HIPFLAGS="$2" HSV_EXTRA_CXXFLAGS="$2" > /dev/null
  shift 2
done
ls -la hsverify/libhsv_*.so
