set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhsv.so libhsv_compact.so libhsv_compact2.so; do
  for v in 3 667; do
    HSV_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05h_prof_${lib%.so}_$v -o qc -- python3 tools/qc_kernel_profile.py $v > gpurun_out/r05h_prof_${lib%.so}_$v.log 2>&1
  done
done
timeout -k 10 600 python -u tools/qc_ab.py --rounds 3 --reps 300 libhsv.so libhsv_compact.so libhsv_compact2.so > gpurun_out/r05h_qc_ab.txt 2>&1
python3 tools/wire_samples.py && ./tools/wire_parse_bench > gpurun_out/r05h_wire_parse.txt 2>&1
