set -o pipefail
# Gather fast path (32-bit group check, wait loop off the common path) vs the previous gather (binary A/B both ways),
# then the compute-schedule parity tests.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/exp_ab_libs.py build/ab/base/libhadoofus_crc32c.so build/ab/opt/libhadoofus_crc32c.so 4 > gpurun_out/s3f_ab.json 2> gpurun_out/s3f_ab.err; rc=$?; cat gpurun_out/s3f_ab.json; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/exp_ab_libs.py build/ab/opt/libhadoofus_crc32c.so build/ab/base/libhadoofus_crc32c.so 4 > gpurun_out/s3f_ba.json 2> gpurun_out/s3f_ba.err; rc=$?; cat gpurun_out/s3f_ba.json; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_shapes.py -k "compute or schedule or mixed" > gpurun_out/s3f_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s3f_tests.log; exit $rc
