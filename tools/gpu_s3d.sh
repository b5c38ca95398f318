set -o pipefail
# Short device runs with speculative layout loads: packet tests, then the device-stream bench alternating
# the previous build (build/ab/base) and this one on the same box.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_packets.py -m gpu > gpurun_out/s3d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s3d_tests.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  DSB_LIB=build/ab/base/libhadoofus_crc32c.so timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/s3d_base$i.json 2> gpurun_out/s3d_base$i.err || exit 1
  timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/s3d_new$i.json 2> gpurun_out/s3d_new$i.err || exit 1
  cat gpurun_out/s3d_base$i.json gpurun_out/s3d_new$i.json
done
