set -o pipefail
# grid_build with its independent loads hoisted above the reductions: packet tests, then the device-stream
# bench under a kernel trace (this build) and the previous build on the same box.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_packets.py -m gpu > gpurun_out/s3k_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s3k_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s3k_new -o run --output-format csv -- python3 tools/device_stream_bench.py > gpurun_out/s3k_new.json 2> gpurun_out/s3k_new.err || exit 1
DSB_LIB=build/ab/base/libhadoofus_crc32c.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s3k_base -o run --output-format csv -- python3 tools/device_stream_bench.py > gpurun_out/s3k_base.json 2> gpurun_out/s3k_base.err || exit 1
cat gpurun_out/s3k_new.json gpurun_out/s3k_base.json
