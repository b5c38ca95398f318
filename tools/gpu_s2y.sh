set -o pipefail
# grid_build in 1024-thread blocks (16 agent fences per 16 K packets instead of 256): packet tests, then the
# device-stream bench under a kernel trace.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_packets.py tests/test_write_packets.py -m gpu > gpurun_out/s2y_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2y_tests.log; [ $rc = 0 ] || exit $rc
HDFS_CRC32C_DSTREAM_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s2y_prof -o run --output-format csv -- python3 tools/device_stream_bench.py > gpurun_out/s2y_dsb.json 2> gpurun_out/s2y_dsb.err; rc=$?; cat gpurun_out/s2y_dsb.json; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 tools/device_stream_bench.py > gpurun_out/s2y_dsb2.json 2> gpurun_out/s2y_dsb2.err; rc=$?; cat gpurun_out/s2y_dsb2.json; exit $rc
