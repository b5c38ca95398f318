set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_packets.py tests/test_write_packets.py tests/test_gpu_session.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s2h_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2h_tests.log; [ $rc = 0 ] || exit $rc
HDFS_CRC32C_DSTREAM_TRACE=1 timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/s2h_dstream.json 2> gpurun_out/s2h_dstream.err; rc=$?; cat gpurun_out/s2h_dstream.json; grep "pkts=16384" gpurun_out/s2h_dstream.err | tail -3; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/s2h_prof -o run --output-format csv -- python3 tools/device_stream_bench.py > gpurun_out/s2h_prof.log 2>&1; rc=$?; tail -1 gpurun_out/s2h_prof.log; exit $rc
