set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s2a_tests.log 2>&1; rc=$?; tail -5 gpurun_out/s2a_tests.log; [ $rc = 0 ] || exit $rc
HDFS_CRC32C_DSTREAM_TRACE=1 timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/s2a_dstream.json 2> gpurun_out/s2a_dstream.err; rc=$?; cat gpurun_out/s2a_dstream.json; grep "pkts=16384" gpurun_out/s2a_dstream.err | tail -3; exit $rc
