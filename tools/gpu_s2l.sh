set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_packets.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s2l_tests.log 2>&1; rc=$?; tail -15 gpurun_out/s2l_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/s2l_dstream.json 2> gpurun_out/s2l_dstream.err; rc=$?; cat gpurun_out/s2l_dstream.json; exit $rc
