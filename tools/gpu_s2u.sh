set -o pipefail
# Product copy-out stores nt sc1: copy-out parity tests, then the device-stream bench.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_packets.py -m gpu > gpurun_out/s2u_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2u_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/s2u_dsb.json 2> gpurun_out/s2u_dsb.err; rc=$?; cat gpurun_out/s2u_dsb.json; exit $rc
