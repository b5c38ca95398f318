# device-stream irregular-header tests + compute store-shape experiment
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_packets.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s2b_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2b_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/exp_knobs.py '[{}, {"store_policy": 12}, {"store_policy": 13}, {"store_policy": 2}]' 3 > gpurun_out/s2b_knobs.json 2> gpurun_out/s2b_knobs.err; rc=$?; cat gpurun_out/s2b_knobs.json; exit $rc
