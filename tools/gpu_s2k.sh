set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mailbox.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 60 --timeout-method thread > gpurun_out/s2k_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s2k_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 5 120 python tools/small_launch.py > gpurun_out/s2k_small.json 2> gpurun_out/s2k_small.err; rc=$?; cat gpurun_out/s2k_small.json; exit $rc
