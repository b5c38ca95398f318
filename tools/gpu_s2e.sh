set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 5 60 python tools/mb_debug.py > gpurun_out/s2e_dbg.out 2>&1; rc=$?; cat gpurun_out/s2e_dbg.out; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_mailbox.py -x -v -p no:cacheprovider --timeout 60 --timeout-method thread > gpurun_out/s2e_mb.log 2>&1; rc=$?; tail -10 gpurun_out/s2e_mb.log; [ $rc = 0 ] || exit $rc
timeout -k 5 120 python tools/small_launch.py > gpurun_out/s2e_small.json 2> gpurun_out/s2e_small.err; rc=$?; cat gpurun_out/s2e_small.json; exit $rc
