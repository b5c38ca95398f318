# schedule 4 + mailbox: full GPU tests, compute A/B, small-call latency, bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mailbox.py -x -v -p no:cacheprovider --timeout 60 --timeout-method thread > gpurun_out/s2d_mb.log 2>&1; rc=$?; tail -12 gpurun_out/s2d_mb.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s2d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2d_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/small_launch.py > gpurun_out/s2d_small.json 2> gpurun_out/s2d_small.err; rc=$?; cat gpurun_out/s2d_small.json; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/exp_knobs.py '[{"runs": 0}, {"runs": 1}]' 4 > gpurun_out/s2d_knobs.json 2> gpurun_out/s2d_knobs.err; rc=$?; cat gpurun_out/s2d_knobs.json; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/s2d_bench.json 2> gpurun_out/s2d_bench.err; rc=$?; cat gpurun_out/s2d_bench.json; exit $rc
