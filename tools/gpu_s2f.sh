set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mailbox.py -x -q -p no:cacheprovider --timeout 60 --timeout-method thread > gpurun_out/s2f_mb.log 2>&1; rc=$?; tail -2 gpurun_out/s2f_mb.log; [ $rc = 0 ] || exit $rc
timeout -k 5 120 python tools/small_launch.py > gpurun_out/s2f_small.json 2> gpurun_out/s2f_small.err; rc=$?; cat gpurun_out/s2f_small.json; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/exp_knobs.py '[{"runs": 0}, {"runs": 1}]' 4 > gpurun_out/s2f_knobs.json 2> gpurun_out/s2f_knobs.err; rc=$?; cat gpurun_out/s2f_knobs.json; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/s2f_bench.json 2> gpurun_out/s2f_bench.err; rc=$?; cat gpurun_out/s2f_bench.json; exit $rc
