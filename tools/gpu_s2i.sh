set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shapes.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "store_schedules" > gpurun_out/s2i_tests.log 2>&1; rc=$?; tail -6 gpurun_out/s2i_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/exp_knobs.py '[{"runs": 0}, {"runs": 1}, {"runs": 2}]' 4 > gpurun_out/s2i_knobs.json 2> gpurun_out/s2i_knobs.err; rc=$?; cat gpurun_out/s2i_knobs.json; exit $rc
