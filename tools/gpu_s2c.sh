# schedule-4 compute: parity tests, A/B against schedule 3, bench line
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s2c_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2c_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/exp_knobs.py '[{"runs": 0}, {"runs": 1}]' 4 > gpurun_out/s2c_knobs.json 2> gpurun_out/s2c_knobs.err; rc=$?; cat gpurun_out/s2c_knobs.json; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/s2c_bench.json 2> gpurun_out/s2c_bench.err; rc=$?; cat gpurun_out/s2c_bench.json; exit $rc
