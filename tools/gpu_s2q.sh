set -o pipefail
# Gather compute kernel with its round pipeline restored across the loop
# head (no noreturn trap in the slot wait; LDS-only fences): parity of the
# compute schedules, then compute vs verify in one process, then the bench.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_shapes.py -k "compute or schedule or mixed" > gpurun_out/s2q_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2q_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"store_policy": 2}, {"runs": 0}, {"runs": 1}]' 4 > gpurun_out/s2q_knobs.json 2> gpurun_out/s2q_knobs.err; rc=$?; cat gpurun_out/s2q_knobs.json; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/s2q_bench.json 2> gpurun_out/s2q_bench.err; rc=$?; cat gpurun_out/s2q_bench.json; exit $rc
