set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s2j_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2j_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/s2j_bench.json 2> gpurun_out/s2j_bench.err; rc=$?; cat gpurun_out/s2j_bench.json; exit $rc
