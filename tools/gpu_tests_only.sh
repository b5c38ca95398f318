set -o pipefail
# GPU test suite + smoke only.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t_${1:-x}.log 2>&1; rc=$?; tail -2 gpurun_out/t_${1:-x}.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
