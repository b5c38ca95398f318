#!/bin/bash
# GPU parity suite + small-launch latencies.  Stops on the first failure.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-quick}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/small_launch.py > gpurun_out/${TAG}_small.json 2> gpurun_out/${TAG}_small.err
rc=$?; cat gpurun_out/${TAG}_small.json; tail -3 gpurun_out/${TAG}_small.err; exit $rc
