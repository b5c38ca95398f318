#!/bin/bash
# GPU tests of a selection, without stopping at the first failure:
#   tools/gpu_tests_sel.sh TAG test-files...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
shift
timeout -k 10 900 python -u -m pytest "$@" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -5 gpurun_out/${TAG}_tests.log; exit $rc
