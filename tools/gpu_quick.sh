#!/bin/bash
# Quick GPU pass: parity tests (one process) + the bench line (no profiler).
#   tools/gpu_quick.sh TAG [pytest selection...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-quick}
shift
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
  && cat gpurun_out/${TAG}_bench.json
