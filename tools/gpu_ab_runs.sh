#!/bin/bash
# Compute-mode store schedules in one process (tools/exp_knobs.py), both
# orders, after the parity tests of the schedules.
#   tools/gpu_ab_runs.sh TAG [RUNS_A] [RUNS_B]   (set_runs values; default 2 vs 4)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-abruns}
A=${2:-2}
B=${3:-4}
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes.py -m gpu -q -x -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "compute_store_schedules or columns" > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/exp_knobs.py "[{\"runs\": $A}, {\"runs\": $B}]" 4 > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err \
  && cat gpurun_out/${TAG}_ab.json && \
timeout -k 10 600 python tools/exp_knobs.py "[{\"runs\": $B}, {\"runs\": $A}]" 4 > gpurun_out/${TAG}_ba.json 2> gpurun_out/${TAG}_ba.err \
  && cat gpurun_out/${TAG}_ba.json
