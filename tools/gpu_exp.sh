#!/bin/bash
# Parity (both tile orders) + A/B experiment.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-exp}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
HDFS_CRC32C_TILE_ORDER=${ALT_ORDER:-3} timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests_${TAG}_o1.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests_${TAG}_o1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/exp_ab.py > gpurun_out/exp_$TAG.json 2> gpurun_out/exp_$TAG.err; rc=$?; cat gpurun_out/exp_$TAG.json; tail -3 gpurun_out/exp_$TAG.err; exit $rc
