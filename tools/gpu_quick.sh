#!/bin/bash
# Quick GPU pass: parity tests + bench (no profiler).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-quick}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json
