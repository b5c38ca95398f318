#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-bab}
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json && \
timeout -k 10 600 python tools/exp_ab.py > gpurun_out/exp_$TAG.json 2> gpurun_out/exp_$TAG.err && cat gpurun_out/exp_$TAG.json
