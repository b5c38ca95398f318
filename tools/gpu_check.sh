#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
mkdir -p gpurun_out
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 && tail -3 gpurun_out/gpu_tests.log && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu --no-extra > gpurun_out/bench_prof.json 2>&1 ; echo prof rc=$?
