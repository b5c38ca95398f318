#!/bin/bash
# Packet-stream verifier: end-to-end host-resident rate + kernel breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/packets_bench.py > gpurun_out/packets_bench.json 2> gpurun_out/packets_bench.err && cat gpurun_out/packets_bench.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pk -o run --output-format csv -- python3 tools/packets_bench.py > gpurun_out/packets_prof.log 2>&1; echo prof rc=$?
find gpurun_out/prof_pk -name "*kernel_stats.csv" | head -1 | xargs -r cat | cut -c1-200
