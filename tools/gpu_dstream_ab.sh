#!/bin/bash
# Device-resident packet runs, two builds on one box (base, new, base, new):
# tools/device_stream_bench.py with DSB_LIB, then a rocprofv3 kernel trace
# of the new build.   tools/gpu_dstream_ab.sh TAG BASE_LIB
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-dsab}
BASE=${2:-build/ab/base/libhadoofus_crc32c.so}
timeout -k 10 600 python -u -m pytest tests/test_packets.py -m gpu -q -x -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  DSB_LIB=$BASE timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/${TAG}_base$i.json 2>> gpurun_out/${TAG}.err || exit $?
  timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/${TAG}_new$i.json 2>> gpurun_out/${TAG}.err || exit $?
done
cat gpurun_out/${TAG}_base*.json gpurun_out/${TAG}_new*.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 tools/device_stream_bench.py > gpurun_out/${TAG}_prof.log 2>&1
