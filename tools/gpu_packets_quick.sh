#!/bin/bash
# Device-stream parity (packet verifier, device checks) + the device-stream
# bench, one call.   tools/gpu_packets_quick.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pq}
timeout -k 10 600 python -u -m pytest tests/test_packets.py tests/test_device_checks.py -m gpu -q -x -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/${TAG}_dstream.json 2> gpurun_out/${TAG}_dstream.err \
  && cat gpurun_out/${TAG}_dstream.json
timeout -k 10 300 python tools/frame_phases.py > gpurun_out/${TAG}_phases.json 2> gpurun_out/${TAG}_phases.err \
  && cat gpurun_out/${TAG}_phases.json
