#!/bin/bash
# Round-4 device-stream evidence call (GPU box): spec / packet / ABI tests,
# device-stream bench (plain and traced), synchronous-call latencies, and a
# rocprofv3 kernel trace of the device-stream bench.  Usage:
#   gpurun --timeout 1200 -- 'bash tools/gpu_r4_dstream.sh TAG'
set -o pipefail
T=${1:-r4}
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_spec_verify.py tests/test_packets.py tests/test_device_checks.py tests/test_abi.py \
  tests/test_gpu_attribution.py tests/test_hostpin.py > $O/${T}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u tools/device_stream_bench.py > $O/${T}_dstream.json 2> $O/${T}_dstream.err || exit $?
HDFS_CRC32C_DSTREAM_TRACE=1 timeout -k 10 300 python -u tools/device_stream_bench.py \
  > $O/${T}_dstream_trace.json 2> $O/${T}_dstream_trace.err || exit $?
timeout -k 10 200 python -u tools/small_launch.py > $O/${T}_small.json 2> $O/${T}_small.err || exit $?
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/${T}_prof -o $T -- \
  python3 $R/tools/device_stream_bench.py > $R/$O/${T}_prof.log 2>&1 || exit $?
echo "done tests_rc=$rc"
