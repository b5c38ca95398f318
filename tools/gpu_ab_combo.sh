#!/bin/bash
# Parity of the new build, then A/Bs against a base build on one box:
# device-resident packet runs (tools/device_stream_bench.py) and the tiled
# plans (tools/exp_ab_libs.py, both orders).   tools/gpu_ab_combo.sh TAG BASE_LIB
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-combo}
BASE=${2:-build/ab/base/libhadoofus_crc32c.so}
NEW=hadoofus_amd/lib/libhadoofus_crc32c.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_packets.py tests/test_hostpin.py tests/test_device_checks.py -m gpu -q -x \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
[ -n "$SKIP_AB" ] || timeout -k 10 600 python tools/exp_ab_libs.py $BASE $NEW 4 > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err || exit $?
cat gpurun_out/${TAG}_ab.json
[ -n "$SKIP_AB" ] || timeout -k 10 600 python tools/exp_ab_libs.py $NEW $BASE 4 > gpurun_out/${TAG}_ba.json 2> gpurun_out/${TAG}_ba.err || exit $?
cat gpurun_out/${TAG}_ba.json
for i in 1 2; do
  DSB_LIB=$BASE timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/${TAG}_dsbase$i.json 2>> gpurun_out/${TAG}_ds.err || exit $?
  timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/${TAG}_dsnew$i.json 2>> gpurun_out/${TAG}_ds.err || exit $?
done
cat gpurun_out/${TAG}_ds*.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 tools/device_stream_bench.py > gpurun_out/${TAG}_prof.log 2>&1
