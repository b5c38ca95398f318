set -o pipefail
# Device-stream bench with the D2D copy ceiling for verify + copy-out.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/s3l_dsb.json 2> gpurun_out/s3l_dsb.err; rc=$?; cat gpurun_out/s3l_dsb.json; exit $rc
