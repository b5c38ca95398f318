set -o pipefail
# Kernel trace of the device-resident packet-run bench (where the 1 GiB run's time goes).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
HDFS_CRC32C_DSTREAM_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s2w_prof -o run --output-format csv -- python3 tools/device_stream_bench.py > gpurun_out/s2w_dsb.json 2> gpurun_out/s2w_dsb.err; rc=$?; cat gpurun_out/s2w_dsb.json; exit $rc
