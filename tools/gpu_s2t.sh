set -o pipefail
# Copy-out store cache policies on the device-resident 1 GiB packet run (diagnostic build, one process).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
DSB_DIAG=1 DSB_POLICIES=0,16,17,18 timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/s2t_dsb.json 2> gpurun_out/s2t_dsb.err; rc=$?; cat gpurun_out/s2t_dsb.json; exit $rc
