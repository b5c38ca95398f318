set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/s2g_prof -o run --output-format csv -- python3 tools/device_stream_bench.py > gpurun_out/s2g_prof.log 2>&1; rc=$?; tail -3 gpurun_out/s2g_prof.log; exit $rc
