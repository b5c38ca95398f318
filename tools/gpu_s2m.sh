set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s2m_prof -o run --output-format csv -- python3 tools/device_stream_bench.py > gpurun_out/s2m_prof.log 2>&1; rc=$?; tail -1 gpurun_out/s2m_prof.log; exit $rc
