set -o pipefail
# Gather compute parity incl. CRC32 and little-endian tables.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "compute_runs_schedule" > gpurun_out/s3m_tests.log 2>&1; rc=$?; tail -9 gpurun_out/s3m_tests.log; exit $rc
