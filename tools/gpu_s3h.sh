set -o pipefail
# Verify bitmap stores sc1 (24), sc0 sc1 (25), one process.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"store_policy": 24}, {"store_policy": 25}, {}]' 5 > gpurun_out/s3h.json 2> gpurun_out/s3h.err; rc=$?; cat gpurun_out/s3h.json; exit $rc
