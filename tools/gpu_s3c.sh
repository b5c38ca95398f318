set -o pipefail
# Gather kernel with the slot protocol skipped and stores dropped (20) vs stores dropped (2) vs the
# per-tile kernel with stores dropped, one process.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"store_policy": 2}, {"store_policy": 20}, {"runs": 0, "store_policy": 2}]' 4 > gpurun_out/s3c.json 2> gpurun_out/s3c.err; rc=$?; cat gpurun_out/s3c.json; exit $rc
