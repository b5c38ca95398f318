set -o pipefail
# Compute gather group store: nt (product) vs default (11) vs sc1 (5) vs sc0 (8), one process.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"store_policy": 11}, {"store_policy": 5}, {"store_policy": 8}]' 5 > gpurun_out/s3i.json 2> gpurun_out/s3i.err; rc=$?; cat gpurun_out/s3i.json; exit $rc
