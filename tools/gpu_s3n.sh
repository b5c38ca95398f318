set -o pipefail
# Dealing group size: 8 (product) vs 16 vs 32 tiles per group, one process.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"group_shift": 4}, {"group_shift": 5}, {}]' 5 > gpurun_out/s3n.json 2> gpurun_out/s3n.err; rc=$?; cat gpurun_out/s3n.json; exit $rc
